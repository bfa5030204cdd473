"""Generate the golden fixtures in tests/golden/ by running the REFERENCE itself.

Runs only in the build container, where /root/reference exists.  It imports open_clip's
`model` module and Patch-Aligned-Contrastive-Learning/model/pacl.py straight from the
read-only reference tree with two in-process stubs:
  * torchvision.ops.misc.FrozenBatchNorm2d (only used by an off-path helper),
  * ftfy.fix_text = identity (tokenizer import; no text is tokenised here).
Weights and inputs come from clipembed.weights (deterministic counter-based generator), are
loaded with load_state_dict, and only OUTPUTS (plus SHA-256 digests of the inputs, which pin
the generator) are written.  No reference source is copied.

    python tests/golden/make_golden.py            # all fixtures
"""
from __future__ import annotations

import hashlib
import importlib
import importlib.util
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "clip-embeds_amd"))
REF = "/root/reference"
OC_ROOT = os.path.join(REF, "open_clip/src/open_clip")
PACL_PY = os.path.join(REF, "Patch-Aligned-Contrastive-Learning/model/pacl.py")

from clipembed.config import get_model_config  # noqa: E402
from clipembed import weights as W  # noqa: E402


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def import_reference():
    import transformers  # noqa: F401  (must precede the torchvision stub)
    import torch
    tv, tvo, tvm = (types.ModuleType(n) for n in ("torchvision", "torchvision.ops", "torchvision.ops.misc"))

    class FrozenBatchNorm2d(torch.nn.Module):
        pass

    tvm.FrozenBatchNorm2d = FrozenBatchNorm2d
    tv.ops, tvo.misc = tvo, tvm
    sys.modules.update({"torchvision": tv, "torchvision.ops": tvo, "torchvision.ops.misc": tvm})
    ft = types.ModuleType("ftfy")
    ft.fix_text = lambda s: s
    sys.modules["ftfy"] = ft
    pkg = types.ModuleType("open_clip")
    pkg.__path__ = [OC_ROOT]
    sys.modules["open_clip"] = pkg
    model_mod = importlib.import_module("open_clip.model")
    loss_mod = importlib.import_module("open_clip.loss")
    # pacl.py does `import open_clip.src.open_clip as oc`
    src = types.ModuleType("open_clip.src")
    src.open_clip = pkg
    pkg.src = src
    sys.modules["open_clip.src"] = src
    sys.modules["open_clip.src.open_clip"] = pkg
    spec = importlib.util.spec_from_file_location("pacl_reference", PACL_PY)
    pacl_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(pacl_mod)
    return model_mod, loss_mod, pacl_mod


def build_clip(model_mod, cfg, seed=7):
    import torch
    m = model_mod.CLIP(**cfg.open_clip_dict())
    sd = W.synthetic_state_dict(cfg, seed)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    m.eval()
    return m, sd


def build_pacl(pacl_mod, clip_model, cls, heads_sd):
    """open_clip_pacl('ViT-L-14-336') without its network fetch: the same heads (pacl.py:70-79)
    around an already-built CLIP."""
    import torch
    from torch import nn
    obj = cls.__new__(cls)
    nn.Module.__init__(obj)
    obj.clip_model = clip_model
    obj.visual_projection = nn.Sequential(nn.LayerNorm(1024), nn.Dropout(0.1), pacl_mod.Patch_Projection(1024, 768))
    obj.text_projection = nn.Sequential(nn.LayerNorm(768), nn.Dropout(0.1), nn.Linear(768, 768))
    for p in obj.clip_model.parameters():
        p.requires_grad = False
    obj.clip_model.visual.output_tokens = True
    missing = obj.load_state_dict({k: torch.from_numpy(v) for k, v in heads_sd.items()}, strict=False)
    assert not missing.unexpected_keys, missing.unexpected_keys
    assert all(k.startswith("clip_model.") for k in missing.missing_keys)
    obj.eval()
    return obj


def token_rows(x, rows):
    return np.ascontiguousarray(x[:, rows, :])


TOKEN_ROWS_V = [0, 1, 23, 24, 287, 300, 551, 575]
TOKEN_ROWS_T = [0, 1, 5, 20, 40, 76]


def gen_clip(model_mod, cfg, n_img, n_txt, tag, out):
    import torch
    m, sd = build_clip(model_mod, cfg)
    imgs = W.synthetic_images(n_img, seed=1000)
    caps = W.synthetic_captions(n_txt, seed=2000)
    caps[-1] = W.synthetic_captions(1, seed=2999, min_len=75, max_len=75)[0]  # longest caption (EOT at 76)
    with torch.no_grad():
        m.visual.output_tokens = True
        m.output_text_tokens = True
        pi, ti = m.encode_image(torch.from_numpy(imgs))
        pt, tt = m.encode_text(torch.from_numpy(caps))
        m.visual.output_tokens = False
        m.output_text_tokens = False
        il, tl = m.get_logits(torch.from_numpy(imgs), torch.from_numpy(caps))
        fi, ft, ls = m(torch.from_numpy(imgs), torch.from_numpy(caps))
    out[f"{tag}"] = dict(
        captions=caps,
        images_sha=sha(imgs),
        weights_probe=np.stack([sd["visual.conv1.weight"].ravel()[:8], sd["token_embedding.weight"].ravel()[:8]]),
        image_pooled=pi.numpy(), text_pooled=pt.numpy(),
        image_tokens_rows=token_rows(ti.numpy(), TOKEN_ROWS_V), image_tokens_sum=ti.numpy().sum((1, 2)),
        text_tokens_rows=token_rows(tt.numpy(), TOKEN_ROWS_T), text_tokens_sum=tt.numpy().sum((1, 2)),
        image_logits=il.numpy(), text_logits=tl.numpy(),
        image_features=fi.numpy(), text_features=ft.numpy(), logit_scale_exp=np.float32(ls.item()),
    )
    return m, sd, imgs, caps


def gen_pacl(pacl_mod, clip_model, cfg, out):
    import torch
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    imgs = W.synthetic_images(2, seed=1100)
    caps = W.synthetic_captions(2, seed=2100)
    res = {"captions": caps, "images_sha": sha(imgs)}
    with torch.no_grad():
        for tag, cls in (("pacl", pacl_mod.open_clip_pacl), ("pacl_rope", pacl_mod.open_clip_pacl_rope),
                         ("pacl_rope_after", pacl_mod.open_clip_pacl_rope_after)):
            mod = build_pacl(pacl_mod, clip_model, cls, heads)
            a, b = mod(torch.from_numpy(imgs), torch.from_numpy(caps))        # diag pairing
            res[f"{tag}_img"], res[f"{tag}_txt"] = a.numpy(), b.numpy()
            a1, b1 = mod(torch.from_numpy(imgs[:1]), torch.from_numpy(caps))  # 1 image x 2 texts (Q6)
            res[f"{tag}_bcast_img"], res[f"{tag}_bcast_txt"] = a1.numpy(), b1.numpy()
        mod = build_pacl(pacl_mod, clip_model, pacl_mod.open_clip_pacl, heads)
        vp = mod.forward_visual(torch.from_numpy(imgs))
        tp = mod.forward_text(torch.from_numpy(caps))
        res["visual_proj_rows"] = token_rows(vp.numpy(), TOKEN_ROWS_V[1:])
        res["visual_proj_sum"] = vp.numpy().sum((1, 2))
        res["text_proj"] = tp.numpy()
        # sigmoid(10 cos) weighting without RoPE: reference patch_alignment + the forward's pooling
        act = mod.patch_alignment(vp, tp)
        pooled = torch.sum(vp * act.unsqueeze(-1), dim=1)
        res["pacl_sigmoid_img"] = torch.nn.functional.normalize(pooled, dim=-1).numpy()
    out["pacl"] = res
    return heads


def gen_rope_sparc_loss(pacl_mod, loss_mod, out):
    import torch
    x = W.uniform("rope-input", 2 * 576 * 128).reshape(2, 576, 128)
    out["rope"] = dict(y=pacl_mod.apply_rope(torch.from_numpy(x)).numpy())  # x regenerated by the tests
    # SPARC forward math (pacl.py:460-476) on synthetic projected embeddings
    v = W.uniform("sparc-v", 2 * 576 * 64).reshape(2, 576, 64)
    l = W.uniform("sparc-l", 2 * 77 * 64).reshape(2, 77, 64)
    res = {}  # v, l regenerated by the tests from the same generator keys
    for name, sigma in (("s576", 1.0 / 576), ("s625", 1.0 / 625)):
        obj = pacl_mod.sparc.__new__(pacl_mod.sparc)
        torch.nn.Module.__init__(obj)
        obj.sigma = sigma
        obj.forward_visual = lambda images: torch.from_numpy(v)
        obj.forward_text = lambda caps: (torch.from_numpy(l), torch.ones(2, 77))
        vp, lt, g, mask = obj.forward(None, None)
        res[f"{name}_grouped"], res[f"{name}_l_norm"] = g.numpy(), lt.numpy()
        res[f"{name}_score_local"] = obj.scoring(torch.zeros(2, 1), torch.zeros(2, 1), local=True).numpy()
        res[f"{name}_score_global"] = obj.scoring(torch.zeros(2, 1), torch.zeros(2, 1), local=False).numpy()
        sl = pacl_mod.SparcLoss(0.1)
        res[f"{name}_sparc_loss"] = np.float32(sl(vp, lt, g, torch.from_numpy(
            (np.arange(77)[None, :] <= np.array([[20], [76]])).astype(np.float32))).item())
    out["sparc"] = res
    # PACL ClipLoss (pacl.py:489-514)
    a = W.uniform("loss-a", 8 * 768).reshape(8, 768)
    b = W.uniform("loss-b", 8 * 768).reshape(8, 768)
    an = torch.nn.functional.normalize(torch.from_numpy(a), dim=-1)
    bn = torch.nn.functional.normalize(torch.from_numpy(b), dim=-1)
    out["loss"] = dict(a=a, b=b, pacl_clip_loss=np.float32(pacl_mod.ClipLoss(0.1)(an, bn).item()),
                       openclip_single=np.float32(loss_mod.ClipLoss()(an, bn, torch.tensor(14.2857)).item()))


def _negclip_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, loss_mod, _ = import_reference()
    B, D, K = 4, 768, [2, 3][rank]
    img = torch.nn.functional.normalize(torch.from_numpy(W.uniform(f"neg-img-{rank}", B * D).reshape(B, D)), dim=-1)
    txt = torch.nn.functional.normalize(torch.from_numpy(W.uniform(f"neg-txt-{rank}", (B + K) * D).reshape(B + K, D)), dim=-1)
    res = {}
    for hard in (True, False):
        t = txt if hard else txt[:B]
        fn = loss_mod.ClipLoss(local_loss=True, gather_with_grad=True, rank=rank, world_size=world, usehardtext=hard)
        res["hard" if hard else "plain_local"] = float(fn(img, t, torch.tensor(14.2857)))
    fn = loss_mod.ClipLoss(local_loss=False, gather_with_grad=False, rank=rank, world_size=world)
    res["plain_global"] = float(fn(img, txt[:B], torch.tensor(14.2857)))
    q.put((rank, res))
    dist.destroy_process_group()


def gen_negclip(out):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29611
    procs = [ctx.Process(target=_negclip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join()
    out["negclip"] = {f"{k}_r{r}": np.float32(v) for r in range(2) for k, v in got[r].items()}


def save(out):
    for name, d in out.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **{k: np.asarray(v) for k, v in d.items()})
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


def main():
    import torch
    torch.manual_seed(0)
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    model_mod, loss_mod, pacl_mod = import_reference()
    out = {}
    base = get_model_config("ViT-L-14-336")
    m_small, _, _, _ = gen_clip(model_mod, base.with_depth(2, 2), 2, 3, "clip_v2t2", out)
    gen_clip(model_mod, get_model_config("ViT-L-14-336-quickgelu").with_depth(1, 1), 2, 2, "clip_quickgelu_v1t1", out)
    gen_clip(model_mod, base, 2, 2, "clip_full", out)
    gen_pacl(pacl_mod, m_small, base.with_depth(2, 2), out)
    gen_rope_sparc_loss(pacl_mod, loss_mod, out)
    gen_negclip(out)
    full, _ = build_clip(model_mod, base.with_depth(1, 1))
    pacl = build_pacl(pacl_mod, full, pacl_mod.open_clip_pacl, W.synthetic_pacl_heads(base.with_pacl(768)))
    meta = {"generator": "tests/golden/make_golden.py", "torch": torch.__version__, "weights_seed": 7,
            "pacl_heads_seed": 11, "reference": "lst627/CLIP-Embeds @ 2025-06-14",
            # state-dict key layout of the reference modules (1-block towers), pins the loader's names
            "clip_state_dict_keys": {k: list(v.shape) for k, v in full.state_dict().items()},
            "pacl_state_dict_keys": {k: list(v.shape) for k, v in pacl.state_dict().items()
                                     if not k.startswith("clip_model.")}}
    out["meta"] = {"json": np.array(json.dumps(meta))}
    save(out)


def main_pacl_full():
    """pacl_full.npz: the three open_clip_pacl variants + the sigmoid(10 cos) weighting around the
    FULL-depth (24 + 12 blocks) reference CLIP ViT-L/14-336, diag pairing of 2 images x 2 captions
    and the 1 image x 2 captions broadcast (Q6); plus the token / patch-head rows."""
    import torch
    torch.manual_seed(0)
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    model_mod, _, pacl_mod = import_reference()
    base = get_model_config("ViT-L-14-336")
    clip_model, _ = build_clip(model_mod, base)
    out = {}
    gen_pacl(pacl_mod, clip_model, base, out)
    res = out["pacl"]
    res["images_seed"] = np.int64(1100)
    res["captions_seed"] = np.int64(2100)
    save({"pacl_full": res})


if __name__ == "__main__":
    main_pacl_full() if sys.argv[1:] == ["pacl_full"] else main()
