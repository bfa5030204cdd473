"""Golden outputs of the reference SPARC model at real dimensions (D = 768, T = 77, P = 576) —
build container only.

Runs Patch-Aligned-Contrastive-Learning/model/pacl.py's `sparc` and `sparc_rope` (pacl.py:380-484)
around the reference open_clip CLIP ViT-L/14-336 with 1-block towers (the SPARC math after the
towers is depth-independent) and the deterministic synthetic weights / PACL-shaped heads, built
without the network fetch in the constructor (the same head modules, pacl.py:397-406).  Writes
outputs only: selected token / patch rows of forward(), both scoring() modes and SparcLoss.

    python tests/golden/make_golden_sparc.py        ->  tests/golden/sparc_full.npz
    python tests/golden/make_golden_sparc.py fulldepth   ->  tests/golden/sparc_fulldepth.npz (24 + 12 blocks)
    python tests/golden/make_golden_sparc.py dist   ->  tests/golden/sparc_dist.npz
    python tests/golden/make_golden_sparc.py train  ->  tests/golden/sparc_train.npz
    python tests/golden/make_golden_sparc.py train_pacl  ->  tests/golden/pacl_train.npz

`dist`: the reference SparcLoss(0.1) (train_sparc.py:105) and PACL ClipLoss(0.1) (train_pacl.py:106)
on the CONCATENATION of two ranks' shards (tests/golden/dist_inputs.py), i.e. the value
train_sparc.py / train_pacl.py compute after nn.DataParallel gathers the replicas' outputs to one
device (train_sparc.py:93, train_pacl.py:95); plus each shard's own single-process loss, which the
sharded path must NOT return.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, os.path.join(REPO, "clip-embeds_amd"), REPO]

import make_golden as MG  # noqa: E402

ROWS_T = [0, 1, 5, 9, 20, 40, 76]
ROWS_P = [0, 1, 23, 24, 287, 300, 550, 575]


def build_sparc(pacl_mod, clip_model, cls, heads_sd, sigma):
    import torch
    from torch import nn
    obj = cls.__new__(cls)
    nn.Module.__init__(obj)
    obj.sigma = sigma
    obj.clip_model = clip_model
    obj.visual_projection = nn.Sequential(nn.LayerNorm(1024), nn.Dropout(0.1), pacl_mod.Patch_Projection(1024, 768))
    obj.text_projection = nn.Sequential(nn.LayerNorm(768), nn.Dropout(0.1), nn.Linear(768, 768))
    for p in obj.clip_model.parameters():
        p.requires_grad = False
    obj.clip_model.visual.output_tokens = True
    obj.clip_model.output_text_tokens = True
    missing = obj.load_state_dict({k: torch.from_numpy(v) for k, v in heads_sd.items()}, strict=False)
    assert not missing.unexpected_keys, missing.unexpected_keys
    obj.eval()
    return obj


def main(full_depth=False):
    import torch
    from clipembed import weights as W
    from clipembed.config import get_model_config
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    model_mod, _, pacl_mod = MG.import_reference()
    cfg = get_model_config("ViT-L-14-336")
    if not full_depth:
        cfg = cfg.with_depth(1, 1)
    clip, _ = MG.build_clip(model_mod, cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1300))
    caps = W.synthetic_captions(2, seed=2300)
    caps[1] = W.synthetic_captions(1, seed=2301, min_len=7, max_len=7)[0]      # EOT at 8: short caption
    caps = torch.from_numpy(caps)
    out = {"captions": caps.numpy(), "images_sha": np.array(MG.sha(imgs.numpy()))}
    with torch.no_grad():
        for tag, cls in (("sparc", pacl_mod.sparc), ("sparc_rope", pacl_mod.sparc_rope)):
            mod = build_sparc(pacl_mod, clip, cls, heads, 1.0 / 576)
            v, l, g, mask = mod.forward(imgs, caps)
            out[f"{tag}_v_rows"] = np.ascontiguousarray(v.numpy()[:, ROWS_P])
            out[f"{tag}_v_sum"] = v.numpy().sum((1, 2))
            out[f"{tag}_l_rows"] = np.ascontiguousarray(l.numpy()[:, ROWS_T])
            out[f"{tag}_g_rows"] = np.ascontiguousarray(g.numpy()[:, ROWS_T])
            out[f"{tag}_g_sum"] = g.numpy().sum((1, 2))
            out[f"{tag}_mask"] = mask.numpy()
            out[f"{tag}_score_local"] = mod.scoring(imgs, caps, local=True).numpy()
            out[f"{tag}_score_global"] = mod.scoring(imgs, caps, local=False).numpy()
            out[f"{tag}_score_bcast"] = mod.scoring(imgs[:1], caps, local=True).numpy()   # 1 image x 2 captions
            out[f"{tag}_loss"] = np.float32(pacl_mod.SparcLoss(0.07)(v, l, g, mask).item())
    path = os.path.join(HERE, "sparc_fulldepth.npz" if full_depth else "sparc_full.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


def main_dist():
    import torch
    from dist_inputs import pacl_shard, sparc_shard
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    _, _, pacl_mod = MG.import_reference()
    sh = [sparc_shard(r) for r in range(2)]
    ph = [pacl_shard(r) for r in range(2)]
    cat = lambda k, xs: torch.from_numpy(np.concatenate([x[k] for x in xs]))   # noqa: E731
    out = {}
    with torch.no_grad():
        sl = pacl_mod.SparcLoss(0.1)
        out["sparc_global"] = np.float32(sl(cat(0, sh), cat(1, sh), cat(2, sh), cat(3, sh)).item())
        cl = pacl_mod.ClipLoss(0.1)
        out["pacl_global"] = np.float32(cl(cat(0, ph), cat(1, ph)).item())
        for r in range(2):
            t = [torch.from_numpy(x) for x in sh[r]]
            out[f"sparc_shard_r{r}"] = np.float32(sl(*t).item())
            out[f"pacl_shard_r{r}"] = np.float32(cl(*[torch.from_numpy(x) for x in ph[r]]).item())
    path = os.path.join(HERE, "sparc_dist.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, out)


# the SPARC head tensors train_sparc.py trains (its Adam sees every parameter, the frozen tower's have
# no gradient); Patch_Projection's text_projection alias is the same module as linear_projection
TRAIN_TENSORS = ["visual_projection.0.weight", "visual_projection.0.bias",
                 "visual_projection.2.linear_projection.0.weight", "visual_projection.2.linear_projection.0.bias",
                 "visual_projection.2.non_linear_projection.0.weight", "visual_projection.2.non_linear_projection.0.bias",
                 "visual_projection.2.non_linear_projection.2.weight", "visual_projection.2.non_linear_projection.2.bias",
                 "text_projection.0.weight", "text_projection.0.bias", "text_projection.2.weight", "text_projection.2.bias"]
GRAD_ROWS = [0, 1, 383, 767]


def main_train():
    """One train_sparc.py step (train_sparc.py:29-37,91,106): sparc_rope(sigma = 1/576) forward, SparcLoss(0.1),
    loss.backward(), torch.optim.Adam(lr = 1e-4).step(), on 3 images + 3 captions with 1-block towers (the
    head math is depth-independent).  Dropout off (the module in eval mode: train_sparc.py's model.train()
    draws torch RNG masks, which no other generator reproduces; the engine's dropout is tested against
    the oracle with its own masks).  Writes the loss, every head gradient (1-d tensors whole, 2-d tensors'
    norms and rows GRAD_ROWS) and the first Adam update of the same entries."""
    import torch
    from clipembed import weights as W
    from clipembed.config import get_model_config
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    model_mod, _, pacl_mod = MG.import_reference()
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    clip, _ = MG.build_clip(model_mod, cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    imgs = torch.from_numpy(W.synthetic_images(3, seed=1400))
    caps = W.synthetic_captions(3, seed=2400)
    caps[1] = W.synthetic_captions(1, seed=2401, min_len=7, max_len=7)[0]
    caps[2] = W.synthetic_captions(1, seed=2402, min_len=60, max_len=60)[0]
    caps = torch.from_numpy(caps)
    mod = build_sparc(pacl_mod, clip, pacl_mod.sparc_rope, heads, 1.0 / 576)
    params = dict(mod.named_parameters())
    opt = torch.optim.Adam(mod.parameters(), lr=1e-4)
    opt.zero_grad()
    v, l, g, mask = mod(imgs, caps)
    loss = pacl_mod.SparcLoss(temperature=0.1)(v, l, g, mask)
    loss.backward()
    out = {"captions": caps.numpy(), "images_sha": np.array(MG.sha(imgs.numpy())), "loss": np.float32(loss.item()),
           "v_sum": v.detach().numpy().sum((1, 2)), "g_sum": g.detach().numpy().sum((1, 2)), "mask": mask.numpy()}
    before = {n: params[n].detach().clone() for n in TRAIN_TENSORS}
    for n in TRAIN_TENSORS:
        gr = params[n].grad.numpy()
        out[f"grad_norm/{n}"] = np.float32(np.linalg.norm(gr.astype(np.float64)))
        out[f"grad/{n}"] = gr if gr.ndim == 1 else np.ascontiguousarray(gr[GRAD_ROWS])
    opt.step()
    for n in TRAIN_TENSORS:
        d = (params[n].detach() - before[n]).numpy()
        out[f"update/{n}"] = d if d.ndim == 1 else np.ascontiguousarray(d[GRAD_ROWS])
    path = os.path.join(HERE, "sparc_train.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, "loss", out["loss"], {k: v.shape for k, v in out.items() if k.startswith("grad/")})


def main_train_pacl():
    """One PACL head training step of train_pacl.py (train_pacl.py:16-40, 106-107: model(images, caps),
    ClipLoss(temperature=0.1), loss.backward(), torch.optim.Adam(lr = 1e-4).step()) with the
    open_clip_pacl / open_clip_pacl_rope heads (the ones-weighted patch sum, pacl.py:135-145, 184-197;
    train_pacl.py's own model, llm2clip_pacl_rope, needs network weights) on 3 images + 3 captions with
    1-block towers, dropout off as in main_train.  Writes, per variant, the loss, every head gradient
    (1-d whole, 2-d norms and rows GRAD_ROWS) and the first Adam update of the same entries."""
    import torch
    from clipembed import weights as W
    from clipembed.config import get_model_config
    torch.set_num_threads(8)
    torch.use_deterministic_algorithms(True)
    model_mod, _, pacl_mod = MG.import_reference()
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    clip, _ = MG.build_clip(model_mod, cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    imgs = torch.from_numpy(W.synthetic_images(3, seed=1450))
    caps = torch.from_numpy(W.synthetic_captions(3, seed=2450))
    out = {"captions": caps.numpy(), "images_sha": np.array(MG.sha(imgs.numpy()))}
    for tag, cls in (("pacl", pacl_mod.open_clip_pacl), ("pacl_rope", pacl_mod.open_clip_pacl_rope)):
        mod = MG.build_pacl(pacl_mod, clip, cls, heads)
        params = dict(mod.named_parameters())
        opt = torch.optim.Adam(mod.parameters(), lr=1e-4)
        opt.zero_grad()
        a, b = mod(imgs, caps)
        loss = pacl_mod.ClipLoss(temperature=0.1)(a, b)
        loss.backward()
        out[f"{tag}/loss"] = np.float32(loss.item())
        before = {n: params[n].detach().clone() for n in TRAIN_TENSORS}
        for n in TRAIN_TENSORS:
            gr = params[n].grad.numpy()
            out[f"{tag}/grad_norm/{n}"] = np.float32(np.linalg.norm(gr.astype(np.float64)))
            out[f"{tag}/grad/{n}"] = gr if gr.ndim == 1 else np.ascontiguousarray(gr[GRAD_ROWS])
        opt.step()
        for n in TRAIN_TENSORS:
            d = (params[n].detach() - before[n]).numpy()
            out[f"{tag}/update/{n}"] = d if d.ndim == 1 else np.ascontiguousarray(d[GRAD_ROWS])
        print(tag, "loss", out[f"{tag}/loss"], flush=True)
    path = os.path.join(HERE, "pacl_train.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    if sys.argv[1:] == ["dist"]:
        main_dist()
    elif sys.argv[1:] == ["train"]:
        main_train()
    elif sys.argv[1:] == ["train_pacl"]:
        main_train_pacl()
    else:
        main(full_depth=sys.argv[1:] == ["fulldepth"])
