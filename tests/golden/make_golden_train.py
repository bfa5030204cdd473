"""Golden fixtures for the text-tower training step from the REFERENCE itself.

Runs only in the build container.  Imports open_clip's model / loss modules from the read-only
reference tree (make_golden.import_reference: two in-process stubs) and runs, on CPU
in f32 with autograd, the step open_clip_train/train.py:85-189 performs for train-clip.sh
(--lock-image --local-loss --gather-with-grad --usehardtext): the locked image tower forward,
the text tower forward, ClipLoss with hard negatives, backward, then torch.optim.AdamW with the
two parameter groups of main.py:335-349 and the logit_scale clamp of train.py:189.  Writes
outputs only: loss values, gradients (small tensors whole, large ones sampled at fixed indices),
parameter updates, the logit_scale trajectory, and (2 gloo ranks) the gradient of the loss w.r.t.
each rank's text features.

    python tests/golden/make_golden_train.py
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from make_golden import W, get_model_config  # noqa: E402

NSAMP = 2048
LR, WD, BETAS, EPS = 1e-4, 0.1, (0.9, 0.98), 1e-6
B_IMG, N_TXT = 4, 6          # 2 hard-negative captions


def sample_idx(name: str, t, used_rows=None):
    n = t.numel()
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    if used_rows is not None:                 # token embedding: only rows that occur carry gradient
        D = t.shape[1]
        rows = rng.choice(used_rows, size=NSAMP)
        return (rows * D + rng.integers(0, D, size=NSAMP)).astype(np.int64)
    if n <= 4096:
        return np.arange(n, dtype=np.int64)
    return rng.choice(n, size=NSAMP, replace=False).astype(np.int64)


def excluded(n, p):
    return p.ndim < 2 or "bn" in n or "ln" in n or "bias" in n or "logit_scale" in n


def train_single(model_mod, loss_mod, out):
    import torch
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 2)
    m, sd = MG.build_clip(model_mod, cfg)
    m.train()
    m.lock_image_tower()
    imgs = torch.from_numpy(W.synthetic_images(B_IMG, seed=3100))
    caps = torch.from_numpy(W.synthetic_captions(N_TXT, seed=3200))
    loss_fn = loss_mod.ClipLoss(local_loss=True, gather_with_grad=True, usehardtext=True)
    named = [(n, p) for n, p in m.named_parameters() if p.requires_grad]
    assert all(not n.startswith("visual.") for n, _ in named)
    opt = torch.optim.AdamW([{"params": [p for n, p in named if excluded(n, p)], "weight_decay": 0.},
                             {"params": [p for n, p in named if not excluded(n, p)], "weight_decay": WD}],
                            lr=LR, betas=BETAS, eps=EPS)
    p0 = {n: p.detach().clone() for n, p in named}
    res = {"images_seed": np.int64(3100), "captions_seed": np.int64(3200), "captions": caps.numpy()}
    losses = []
    for it in range(3):
        opt.zero_grad()
        f_img, f_txt, scale = m(imgs, caps)
        f_txt.retain_grad()
        loss = loss_fn(f_img, f_txt, scale)
        loss.backward()
        losses.append(float(loss))
        if it == 0:
            res["dtxt"] = f_txt.grad.numpy().copy()
            used = np.unique(caps.numpy())
            for n, p in named:
                idx = sample_idx(n, p, used if n == "token_embedding.weight" else None)
                res[f"gidx:{n}"] = idx
                res[f"grad:{n}"] = p.grad.reshape(-1)[idx].numpy().copy()
                res[f"gnorm:{n}"] = np.float64(p.grad.double().norm())
        opt.step()
        with torch.no_grad():
            m.logit_scale.clamp_(0, np.log(100))
        if it == 0:
            for n, p in named:
                idx = res[f"gidx:{n}"]
                res[f"delta:{n}"] = (p.detach() - p0[n]).reshape(-1)[idx].numpy().copy()
    res["losses"] = np.array(losses, dtype=np.float64)
    res["logit_scale_final"] = np.float64(m.logit_scale.detach())
    out["train"] = res


def _dist_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, loss_mod, _ = MG.import_reference()
    B, E, K = 3, 768, [2, 1][rank]
    img = torch.nn.functional.normalize(torch.from_numpy(W.uniform(f"tr-img-{rank}", B * E).reshape(B, E)), dim=-1)
    txt = torch.nn.functional.normalize(
        torch.from_numpy(W.uniform(f"tr-txt-{rank}", (B + K) * E).reshape(B + K, E)), dim=-1).requires_grad_(True)
    scale = torch.tensor(12.5, requires_grad=True)
    fn = loss_mod.ClipLoss(local_loss=True, gather_with_grad=True, rank=rank, world_size=world, usehardtext=True)
    loss = fn(img, txt, scale)
    loss.backward()
    q.put((rank, {"img": img.numpy(), "txt": txt.detach().numpy(), "loss": float(loss),
                  "dtxt": txt.grad.numpy(), "dscale": float(scale.grad)}))
    dist.destroy_process_group()


def train_dist(out):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, 29631, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join()
    res = {}
    for r in range(2):
        for k, v in got[r].items():
            res[f"{k}_r{r}"] = np.asarray(v)
    out["train_dist"] = res


def main():
    import torch
    torch.manual_seed(0)
    torch.set_num_threads(8)
    model_mod, loss_mod, _ = MG.import_reference()
    out = {}
    train_single(model_mod, loss_mod, out)
    train_dist(out)
    MG.save(out)


if __name__ == "__main__":
    main()
