"""The N > 1 NegCLIP text-tower trainer on the device (BASELINE configs[3]'s exchange), two ranks.

The reference step: ClipLoss(local_loss=True, gather_with_grad=True, usehardtext) gathers image
features, text sizes and padded text features (open_clip loss.py:67-87,137-193), and DDP averages the
text tower's gradients over ranks (open_clip_train/main.py:302).  clipembed.train implements both
with torch.distributed: all_gather (features, sizes), reduce_scatter_tensor (the gather's backward)
and one all_reduce of the flat gradient buffer.  Here two spawned ranks share cuda:0 over gloo (RCCL
runs one rank per device; the driver's 8-GPU run uses RCCL) and run the engine:

  * feature level: negclip_feature_grad with the engine's ce_contrastive_grad on the reference's
    2-rank inputs, against the reference's own 2-rank autograd (tests/golden/train_dist.npz: loss,
    d loss / d scale, d loss / d text features per rank);
  * whole step (with the bucketed, backward-overlapped gradient all-reduce and with one all-reduce
    after the backward): TextTowerTrainer(rank, world_size=2) on 3 images + 3 / 2 captions per rank (hard
    negatives of different counts, so the size gather and padding are exercised), against one
    TextTowerTrainer(world_size=1) on the concatenated batch [originals r0, originals r1, hard r0,
    hard r1]: data parallelism must not change the step, so the DDP-averaged gradient equals the
    single-process gradient (the sum of the two local losses' gradients is twice the global one) and
    the first AdamW update equals the single-process update.

If this torch build's gloo has no reduce_scatter for device tensors, the workers stage only that one
collective through host memory (the product's call is unchanged; the result records which ran)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
B, HARD = 3, (2, 1)
N_SAMPLE = 8192


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(rank, world, port):
    sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # probe: gloo's reduce_scatter on device tensors (some builds support CPU tensors only)
    staged = False
    try:
        o = torch.zeros(2, device="cuda")
        dist.reduce_scatter_tensor(o, torch.ones(2 * world, device="cuda"))
        assert torch.equal(o.cpu(), torch.full((2,), float(world)))
    except (RuntimeError, ValueError, NotImplementedError):
        staged = True
        real = dist.reduce_scatter_tensor

        def host_staged(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
            o = output.cpu()
            real(o, input.cpu(), op=op, group=group)
            output.copy_(o)

        dist.reduce_scatter_tensor = host_staged      # this test process's backend only
    return dist, staged


def _feature_worker(rank, world, port, q):
    dist, staged = _setup(rank, world, port)
    try:
        from clipembed import _lib
        from clipembed.model import _ptr, _stream, kernel_engine
        from clipembed.train import negclip_feature_grad
        g = dict(np.load(os.path.join(HERE, "golden", "train_dist.npz")))
        e = kernel_engine(torch.device("cuda", 0))
        lossbuf = torch.zeros(2, device="cuda")

        def cgrad(a, b, scale, labels, inv_count, da, db, weight):    # the trainer's _cgrad
            _lib.call("ce_contrastive_grad", e.h, _stream(e.device), _ptr(a), a.shape[0], _ptr(b), b.shape[0],
                      a.shape[1], float(scale), _ptr(labels), float(weight), float(inv_count), _ptr(lossbuf),
                      _ptr(da), _ptr(db))

        img = torch.from_numpy(g[f"img_r{rank}"]).cuda()
        txt = torch.from_numpy(g[f"txt_r{rank}"]).cuda()
        dtxt = negclip_feature_grad(img, txt, 12.5, rank, world, cgrad)
        torch.cuda.synchronize()
        q.put((rank, {"dtxt": dtxt.cpu().numpy(), "loss": float(lossbuf[0]), "dls": float(lossbuf[1]),
                      "staged": staged}))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(target, extra=()):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, 2, port, q) + tuple(extra)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=300) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return got


def test_negclip_feature_grad_two_ranks_engine_vs_reference(golden):
    g = golden("train_dist")
    got = _spawn(_feature_worker)
    for r in range(2):
        np.testing.assert_allclose(got[r]["loss"], float(g[f"loss_r{r}"]), rtol=1e-5, err_msg=f"rank {r}")
        # the engine's second slot is d loss / d logit_scale = scale * d loss / d scale
        np.testing.assert_allclose(got[r]["dls"], 12.5 * float(g[f"dscale_r{r}"]), rtol=1e-4, err_msg=f"rank {r}")
        np.testing.assert_allclose(got[r]["dtxt"], g[f"dtxt_r{r}"], rtol=1e-4, atol=1e-7, err_msg=f"rank {r}")
    print("reduce_scatter on device tensors:", "host-staged (gloo)" if got[0]["staged"] else "gloo native")


# ---------------------------------------------------------------------------------------- whole step
def _inputs():
    sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]
    from clipembed import weights as W
    imgs = [W.synthetic_images(B, seed=300 + r) for r in range(2)]
    caps = [W.synthetic_captions(B + HARD[r], seed=400 + r) for r in range(2)]
    return imgs, caps


def _trainer(world, rank, bucket_blocks=1):
    import clipembed
    from clipembed import weights as W
    from clipembed.config import get_model_config
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 2)
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    m.to("cuda")
    return clipembed.TextTowerTrainer(m, lr=5e-6, usehardtext=True, rank=rank, world_size=world,
                                      bucket_blocks=bucket_blocks)


def _summary(tr, loss, before, idx):
    g = tr.grad
    upd = (tr.param - before)
    names = ["text_projection", "transformer.resblocks.1.mlp.c_proj.weight", "transformer.resblocks.0.attn.in_proj_bias",
             "ln_final.weight", "positional_embedding"]
    return {"loss": float(loss), "g_sample": g[idx].cpu().numpy(), "u_sample": upd[idx].cpu().numpy(),
            "g_norm": float(g.norm()), "g_tensors": {n: tr.gviews[n].cpu().numpy() for n in names},
            "dls": float(g[-1]), "u_ls": float(upd[-1])}


def _step_worker(rank, world, port, q, idx, bucket_blocks):
    dist, staged = _setup(rank, world, port)
    try:
        imgs, caps = _inputs()
        tr = _trainer(world, rank, bucket_blocks)
        before = tr.param.clone()
        loss = tr.compute_grads(torch.from_numpy(imgs[rank]).cuda(), torch.from_numpy(caps[rank]).cuda())
        tr.apply_update()
        torch.cuda.synchronize()
        res = _summary(tr, loss, before, torch.from_numpy(idx).cuda())
        res["staged"] = staged
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _cos(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


@pytest.mark.parametrize("bucket_blocks", [1, 0])
def test_negclip_step_two_ranks_equals_one_rank_on_concatenated_batch(bucket_blocks):
    """bucket_blocks 1: the per-block bucketed all-reduce overlapped with the backward (the default);
    0: one all-reduce of the whole buffer after it."""
    imgs, caps = _inputs()
    tr = _trainer(1, 0)
    n = tr.n_total
    idx = np.random.default_rng(5).choice(n - 1, N_SAMPLE, replace=False).astype(np.int64)
    idx = np.concatenate([idx, [n - 1]])
    # the single process sees originals of every rank first, then every rank's hard negatives
    # (the order the 2-rank gather builds, loss.py:144-153)
    all_caps = np.concatenate([caps[0][:B], caps[1][:B], caps[0][B:], caps[1][B:]])
    before = tr.param.clone()
    loss1 = tr.compute_grads(torch.from_numpy(np.concatenate(imgs)).cuda(), torch.from_numpy(all_caps).cuda())
    tr.apply_update()
    torch.cuda.synchronize()
    one = _summary(tr, loss1, before, torch.from_numpy(idx).cuda())
    del tr
    torch.cuda.empty_cache()

    got = _spawn(_step_worker, (idx, bucket_blocks))
    print("reduce_scatter on device tensors:", "host-staged (gloo)" if got[0]["staged"] else "gloo native")
    # the mean of the two local losses is the global loss
    np.testing.assert_allclose((got[0]["loss"] + got[1]["loss"]) / 2, one["loss"], rtol=2e-4)
    for r in range(2):
        two = got[r]
        # DDP-averaged gradient == single-process gradient (bf16 GEMMs on different row tilings)
        assert _cos(two["g_sample"], one["g_sample"]) > 0.9999, r
        np.testing.assert_allclose(two["g_norm"], one["g_norm"], rtol=5e-3)
        np.testing.assert_allclose(two["dls"], one["dls"], rtol=2e-3, atol=1e-6)
        for name, v in one["g_tensors"].items():
            assert _cos(two["g_tensors"][name], v) > 0.999, (r, name)
        # both ranks hold the same averaged gradient and apply the same update
        np.testing.assert_array_equal(two["g_sample"], got[0]["g_sample"])
        np.testing.assert_array_equal(two["u_sample"], got[0]["u_sample"])
        # first AdamW step: update = -lr * g / (|g| + eps) (+ decay): equal wherever g is clear of eps and
        # of the bf16 GEMMs' noise, which is relative to the tensor's scale, not to each element
        # (|g| >= 1e-4 = 100 eps: there du/u = eps / (|g| + eps) * dg/g <= 1e-2 dg/g)
        gs = np.abs(one["g_sample"])
        big = gs > max(1e-4, float(np.quantile(gs, 0.9)))
        assert big.sum() >= 50
        np.testing.assert_allclose(two["u_sample"][big], one["u_sample"][big], rtol=2e-2, atol=1e-7)
        np.testing.assert_allclose(two["u_ls"], one["u_ls"], rtol=2e-2, atol=1e-7)
