"""The multi-GPU exchange step (NegCLIP variable-size all-gather, reorder, local-loss labels:
open_clip loss.py:67-87,127-164) on 2 CPU ranks over gloo, checked against the reference's
2-rank losses (tests/golden/negclip.npz).  Logits/CE are evaluated with the oracle here because
there is no device; on a GPU box the same ClipLoss runs them in libclipembed."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "clip-embeds_amd"), repo]
    from clipembed import weights as W
    from clipembed.loss import ClipLoss
    from oracle import clip_oracle as O

    class CpuCheckedLoss(ClipLoss):     # test double: oracle arithmetic, product exchange logic
        def _logits_both(self, a, b, scale, transpose=True):
            z = torch.from_numpy(np.float32(scale) * a.numpy() @ b.numpy().T)
            return z, (z.t().contiguous() if transpose else None)

        def _ce(self, logits, labels):
            return torch.tensor(O.cross_entropy(logits.numpy(), labels.numpy()))

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, D, K = 4, 768, [2, 3][rank]
    img = torch.from_numpy(O.l2normalize(W.uniform(f"neg-img-{rank}", B * D).reshape(B, D)))
    txt = torch.from_numpy(O.l2normalize(W.uniform(f"neg-txt-{rank}", (B + K) * D).reshape(B + K, D)))
    # the bench's exchange (bench.py build_clip / build_pacl): ClipLoss(local_loss=True).get_logits
    exch = CpuCheckedLoss(local_loss=True, rank=rank, world_size=world)
    li, lt = exch.get_logits(img, txt[:B], 14.2857)
    res = {
        "bench_li": li.numpy(), "bench_lt": lt.numpy(), "img": img.numpy(), "txt": txt[:B].numpy(),
        "hard": float(CpuCheckedLoss(local_loss=True, rank=rank, world_size=world, usehardtext=True)(img, txt, 14.2857)),
        "plain_local": float(CpuCheckedLoss(local_loss=True, rank=rank, world_size=world)(img, txt[:B], 14.2857)),
        "plain_global": float(CpuCheckedLoss(local_loss=False, rank=rank, world_size=world)(img, txt[:B], 14.2857)),
    }
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_negclip_exchange_two_ranks(golden):
    g = golden("negclip")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    all_img = np.concatenate([got[r]["img"] for r in range(2)])
    all_txt = np.concatenate([got[r]["txt"] for r in range(2)])
    for r in range(2):
        for k in ("hard", "plain_local", "plain_global"):
            np.testing.assert_allclose(got[r][k], float(g[f"{k}_r{r}"]), rtol=1e-5, err_msg=f"{k} rank {r}")
        # bench.py's exchange: this rank's rows against every rank's embeddings, rank order
        # (loss.py:155-157: logits_per_image = s I_local T_all^T, logits_per_text = s T_local I_all^T)
        li, lt = got[r]["bench_li"], got[r]["bench_lt"]
        assert li.shape == (4, 8) and lt.shape == (4, 8)
        np.testing.assert_allclose(li, np.float32(14.2857) * got[r]["img"] @ all_txt.T, rtol=1e-6)
        np.testing.assert_allclose(lt, np.float32(14.2857) * got[r]["txt"] @ all_img.T, rtol=1e-6)
        # and its loss is the reference's 2-rank ClipLoss(local_loss=True)
        lab = np.arange(4) + 4 * r
        from oracle import clip_oracle as O
        loss = (O.cross_entropy(li, lab) + O.cross_entropy(lt, lab)) / 2
        np.testing.assert_allclose(loss, float(g[f"plain_local_r{r}"]), rtol=1e-5)


def _train_worker(rank, world, port, q):
    """negclip_feature_grad (the trainer's exchange + gradient bookkeeping) with a torch test double
    for the engine's ce_contrastive_grad, against the reference's autograd through its 2-rank
    ClipLoss(local_loss, gather_with_grad, usehardtext) (tests/golden/train_dist.npz)."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "clip-embeds_amd"), repo]
    from clipembed.train import negclip_feature_grad

    g = dict(np.load(os.path.join(repo, "tests", "golden", "train_dist.npz")))
    acc = torch.zeros(2, dtype=torch.float64)

    def cgrad(a, b, scale, labels, inv_count, da, db, weight):   # f64 restatement of ce_contrastive_grad
        a64, b64 = a.double(), b.double()
        z = scale * a64 @ b64.T
        p = torch.softmax(z, dim=1)
        valid = labels >= 0
        onehot = torch.zeros_like(z)
        onehot[valid, labels[valid]] = 1.0
        gz = weight * inv_count * (p - onehot) * valid[:, None]
        lse = torch.logsumexp(z, dim=1)
        zl = z.gather(1, labels.clamp(min=0)[:, None])[:, 0]
        acc[0] += (weight * inv_count * (lse - zl) * valid).sum()
        acc[1] += (gz * z).sum()
        if da is not None:
            da += (scale * gz @ b64).to(da.dtype)
        if db is not None:
            db += (scale * gz.T @ a64).to(db.dtype)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    img = torch.from_numpy(g[f"img_r{rank}"])
    txt = torch.from_numpy(g[f"txt_r{rank}"])
    dtxt = negclip_feature_grad(img, txt, 12.5, rank, world, cgrad)
    q.put((rank, {"dtxt": dtxt.numpy(), "loss": float(acc[0]), "dlogit_scale": float(acc[1])}))
    dist.barrier()
    dist.destroy_process_group()


def test_train_feature_grad_two_ranks(golden):
    g = golden("train_dist")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        np.testing.assert_allclose(got[r]["loss"], float(g[f"loss_r{r}"]), rtol=1e-5)
        # d loss / d logit_scale = scale * d loss / d scale (the reference differentiates w.r.t. scale)
        np.testing.assert_allclose(got[r]["dlogit_scale"], 12.5 * float(g[f"dscale_r{r}"]), rtol=1e-4)
        np.testing.assert_allclose(got[r]["dtxt"], g[f"dtxt_r{r}"], rtol=1e-4, atol=1e-7)


def _loss_worker(rank, world, port, q, uneven=None):
    """clipembed.pacl.SparcLoss / ClipLoss(rank, world_size) on 2 gloo ranks: the product's exchange
    (all-gather of the [B,768] means / features, shard row offsets, all-reduce of the 5 partial sums)
    with the oracle's arithmetic in place of the engine calls (test double: no device here)."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "clip-embeds_amd"), repo, os.path.join(repo, "tests", "golden")]
    from clipembed.pacl import ClipLoss, SparcLoss
    from dist_inputs import pacl_shard, sparc_shard
    from oracle import clip_oracle as O

    class Double:
        def _engine(self, t):
            return None

        def _contrastive_parts(self, e, img_all, txt_all, row0, B):
            return torch.from_numpy(O.contrastive_loss_parts(img_all.numpy(), txt_all.numpy(), row0, B,
                                                             self.logit_scale).astype(np.float32))

        def _combine(self, e, parts, n, wg, wl):
            return torch.tensor(O.loss_combine(parts.double().numpy(), n, wg, wl))

        def _means(self, e, v, lt):
            gi, gt = O.sparc_loss_means(v.numpy(), lt.numpy())
            return torch.from_numpy(gi), torch.from_numpy(gt)

        def _sparc_parts(self, e, img_all, txt_all, row0, lt, g, m):
            return torch.from_numpy(O.sparc_loss_parts(img_all.numpy(), txt_all.numpy(), row0, lt.numpy(), g.numpy(),
                                                       m.numpy(), 1.0 / self.logit_scale).astype(np.float32))

    class CpuSparcLoss(Double, SparcLoss):
        pass

    class CpuClipLoss(Double, ClipLoss):
        pass

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = uneven[rank] if uneven else 4
    v, l, g, m = (torch.from_numpy(x[:n]) for x in sparc_shard(rank))
    img, txt = (torch.from_numpy(x[:n]) for x in pacl_shard(rank))
    res = {"sparc": float(CpuSparcLoss(0.1, rank=rank, world_size=world)(v, l, g, m)),
           "pacl": float(CpuClipLoss(0.1, rank=rank, world_size=world)(img, txt))}
    if rank == 0:     # the sharded loss is value-only: inputs that require grad are refused
        try:
            CpuClipLoss(0.1, rank=rank, world_size=world)(img.clone().requires_grad_(), txt)
            res["grad_refused"] = False
        except RuntimeError:
            res["grad_refused"] = True
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_sparc_pacl_global_loss_two_ranks(golden):
    """Every rank returns the reference's loss over the WHOLE 2-rank batch (train_sparc.py:93,105 /
    train_pacl.py:34-36,95: DataParallel gathers, the loss runs on the global batch), not its shard's."""
    g = golden("sparc_dist")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loss_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        np.testing.assert_allclose(got[r]["sparc"], float(g["sparc_global"]), rtol=1e-5, err_msg=f"rank {r}")
        np.testing.assert_allclose(got[r]["pacl"], float(g["pacl_global"]), rtol=1e-5, err_msg=f"rank {r}")
        assert abs(got[r]["sparc"] - float(g[f"sparc_shard_r{r}"])) > 0.05     # not the shard-local value
        assert abs(got[r]["pacl"] - float(g[f"pacl_shard_r{r}"])) > 0.05


def test_sparc_pacl_global_loss_uneven_shards():
    """Ranks holding different batch sizes (4 and 2 samples: an uneven last batch; nn.DataParallel
    scatters unevenly too): sizes are gathered first, rows padded, and every rank returns the loss
    over the whole 6-sample batch (the oracle, pinned to the reference by the tests above, on the
    concatenated batch)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from dist_inputs import pacl_shard, sparc_shard
    from oracle import clip_oracle as O
    sizes = (4, 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loss_worker, args=(r, 2, port, q, sizes)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sh = [[x[:n] for x in sparc_shard(r)] for r, n in enumerate(sizes)]
    v, l, g, m = (np.concatenate([s[k] for s in sh]) for k in range(4))
    gi, gt = O.sparc_loss_means(v, l)
    want_sparc = O.loss_combine(O.sparc_loss_parts(gi, gt, 0, l, g, m, 0.1), 6, 0.5, 1.0)
    ph = [[x[:n] for x in pacl_shard(r)] for r, n in enumerate(sizes)]
    img, txt = (np.concatenate([s[k] for s in ph]) for k in range(2))
    want_pacl = O.loss_combine(O.contrastive_loss_parts(img, txt, 0, 6, 10.0), 6, 1.0, 0.0)
    for r in range(2):
        np.testing.assert_allclose(got[r]["sparc"], want_sparc, rtol=1e-5, err_msg=f"rank {r}")
        np.testing.assert_allclose(got[r]["pacl"], want_pacl, rtol=1e-5, err_msg=f"rank {r}")
    assert got[0]["grad_refused"]


def test_oracle_shard_parts_add_up(golden):
    """The oracle's shard decomposition (the arithmetic ce_sparc_loss_partial / ce_loss_combine
    follow) reproduces the reference's one-shard losses too."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from dist_inputs import sparc_shard
    from oracle import clip_oracle as O
    g = golden("sparc_dist")
    for r in range(2):
        v, l, gr, m = sparc_shard(r)
        gi, gt = O.sparc_loss_means(v, l)
        p = O.sparc_loss_parts(gi, gt, 0, l, gr, m, 0.1)
        np.testing.assert_allclose(O.loss_combine(p, 4, 0.5, 1.0), float(g[f"sparc_shard_r{r}"]), rtol=1e-5)
