"""Sharded SparcLoss / PACL ClipLoss on the device (ce_sparc_loss_means, ce_sparc_loss_partial,
ce_contrastive_loss_partial, ce_loss_combine) against the reference's losses over the whole
2-rank batch (tests/golden/sparc_dist.npz, made by running pacl.py:489-584 on the concatenated
shards: the nn.DataParallel semantics of train_sparc.py:93,105 / train_pacl.py:34-36,95).

The two-process test runs the product's exchange (clipembed.pacl, torch.distributed) with the
engine on both ranks.  Both ranks share the one GPU of the test box, which RCCL does not allow,
so it uses the gloo backend on the device tensors; bench.py's N > 1 legs run the same code on RCCL.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

RTOL = 1e-5      # f32 throughout (the reference's precision); sums in a different order


def _dev(xs):
    return [torch.from_numpy(x).cuda() for x in xs]


def test_sharded_sparc_loss_parts_vs_global_golden(golden):
    from clipembed.pacl import ClipLoss, SparcLoss
    from dist_inputs import pacl_shard, sparc_shard
    g = golden("sparc_dist")
    sl = SparcLoss(0.1)
    e = sl._engine(torch.empty(1, device="cuda"))
    sh = [_dev(sparc_shard(r)) for r in range(2)]
    means = [sl._means(e, v, l) for v, l, _, _ in sh]
    img_all = torch.cat([m[0] for m in means])
    txt_all = torch.cat([m[1] for m in means])
    parts = sum(sl._sparc_parts(e, img_all, txt_all, 4 * r, sh[r][1], sh[r][2], sh[r][3]) for r in range(2))
    got = float(sl._combine(e, parts, 8, 0.5, 1.0))
    np.testing.assert_allclose(got, float(g["sparc_global"]), rtol=RTOL)
    # one shard = the single-process ce_sparc_loss, = the reference on that shard alone
    for r in range(2):
        np.testing.assert_allclose(float(sl(*sh[r])), float(g[f"sparc_shard_r{r}"]), rtol=RTOL)
    # PACL ClipLoss: gathered features, each shard's rows, combine
    cl = ClipLoss(0.1)
    ph = [_dev(pacl_shard(r)) for r in range(2)]
    ia = torch.cat([p[0] for p in ph])
    ta = torch.cat([p[1] for p in ph])
    parts = sum(cl._contrastive_parts(e, ia, ta, 4 * r, 4) for r in range(2))
    np.testing.assert_allclose(float(cl._combine(e, parts, 8, 1.0, 0.0)), float(g["pacl_global"]), rtol=RTOL)
    for r in range(2):
        np.testing.assert_allclose(float(cl(*ph[r])), float(g[f"pacl_shard_r{r}"]), rtol=RTOL)


def test_sharded_loss_bad_shard_is_an_error():
    from clipembed import _lib
    from clipembed.model import _ptr, _stream, kernel_engine
    e = kernel_engine(torch.device("cuda", 0))
    x = torch.zeros(8, 768, device="cuda")
    parts = torch.zeros(5, device="cuda")
    with pytest.raises(_lib.ClipEmbedError, match="outside the global batch"):
        _lib.call("ce_contrastive_loss_partial", e.h, _stream(e.device), _ptr(x), _ptr(x), 8, 6, 4, 768, 10.0,
                  _ptr(parts))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    repo = os.path.dirname(HERE)
    sys.path[:0] = [os.path.join(repo, "clip-embeds_amd"), repo, os.path.join(HERE, "golden")]
    import torch.distributed as dist
    from clipembed.pacl import ClipLoss, SparcLoss
    from dist_inputs import pacl_shard, sparc_shard
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        v, l, g, m = _dev(sparc_shard(rank))
        img, txt = _dev(pacl_shard(rank))
        res = {"sparc": float(SparcLoss(0.1, rank=rank, world_size=world)(v, l, g, m)),
               "pacl": float(ClipLoss(0.1, rank=rank, world_size=world)(img, txt))}
        q.put((rank, res))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sparc_pacl_global_loss_two_ranks_on_device(golden):
    import torch.multiprocessing as mp
    g = golden("sparc_dist")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=180) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for r in range(2):
        np.testing.assert_allclose(got[r]["sparc"], float(g["sparc_global"]), rtol=RTOL, err_msg=f"rank {r}")
        np.testing.assert_allclose(got[r]["pacl"], float(g["pacl_global"]), rtol=RTOL, err_msg=f"rank {r}")
