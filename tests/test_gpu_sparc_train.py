"""SPARC head training step on the device (BASELINE configs[4]; train_sparc.py:29-37,91,106 on
model/pacl.py:380-584) through the C ABI (ce_sparc_train_*, clipembed.SparcHeadTrainer):

  * vs the reference's own step (tests/golden/sparc_train.npz, make_golden_sparc.py train: sparc_rope on
    1-block towers, SparcLoss(0.1), loss.backward(), torch.optim.Adam(lr 1e-4), dropout off): loss, every
    head gradient (rows / norms) and the first Adam update;
  * vs the f32 autograd restatement (oracle/sparc_train_torch.py, pinned to that golden step on the CPU)
    on the engine's own tower tokens at 16 samples: without dropout, with the engine's dropout masks
    (restated here from the counter hash), and with precomputed token embeddings (the configs[4] input);
  * loss decreasing over a few steps.
Tolerances: the visual head's GEMMs run on bf16 operands with f32 accumulation (the text head and the
alignment in f32), so gradients are compared by cosine (>= 0.995) and norm (within 3 %)."""
import numpy as np
import pytest
import torch

import clipembed
from clipembed import weights as W
from clipembed.config import get_model_config
from clipembed.pacl import sparc, sparc_rope
from clipembed.sparc_train import HEAD_TENSORS

pytestmark = pytest.mark.gpu

ROWS = [0, 1, 383, 767]


def _cos(a, b):
    a, b = torch.as_tensor(a).double().reshape(-1), torch.as_tensor(b).double().reshape(-1)
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-30))


def keep_mask(seed, n, p):
    """The engine's dropout keep mask (sparc_train.hip drop_keep): top 24 bits of splitmix64's n-th
    output for state `seed` >= p * 2^24."""
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64)
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z ^= z >> np.uint64(31)
    return (z >> np.uint64(40)) >= np.uint64(int(p * 16777216.0))


@pytest.fixture(scope="module")
def cfg():
    return get_model_config("ViT-L-14-336").with_depth(1, 1)


@pytest.fixture(scope="module")
def sd(cfg):
    return W.synthetic_state_dict(cfg)


def _model(cls, cfg, sd):
    m = cls(sigma=1.0 / 576, cfg=cfg, clip_state_dict=sd)
    m.init_synthetic_heads()
    m.to("cuda")
    return m


def test_step_matches_reference(golden, cfg, sd):
    g = golden("sparc_train")
    m = _model(sparc_rope, cfg, sd)
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    imgs = torch.from_numpy(W.synthetic_images(3, seed=1400)).cuda()
    caps = torch.from_numpy(g["captions"]).cuda()
    before = {n: v.detach().clone() for n, v in tr.views.items()}
    loss = float(tr.compute_grads(imgs, caps))
    np.testing.assert_allclose(loss, g["loss"], rtol=5e-3)
    bad = []
    for n in HEAD_TENSORS:
        gv = tr.gviews[n].cpu()
        ours = gv if gv.dim() == 1 else gv[ROWS]
        c = _cos(ours, g[f"grad/{n}"])
        nr = float(gv.double().norm()) / float(g[f"grad_norm/{n}"])
        if not (c >= 0.995 and abs(nr - 1) < 0.03):
            bad.append((n, round(c, 5), round(nr, 4)))
    assert not bad, bad
    # first Adam step: (a) the engine's update is torch.optim.Adam's on the engine's own gradients (to f32
    # rounding); (b) vs the reference's update (lr * m_hat / (sqrt(v_hat) + eps) = -lr sign(g) where
    # |g| >> eps) on every entry above 10 % of the tensor's largest gradient -- below that the bf16
    # operands of the visual head's GEMMs may flip the sign of a small gradient, and Adam's first step
    # turns that into a full -/+ lr difference
    ref_p = {n: before[n].clone().requires_grad_(True) for n in HEAD_TENSORS}
    for n in HEAD_TENSORS:
        ref_p[n].grad = tr.gviews[n].detach().clone()
    torch.optim.Adam(list(ref_p.values()), lr=1e-4).step()
    tr.apply_update()
    for n in HEAD_TENSORS:
        torch.testing.assert_close(tr.views[n], ref_p[n].detach(), rtol=1e-5, atol=1e-9, msg=n)
        d = (tr.views[n] - before[n]).cpu().numpy()
        d = d if d.ndim == 1 else d[ROWS]
        ref, gref = g[f"update/{n}"], g[f"grad/{n}"]
        big = np.abs(gref) > 0.1 * np.abs(gref).max()
        np.testing.assert_allclose(d[big], ref[big], rtol=2e-3, atol=1e-9, err_msg=n)


@pytest.fixture(scope="module")
def b16(cfg, sd):
    """16 samples' frozen tower tokens from the engine (reduced depth), shared by the oracle comparisons."""
    m = _model(sparc_rope, cfg, sd)
    imgs = torch.from_numpy(W.synthetic_images(16, seed=1500)).cuda()
    caps = torch.from_numpy(W.synthetic_captions(16, seed=2500)).cuda()
    _, pt = m.clip_model.encode_image(imgs)
    _, tt = m.clip_model.encode_text(caps)
    mask = (torch.arange(77, device="cuda")[None, :] <= caps.argmax(-1)[:, None]).float()
    return dict(m=m, imgs=imgs, caps=caps, pt=pt, tt=tt, mask=mask)


def _vs_oracle(tr, ref_loss, ref_grads, loss, skip=()):
    np.testing.assert_allclose(loss, ref_loss, rtol=5e-3)
    bad = []
    for n in HEAD_TENSORS:
        if n in skip:
            assert float(tr.gviews[n].abs().max()) == 0.0, n
            continue
        c = _cos(tr.gviews[n], ref_grads[n])
        nr = float(tr.gviews[n].double().norm() / ref_grads[n].double().norm())
        if not (c >= 0.995 and abs(nr - 1) < 0.03):
            bad.append((n, round(c, 5), round(nr, 4)))
    assert not bad, bad


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_step_matches_oracle(b16, dropout):
    from oracle.sparc_train_torch import TorchSparcTrainStep
    m = b16["m"]
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=dropout, seed=11)
    loss = float(tr.compute_grads(b16["imgs"], b16["caps"]))
    B, P, Dv = b16["pt"].shape
    T, E = b16["tt"].shape[1:]
    kv = kt = None
    if dropout:
        s = tr.last_seed
        kv = torch.from_numpy(keep_mask(2 * s, B * P * Dv, dropout).reshape(B, P, Dv).astype(np.float32))
        kt = torch.from_numpy(keep_mask(2 * s + 1, B * T * E, dropout).reshape(B, T, E).astype(np.float32))
        assert abs(float(kv.mean()) - (1 - dropout)) < 2e-3
    step = TorchSparcTrainStep({n: v.detach() for n, v in tr.views.items()}, device="cuda")
    pv = clipembed.pacl.apply_rope(b16["pt"], engine=m.engine)
    ref_loss, ref_grads, _ = step.loss_and_grads(pv, b16["mask"], text_tokens=b16["tt"], p=dropout, keep_v=kv,
                                                 keep_t=kt)
    _vs_oracle(tr, ref_loss, ref_grads, loss)


def test_text_embeddings_input(b16, cfg, sd):
    """BASELINE configs[4]'s input: precomputed token embeddings [B, 77, 768] + mask, no text head (its
    gradients are zero); sparc (no RoPE)."""
    from oracle.sparc_train_torch import TorchSparcTrainStep
    m = _model(sparc, cfg, sd)
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    gen = torch.Generator(device="cpu").manual_seed(3)
    l_tok = (torch.randn(16, 77, 768, generator=gen) * 0.5).cuda()
    mask = b16["mask"]
    loss = float(tr.compute_grads(b16["imgs"], l_token_embed=l_tok, language_mask=mask))
    step = TorchSparcTrainStep({n: v.detach() for n, v in tr.views.items()}, device="cuda")
    ref_loss, ref_grads, _ = step.loss_and_grads(b16["pt"], mask, l_token_embed=l_tok, p=0.0)
    _vs_oracle(tr, ref_loss, ref_grads, loss, skip=[n for n in HEAD_TENSORS if n.startswith("text_projection")])


def test_loss_decreases(b16):
    tr = clipembed.SparcHeadTrainer(b16["m"], lr=1e-4, dropout=0.1)
    losses = [tr.step(b16["imgs"], b16["caps"]) for _ in range(4)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses


# ------------------------------------------------------------------------------- two ranks (gloo)
def _dist_inputs(r):
    gen = torch.Generator(device="cpu").manual_seed(40 + r)
    l_tok = torch.randn(3, 77, 768, generator=gen) * 0.5
    eot = torch.randint(6, 42, (3,), generator=gen)
    mask = (torch.arange(77)[None, :] <= eot[:, None]).float()
    return W.synthetic_images(3, seed=1600 + r), l_tok, mask


def _dist_trainer(world, rank, dropout):
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    m = _model(sparc_rope, cfg, W.synthetic_state_dict(cfg))
    return clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=dropout, rank=rank, world_size=world)


def _dist_worker(rank, world, port, q, dropout):
    import os
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        imgs, l_tok, mask = _dist_inputs(rank)
        tr = _dist_trainer(world, rank, dropout)
        before = tr.param.clone()
        loss = tr.compute_grads(torch.from_numpy(imgs).cuda(), l_token_embed=l_tok.cuda(), language_mask=mask.cuda())
        tr.apply_update()
        torch.cuda.synchronize()
        q.put((rank, {"loss": float(loss), "grad": tr.grad.cpu().numpy(), "upd": (tr.param - before).cpu().numpy()}))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_two_ranks_equal_one_rank_on_concatenated_batch(dropout):
    """BASELINE configs[4]'s exchange (train_sparc.py:93: nn.DataParallel, the loss over the gathered
    batch, the replicas' gradients summed): two spawned ranks on cuda:0 over gloo (RCCL on the
    driver's multi-GPU node), 3 samples each, against one rank on the 6 concatenated samples: the same
    loss, the same summed gradient and the same first Adam step on both ranks.  With dropout the masks
    index the global batch, so the two ranks draw the single-device step's masks."""
    import socket
    import torch.multiprocessing as mp
    ins = [_dist_inputs(r) for r in range(2)]
    tr = _dist_trainer(1, 0, dropout)
    before = tr.param.clone()
    loss1 = float(tr.compute_grads(torch.from_numpy(np.concatenate([i[0] for i in ins])).cuda(),
                                   l_token_embed=torch.cat([i[1] for i in ins]).cuda(),
                                   language_mask=torch.cat([i[2] for i in ins]).cuda()))
    g1 = tr.grad.cpu().numpy()
    tr.apply_update()
    u1 = (tr.param - before).cpu().numpy()
    del tr
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q, dropout)) for r in range(2)]
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
    for r in range(2):
        np.testing.assert_allclose(got[r]["loss"], loss1, rtol=1e-4)
        assert _cos(got[r]["grad"], g1) > 0.9999, r
        np.testing.assert_allclose(np.linalg.norm(got[r]["grad"]), np.linalg.norm(g1), rtol=2e-3)
        np.testing.assert_array_equal(got[r]["grad"], got[0]["grad"])
        np.testing.assert_array_equal(got[r]["upd"], got[0]["upd"])
        big = np.abs(g1) > 0.1 * np.abs(g1).max()
        np.testing.assert_allclose(got[r]["upd"][big], u1[big], rtol=2e-3, atol=1e-9)


@pytest.mark.parametrize("B", [1, 5])
def test_small_batches_vs_oracle(cfg, sd, B):
    """B = 1 (the global term's 1 x 1 logits: zero loss and gradient) and an odd batch, sparc without
    RoPE on the caption path, vs the f32 autograd restatement."""
    from oracle.sparc_train_torch import TorchSparcTrainStep
    m = _model(sparc, cfg, sd)
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1700 + B)).cuda()
    caps = torch.from_numpy(W.synthetic_captions(B, seed=2700 + B)).cuda()
    loss = float(tr.compute_grads(imgs, caps))
    _, pt = m.clip_model.encode_image(imgs)
    _, tt = m.clip_model.encode_text(caps)
    mask = (torch.arange(77, device="cuda")[None, :] <= caps.argmax(-1)[:, None]).float()
    step = TorchSparcTrainStep({n: v.detach() for n, v in tr.views.items()}, device="cuda")
    ref_loss, ref_grads, _ = step.loss_and_grads(pt, mask, text_tokens=tt, p=0.0)
    _vs_oracle(tr, ref_loss, ref_grads, loss)


def test_errors(cfg, sd):
    """The C ABI's state machine and argument checks (include/clipembed.h: ce_sparc_train_*)."""
    from clipembed import _lib
    from clipembed.model import _ptr, _stream
    m = _model(sparc_rope, cfg, sd)
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    h, s = tr.e.h, _stream(tr.dev)
    with pytest.raises(RuntimeError, match="needs ce_sparc_train_forward"):
        _lib.call("ce_sparc_train_backward", h, s)
    x = torch.zeros(2, 576, 1024, device="cuda")
    t = torch.zeros(2, 81, 768, device="cuda")
    with pytest.raises(RuntimeError, match="no ce_sparc_train_forward"):
        _lib.call("ce_sparc_train_loss_grad", h, s, _ptr(x), _ptr(x), 2, 0, _ptr(x), 1.0, 0.1, 0.5, 1.0, _ptr(x))
    import ctypes
    fwd = lambda P, rope, T, p: _lib.call("ce_sparc_train_forward", h, s, _ptr(x), 2, P, rope, _ptr(t), 0, T, 1 / 576, p,
                                          ctypes.c_uint64(0), ctypes.c_int64(0), None, None, None)
    with pytest.raises(RuntimeError, match="T <= 80"):
        fwd(576, 1, 81, 0.0)
    with pytest.raises(RuntimeError, match="rope tables"):
        fwd(500, 1, 77, 0.0)
    with pytest.raises(RuntimeError, match="dropout"):
        fwd(576, 1, 77, 1.0)
    # a bind that leaves a head tensor out
    Pn = (_lib.Tensor * 1)()
    from clipembed.train import _tensor_entry
    Pn[0] = _tensor_entry(b"visual_projection.0.weight", tr.views["visual_projection.0.weight"])
    with pytest.raises(RuntimeError, match="not bound"):
        _lib.call("ce_sparc_train_bind", h, Pn, Pn, 1)


def test_bench_size_step_vs_oracle():
    """BASELINE configs[4] at the bench's size: full-depth towers, B = 256 images with precomputed
    text-token embeddings [256, 77, 768] + mask (bench.py --workload sparc), one engine step against
    the f32 autograd restatement of the heads + SparcLoss on the engine's own tower tokens (dropout
    off here; the masks are checked at 16 samples above)."""
    from oracle.sparc_train_torch import TorchSparcTrainStep
    cfg = get_model_config("ViT-L-14-336")
    m = _model(sparc, cfg, W.synthetic_state_dict(cfg))
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    B, T = 256, 77
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000)).cuda()
    gen = torch.Generator(device="cpu").manual_seed(3000)
    l_tok = (torch.randn(B, T, 768, generator=gen) * 0.5).cuda()
    eot = torch.randint(6, 42, (B,), generator=gen)
    mask = (torch.arange(T)[None, :] <= eot[:, None]).float().cuda()
    loss = float(tr.compute_grads(imgs, l_token_embed=l_tok, language_mask=mask))
    _, pt = m.clip_model.encode_image(imgs)
    step = TorchSparcTrainStep({n: v.detach() for n, v in tr.views.items()}, device="cuda")
    ref_loss, ref_grads, _ = step.loss_and_grads(pt, mask, l_token_embed=l_tok, p=0.0)
    _vs_oracle(tr, ref_loss, ref_grads, loss, skip=[n for n in HEAD_TENSORS if n.startswith("text_projection")])


def test_trainer_argument_errors(cfg, sd):
    """SparcHeadTrainer's host checks: exactly one text input; a mask with token embeddings; sparc
    models only."""
    m = _model(sparc, cfg, sd)
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1)).cuda()
    caps = torch.from_numpy(W.synthetic_captions(2, seed=2)).cuda()
    l_tok = torch.zeros(2, 77, 768, device="cuda")
    with pytest.raises(ValueError, match="one of them"):
        tr.compute_grads(imgs)
    with pytest.raises(ValueError, match="one of them"):
        tr.compute_grads(imgs, caps, l_token_embed=l_tok)
    with pytest.raises(ValueError, match="language_mask is required"):
        tr.compute_grads(imgs, l_token_embed=l_tok)
    with pytest.raises(TypeError, match="sparc"):
        clipembed.SparcHeadTrainer(m.clip_model)


@pytest.mark.parametrize("T", [1, 8])
def test_few_tokens_vs_oracle(b16, T):
    """Token counts below 28 (T x T < the head width): the backward's per-sample mean gradients have
    buffers of their own (they once shared the [B, T, T] local-loss scratch, which overflowed there);
    precomputed token embeddings with a ragged mask vs the oracle."""
    from oracle.sparc_train_torch import TorchSparcTrainStep
    m = b16["m"]
    tr = clipembed.SparcHeadTrainer(m, lr=1e-4, dropout=0.0)
    gen = torch.Generator(device="cpu").manual_seed(40 + T)
    l_tok = (torch.randn(16, T, 768, generator=gen) * 0.5).cuda()
    mask = torch.ones(16, T, device="cuda")
    if T > 1:
        mask[::2, T // 2:] = 0.0
    loss = float(tr.compute_grads(b16["imgs"], l_token_embed=l_tok, language_mask=mask))
    step = TorchSparcTrainStep({n: v.detach() for n, v in tr.views.items()}, device="cuda")
    pv = clipembed.pacl.apply_rope(b16["pt"], engine=m.engine)
    ref_loss, ref_grads, _ = step.loss_and_grads(pv, mask, l_token_embed=l_tok, p=0.0)
    _vs_oracle(tr, ref_loss, ref_grads, loss, skip=[n for n in HEAD_TENSORS if n.startswith("text_projection")])
