"""Parity of the exact kernel paths the benchmark configuration runs (BASELINE configs[1], batch 256).

At B = 256 the engine's default policy selects GEMM instantiations that small-batch tests never
reach: the vision QKV GEMM on the four-wave persistent schedule with the LN-fold epilogue (grids of
>= 4 tiles per CU), and the split-K tail + fixup with the LN-statistics epilogue on the out-proj /
c_proj GEMMs (grids just over a whole number of rounds).  These tests run them at the bench's own
shapes, assert through ce_gemm_path_counts that those paths fired, and check them against
  * a torch f32 reference of the same op (kernel level, M = 256 * 577 = 147,712), and
  * the golden reference outputs (tests/golden/clip_full.npz, open_clip f32 CPU forward) with the
    golden images / captions placed at batch rows 0 and 255 of a 256 batch, and
  * the same batch run with the plain path (auto schedule, split-K and LN fold all off).
Tolerances: 1e-3 cosine distance vs the f32 reference (north_star), 2e-4 between the two GPU paths
(both bf16; they differ only in summation order and the folded LayerNorm algebra)."""
import ctypes

import numpy as np
import pytest
import torch

import clipembed
from clipembed import _lib, weights as W
from clipembed.config import get_model_config

pytestmark = pytest.mark.gpu

DEV = "cuda"
M_BENCH = 256 * 577
ROWS_V = [0, 1, 23, 24, 287, 300, 551, 575]
COS_TOL = 1e-3
PATH_TOL = 2e-4
# ce_gemm_path_counts indices (include/clipembed.h)
W4PP, NT, FIXUP, W2 = 0, 3, 6, 10
PLAIN, STATS, FOLD = 0, 1, 2


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def path_counts(reset=True):
    c = (ctypes.c_int64 * 13)()
    _lib.call("ce_gemm_path_counts", c, 13, 1 if reset else 0)
    return list(c)


def cos_dist(a, b):
    a = np.asarray(a, np.float64).reshape(-1, a.shape[-1])
    b = np.asarray(b, np.float64).reshape(-1, b.shape[-1])
    c = (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    return float((1 - c).max())


def _operands(M, N, K, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    Wt = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    return g, A, Wt, bias


@pytest.mark.parametrize("N,act,expect", [(3072, 0, W4PP + FOLD), (4096, 1, W4PP + FOLD)])
def test_ln_fold_epilogue_at_bench_shape(N, act, expect):
    """QKV (N = 3072, no activation) and c_fc (N = 4096, GELU), both on SCHED 11, with the LN-fold
    epilogue: out = act(rstd_m (A W^T - mu_m c_n) + d_n), vs torch f32."""
    M, K = M_BENCH, 1024
    g, A, Wt, bias = _operands(M, N, K, 11 + N)
    mu = (torch.randn(M, generator=g) * 0.2).to(DEV)
    rstd = (torch.rand(M, generator=g) * 1.5 + 0.5).to(DEV)
    stats = torch.stack([mu, rstd], 1).contiguous()
    fold_c = Wt.float().sum(1).contiguous()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    path_counts()
    prev = _lib.lib().ce_set_gemm_schedule(1)
    try:
        _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(Wt), M, N, K, P(bias), act, None, P(out), _lib.CE_BF16,
                  FOLD, None, None, P(stats), P(fold_c))
        torch.cuda.synchronize()
    finally:
        _lib.lib().ce_set_gemm_schedule(prev)
    cnt = path_counts()
    # (plus, on SCHED 11, the split-K tail's fixup when the last round is short)
    assert cnt[expect] == 1 and sum(cnt) - cnt[FIXUP + FOLD] == 1 and cnt[FIXUP + FOLD] <= 1, cnt
    ref = rstd[:, None] * (A.float() @ Wt.float().t() - mu[:, None] * fold_c[None, :]) + bias
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 8e-3 * scale + 1e-5, f"max err {err} vs scale {scale}"


@pytest.mark.parametrize("K", [1024, 4096])
def test_ln_stats_epilogue_at_bench_shape(K):
    """out-proj (K = 1024) and c_proj (K = 4096) shapes, N = 1024, with the LN-statistics epilogue:
    2308 tiles = 9 rounds + 4, so the last 4 tiles run as split-K chunks + the LN-stats fixup.
    Checks out (f32), xb = bf16(out), the 64-column slab (mean, M2) and the finalized (mu, rstd)
    against torch f32, and against the same launch with split-K off."""
    M, N = M_BENCH, 1024
    g, A, Wt, bias = _operands(M, N, K, 5 + K)
    resid = torch.randn(M, N, generator=g).to(DEV)
    ns = N // 64
    res = {}
    for split in (1, 0):
        prev = _lib.lib().ce_set_gemm_splitk(split)
        out = torch.empty(M, N, device=DEV)
        xb = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        part = torch.full((M, ns, 2), float("nan"), device=DEV)
        stats = torch.empty(M, 2, device=DEV)
        path_counts()
        try:
            _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(Wt), M, N, K, P(bias), 0, P(resid), P(out),
                      _lib.CE_F32, STATS, P(xb), P(part), None, None)
            _lib.call("ce_kernel_ln_stats_finalize", S(), P(stats), P(part), M, ns)
            torch.cuda.synchronize()
        finally:
            _lib.lib().ce_set_gemm_splitk(prev)
        cnt = path_counts()
        if split:
            assert cnt[NT + STATS] == 1 and cnt[FIXUP + STATS] == 1 and sum(cnt) == 2, cnt
        else:
            assert cnt[NT + STATS] == 1 and sum(cnt) == 1, cnt
        res[split] = (out, xb, part, stats)
    ref = A.float() @ Wt.float().t() + bias + resid
    scale = ref.abs().max().item()
    for split, (out, xb, part, stats) in res.items():
        assert (out - ref).abs().max().item() <= 2e-4 * scale + 1e-5
        assert torch.equal(xb, out.to(torch.bfloat16))
        assert not torch.isnan(part).any()
        sl = out.view(M, ns, 64)
        smean = sl.mean(-1)
        np.testing.assert_allclose(part[..., 0].cpu().numpy(), smean.cpu().numpy(), atol=1e-5 * scale)
        m2 = ((sl - smean[..., None]) ** 2).sum(-1)
        np.testing.assert_allclose(part[..., 1].cpu().numpy(), m2.cpu().numpy(), rtol=1e-4, atol=1e-4)
        mu = out.mean(-1)
        rstd = torch.rsqrt(out.var(-1, unbiased=False) + 1e-5)
        np.testing.assert_allclose(stats[:, 0].cpu().numpy(), mu.cpu().numpy(), atol=1e-5)
        np.testing.assert_allclose(stats[:, 1].cpu().numpy(), rstd.cpu().numpy(), rtol=1e-4)
    # the split tail tiles differ only in f32 summation order
    assert (res[1][0] - res[0][0]).abs().max().item() <= 1e-4 * scale


@pytest.fixture(scope="module")
def full_model():
    cfg = get_model_config("ViT-L-14-336")
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    return m.to(DEV)


def _bench_batch(golden):
    """256 synthetic pairs (the bench's generator) with the two golden pairs at rows 0 and 255."""
    g = golden("clip_full")
    imgs = W.synthetic_images(256, seed=1000)
    gi = W.synthetic_images(2, seed=1000)
    imgs[0], imgs[255] = gi[0], gi[1]
    caps = W.synthetic_captions(256, seed=2000)
    caps[0], caps[255] = g["captions"][0], g["captions"][1]
    return g, torch.from_numpy(imgs).to(DEV), torch.from_numpy(caps).to(DEV)


def test_batch256_full_depth_bench_path(full_model, golden):
    """The whole bench step's encoders at B = 256 on the default policy: golden rows within 1e-3
    cosine of the reference + identical top-1; the whole batch within 2e-4 of the plain path."""
    m = full_model
    g, imgs, caps = _bench_batch(golden)
    m.visual.output_tokens = True
    try:
        path_counts()
        pi, ti = m.encode_image(imgs)
        torch.cuda.synchronize()
        cnt = path_counts()
        # 24 QKV + 24 c_fc on SCHED 11 + LN fold; 24 out-proj + 23 c_proj with LN stats on the hi/lo
        # stream on the staged-residual four-wave kernel, each with a split-K tail (2308 tiles =
        # 9 x 256 + 4; the last c_proj writes the f32 stream: nothing consumes its stats)
        assert cnt[W4PP + FOLD] == 48, cnt
        assert cnt[NT + FOLD] == 0, cnt
        assert cnt[W4PP + STATS] == 47 and cnt[NT + STATS] == 0 and cnt[FIXUP + STATS] == 47, cnt
        pt = m.encode_text(caps)
        pi_n, ti_n, pt_n = pi.cpu().numpy(), ti.cpu().numpy(), pt.cpu().numpy()
        sel = [0, 255]
        assert cos_dist(pi_n[sel], g["image_pooled"]) < COS_TOL
        assert cos_dist(pt_n[sel], g["text_pooled"]) < COS_TOL
        assert cos_dist(ti_n[sel][:, ROWS_V], g["image_tokens_rows"]) < COS_TOL
        il, _ = m.logits(torch.nn.functional.normalize(pi[sel], dim=-1),
                         torch.nn.functional.normalize(pt[sel], dim=-1), 100.0)
        il = il.cpu().numpy()
        assert (il.argmax(1) == g["image_logits"].argmax(1)).all()
        assert (il.argmax(0) == g["image_logits"].argmax(0)).all()

        # the same batch on the plain path: 4-phase schedule only, no split-K tail, no LN fold
        L = _lib.lib()
        pa, ps = L.ce_set_gemm_auto(0), L.ce_set_gemm_splitk(0)
        pf = m.engine.set_ln_fold(False)
        try:
            path_counts()
            qi, qt_tok = m.encode_image(imgs)
            qt = m.encode_text(caps)
            torch.cuda.synchronize()
            cnt = path_counts()
            assert cnt[W4PP + FOLD] == 0 and cnt[FIXUP + STATS] == 0 and cnt[NT + FOLD] == 0, cnt
        finally:
            L.ce_set_gemm_auto(pa)
            L.ce_set_gemm_splitk(ps)
            m.engine.set_ln_fold(pf)
        assert cos_dist(pi_n, qi.cpu().numpy()) < PATH_TOL
        assert cos_dist(ti_n[:, ROWS_V], qt_tok.cpu().numpy()[:, ROWS_V]) < PATH_TOL
        assert cos_dist(pt_n, qt.cpu().numpy()) < PATH_TOL
        assert np.isfinite(ti_n).all()
    finally:
        m.visual.output_tokens = False


def test_batch256_pooled_prune(full_model, golden):
    """The bench's own calls (pooled features only): each tower's last block runs for the pooled
    rows alone (CLS / EOT; ce_set_pooled_prune).  Asserts the paths (23 c_fc on SCHED 11, the
    pruned B-row c_fc / out-proj on SCHED 1 with split-K over every tile) and checks the pooled outputs against the unpruned
    path (2e-5 cosine: the pruned attention keeps P in f32, the small GEMMs sum in another order)
    and the golden rows against the reference (1e-3)."""
    m = full_model
    g, imgs, caps = _bench_batch(golden)
    assert not m.visual.output_tokens and not m.output_text_tokens
    path_counts()
    pi = m.encode_image(imgs)
    torch.cuda.synchronize()
    cnt = path_counts()
    # (the pruned B-row GEMMs: 4 / 16 tiles, split-K over every tile + fixup)
    assert cnt[W4PP + FOLD] == 47 and cnt[NT + FOLD] == 1 and cnt[FIXUP + FOLD] == 1, cnt
    assert cnt[W4PP + STATS] == 46 and cnt[NT + STATS] == 1 and cnt[FIXUP + STATS] == 47, cnt
    pt = m.encode_text(caps)
    prev = m.engine.set_pooled_prune(False)
    try:
        assert prev
        qi = m.encode_image(imgs)
        qt = m.encode_text(caps)
    finally:
        m.engine.set_pooled_prune(prev)
    pi_n, pt_n = pi.cpu().numpy(), pt.cpu().numpy()
    d_img, d_txt = cos_dist(pi_n, qi.cpu().numpy()), cos_dist(pt_n, qt.cpu().numpy())
    print(f"pruned vs full: image {d_img:.3g} text {d_txt:.3g}")
    assert d_img < 2e-5 and d_txt < 2e-5
    sel = [0, 255]
    assert cos_dist(pi_n[sel], g["image_pooled"]) < COS_TOL
    assert cos_dist(pt_n[sel], g["text_pooled"]) < COS_TOL


@pytest.mark.parametrize("tag", ["pacl", "pacl_rope_after"])
def test_pacl_batch512_golden_rows(golden, tag):
    """PACL forward at the C3 batch (512 pairs, BASELINE configs[2]) with the two golden pairs of
    tests/golden/pacl.npz at rows 0 and 511 (2-block towers as in the fixture): those rows within
    1e-3 cosine of the reference's open_clip_pacl outputs; every row finite and unit-norm."""
    from clipembed.pacl import open_clip_pacl, open_clip_pacl_rope_after
    cls = {"pacl": open_clip_pacl, "pacl_rope_after": open_clip_pacl_rope_after}[tag]
    cfg = get_model_config("ViT-L-14-336").with_depth(2, 2)
    g = golden("pacl")
    mod = cls(cfg=cfg, clip_state_dict=W.synthetic_state_dict(cfg))
    mod.load_state_dict(W.synthetic_pacl_heads(cfg.with_pacl(768)))
    mod.to(DEV)
    imgs = W.synthetic_images(512, seed=1200)
    gi = W.synthetic_images(2, seed=1100)
    imgs[0], imgs[511] = gi[0], gi[1]
    caps = W.synthetic_captions(512, seed=2200)
    caps[0], caps[511] = g["captions"][0], g["captions"][1]
    path_counts()
    a, b = mod(torch.from_numpy(imgs).to(DEV), torch.from_numpy(caps).to(DEV))
    torch.cuda.synchronize()
    cnt = path_counts()
    # the big-grid paths ran: QKV + c_fc of the 2 image and the 2 text blocks (both towers folded;
    # text M = 512 x 77 = 39,424 rows is >= 4 tiles per CU too) on the four-wave kernel
    assert cnt[W4PP + FOLD] == 8 and cnt[W4PP + STATS] >= 1, cnt
    a, b = a.cpu().numpy(), b.cpu().numpy()
    assert cos_dist(a[[0, 511]], g[f"{tag}_img"]) < COS_TOL
    assert cos_dist(b[[0, 511]], g[f"{tag}_txt"]) < COS_TOL
    assert np.isfinite(a).all() and np.isfinite(b).all()
    np.testing.assert_allclose(np.linalg.norm(a, axis=-1), 1.0, rtol=1e-4)


@pytest.mark.parametrize("rows,ns", [(147712, 16), (19713, 12), (1000, 9), (65, 16), (3, 2)])
def test_ln_stats_finalize_kernels(rows, ns):
    """(mu, rstd) from 64-column slab (mean, M2) partials: the two-row 16-B-load kernel (even ns <= 16:
    D = 1024 / 768) and the 16-lane kernel (odd ns), ragged row counts, vs torch f32 from the same
    partials (Chan's combine of equal-count slabs)."""
    g = torch.Generator(device="cpu").manual_seed(rows + ns)
    x = (torch.randn(rows, ns, 64, generator=g) * torch.rand(rows, 1, 1, generator=g) * 3 + 0.5).to(DEV)
    part = torch.stack([x.mean(-1), ((x - x.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).contiguous()
    stats = torch.full((rows + 8, 2), 7.0, device=DEV)
    _lib.call("ce_kernel_ln_stats_finalize", S(), P(stats), P(part), rows, ns)
    torch.cuda.synchronize()
    xf = x.reshape(rows, ns * 64)
    mu = xf.mean(-1)
    rstd = torch.rsqrt(xf.var(-1, unbiased=False) + 1e-5)
    np.testing.assert_allclose(stats[:rows, 0].cpu().numpy(), mu.cpu().numpy(), atol=1e-5)
    np.testing.assert_allclose(stats[:rows, 1].cpu().numpy(), rstd.cpu().numpy(), rtol=1e-4)
    assert bool((stats[rows:] == 7.0).all())
