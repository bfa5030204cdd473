"""Kernel-level numerics of the HIP kernels against plain PyTorch fp32 references of the same op,
called through the C ABI's kernel entry points (include/clipembed.h, ce_kernel_*)."""
import ctypes

import pytest
import torch

from clipembed import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda"


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def path_counts():
    """ce_gemm_path_counts, reset after reading (indices: include/clipembed.h)."""
    c = (ctypes.c_int64 * 13)()
    _lib.call("ce_gemm_path_counts", c, 13, 1)
    return list(c)


def gemm_ref(A, W, bias, act, resid):
    y = A.float() @ W.float().t()
    if bias is not None:
        y = y + bias
    if act == 1:
        y = torch.nn.functional.gelu(y)
    elif act == 2:
        y = y * torch.sigmoid(1.702 * y)
    if resid is not None:
        y = y + resid
    return y


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 512, 1024), (4617, 3072, 1024), (1154, 1024, 4096),
                                   (231, 2304, 768), (5, 768, 1024), (700, 832, 640), (1, 64, 64)])
@pytest.mark.parametrize("variant", ["bias_bf16", "gelu_bf16", "qgelu_bf16", "resid_f32", "plain_f32"])
@pytest.mark.parametrize("sched", [1, 11])
def test_gemm(M, N, K, variant, sched):
    prev = _lib.lib().ce_set_gemm_schedule(sched)
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 3 + K)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV) if variant != "plain_f32" else None
    resid = torch.randn(M, N, generator=g).to(DEV) if variant == "resid_f32" else None
    act = {"gelu_bf16": 1, "qgelu_bf16": 2}.get(variant, 0)
    out_bf16 = variant.endswith("bf16")
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16 if out_bf16 else torch.float32)
    _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, P(bias), act, P(resid), P(out),
              _lib.CE_BF16 if out_bf16 else _lib.CE_F32)
    torch.cuda.synchronize()
    _lib.lib().ce_set_gemm_schedule(prev)
    ref = gemm_ref(A, W, bias, act, resid)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    tol = (8e-3 if out_bf16 else 2e-4) * scale + 1e-5   # bf16 output rounding / f32 accumulation order
    assert err <= tol, f"max err {err} vs tol {tol}"


@pytest.mark.parametrize("M,N,K", [(66560, 256, 1024), (66460, 512, 512), (33280, 1024, 4096)])
@pytest.mark.parametrize("variant", ["gelu_bf16", "resid_f32", "bias_bf16"])
def test_gemm_splitk_tail(M, N, K, variant):
    """Grids of 256 * rounds + a few tiles: the last tiles run as K-chunks + a fixup launch.  Checked
    against the f32 reference and against the same launch with the split disabled."""
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    resid = torch.randn(M, N, generator=g).to(DEV) if variant == "resid_f32" else None
    act = 1 if variant == "gelu_bf16" else 0
    out_bf16 = variant.endswith("bf16")
    outs = []
    for split in (1, 0):
        prev = _lib.lib().ce_set_gemm_splitk(split)
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16 if out_bf16 else torch.float32)
        _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, P(bias), act, P(resid), P(out),
                  _lib.CE_BF16 if out_bf16 else _lib.CE_F32)
        torch.cuda.synchronize()
        _lib.lib().ce_set_gemm_splitk(prev)
        outs.append(out.float())
    ref = A.float() @ W.float().t() + bias
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    if resid is not None:
        ref = ref + resid
    tol = (2e-2 if out_bf16 else 2e-3) * max(1.0, ref.abs().max().item())
    for o in outs:
        assert (o - ref).abs().max().item() < tol
    # the two paths differ only in the summation order of the tail tiles
    assert (outs[0] - outs[1]).abs().max().item() < tol


@pytest.mark.parametrize("M,N,K", [(33280, 1024, 1024), (20000, 3072, 1024), (17000, 1024, 4096)])
@pytest.mark.parametrize("variant", ["gelu_bf16", "resid_f32", "bias_bf16"])
@pytest.mark.parametrize("bits", [0, 1, 3, 19, 35])
def test_gemm_persistent_multitile(M, N, K, variant, bits):
    """The four-wave persistent schedule (SCHED 11) with several tiles per workgroup, so the
    epilogue -> next-tile hand-over (and its variant bits: 1 no drain, 2 the four-wave epilogues,
    16 one tile per workgroup, 32 split-K tail) runs; vs the f32 reference.  The f32 residual
    epilogue (and every GEMM with bit 1 off) takes SCHED 1."""
    L = _lib.lib()
    prev, prev_v = L.ce_set_gemm_schedule(11), L.ce_set_gemm_variant(bits)
    try:
        g = torch.Generator(device="cpu").manual_seed(M + N + K + bits)
        A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
        W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
        bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
        resid = torch.randn(M, N, generator=g).to(DEV) if variant == "resid_f32" else None
        act = 1 if variant == "gelu_bf16" else 0
        out_bf16 = variant.endswith("bf16")
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16 if out_bf16 else torch.float32)
        _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, P(bias), act, P(resid), P(out),
                  _lib.CE_BF16 if out_bf16 else _lib.CE_F32)
        torch.cuda.synchronize()
    finally:
        L.ce_set_gemm_schedule(prev)
        L.ce_set_gemm_variant(prev_v)
    ref = gemm_ref(A, W, bias, act, resid)
    err = (out.float() - ref).abs().max().item()
    tol = (8e-3 if out_bf16 else 2e-4) * ref.abs().max().item() + 1e-5
    assert err <= tol, f"max err {err} vs tol {tol}"


@pytest.mark.parametrize("M,N,act", [(20000, 3072, 0), (20000, 4096, 1), (20000, 4096, 2), (300, 1024, 1),
                                     (5602, 3072, 0), (4252, 4096, 1)])
@pytest.mark.parametrize("bits", [1, 3, 19, 35])
def test_gemm_persistent_ln_fold(M, N, act, bits):
    """SCHED 11 with the LN-fold epilogue (QKV / c_fc of the folded image tower; bit 1 off: SCHED 1),
    one tile per workgroup (bit 4) and the split-K tail (bit 5; 5602 x 3072 = 256 + 8 tiles,
    4252 x 4096 = 256 + 16 tiles):
    out = act(rstd_m (A W^T - mu_m c_n) + d_n) vs torch f32; M % 256 != 0 exercises the row clip."""
    K = 1024
    L = _lib.lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + act + bits)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    mu = (torch.randn(M, generator=g) * 0.2).to(DEV)
    rstd = (torch.rand(M, generator=g) * 1.5 + 0.5).to(DEV)
    stats = torch.stack([mu, rstd], 1).contiguous()
    fold_c = W.float().sum(1).contiguous()
    out = torch.full((M + 64, N), 7.0, device=DEV, dtype=torch.bfloat16)   # rows >= M must stay untouched
    prev, prev_v = L.ce_set_gemm_schedule(11), L.ce_set_gemm_variant(bits)
    try:
        _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), act, None, P(out), _lib.CE_BF16,
                  2, None, None, P(stats), P(fold_c))
        torch.cuda.synchronize()
    finally:
        L.ce_set_gemm_schedule(prev)
        L.ce_set_gemm_variant(prev_v)
    ref = rstd[:, None] * (A.float() @ W.float().t() - mu[:, None] * fold_c[None, :]) + bias
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    elif act == 2:
        ref = ref * torch.sigmoid(1.702 * ref)
    err = (out[:M].float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item() + 1e-5, err
    assert bool((out[M:] == 7.0).all())


@pytest.mark.parametrize("M,K", [(20000, 1024), (9000, 4096), (300, 1024)])
@pytest.mark.parametrize("bits", [1, 3, 19])
def test_gemm_persistent_ln_stats(M, K, bits):
    """SCHED 11 with the LN-statistics epilogue (the f32-stream out-proj / c_proj; bit 1 off: SCHED 1),
    one tile per workgroup (bit 4): out f32 = A W^T + bias + resid, xb = bf16(out), per-64-column (mean, M2)
    slab statistics, vs torch f32; rows >= M of every output stay untouched."""
    N = 1024
    L = _lib.lib()
    g = torch.Generator(device="cpu").manual_seed(M + K + bits)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    resid = torch.randn(M, N, generator=g).to(DEV)
    ns = N // 64
    out = torch.full((M + 32, N), 7.0, device=DEV)
    xb = torch.full((M + 32, N), 7.0, device=DEV, dtype=torch.bfloat16)
    part = torch.full((M + 32, ns, 2), 7.0, device=DEV)
    prev, prev_v = L.ce_set_gemm_schedule(11), L.ce_set_gemm_variant(bits)
    try:
        _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), 0, P(resid), P(out), _lib.CE_F32,
                  1, P(xb), P(part), None, None)
        torch.cuda.synchronize()
    finally:
        L.ce_set_gemm_schedule(prev)
        L.ce_set_gemm_variant(prev_v)
    ref = A.float() @ W.float().t() + bias + resid
    scale = ref.abs().max().item()
    assert (out[:M] - ref).abs().max().item() <= 2e-4 * scale + 1e-5
    assert (xb[:M].float() - ref).abs().max().item() <= 8e-3 * scale
    r3 = ref.reshape(M, ns, 64)
    mean = r3.mean(-1)
    m2 = ((r3 - mean[..., None]) ** 2).sum(-1)
    assert (part[:M, :, 0] - mean).abs().max().item() <= 1e-4 * scale
    assert (part[:M, :, 1] - m2).abs().max().item() <= 1e-4 * m2.abs().max().item() + 1e-4
    assert bool((out[M:] == 7.0).all()) and bool((xb[M:] == 7.0).all()) and bool((part[M:] == 7.0).all())


@pytest.mark.parametrize("M,K,N,rhl", [(147712, 1024, 1024, 0), (147712, 4096, 1024, 0), (300, 1024, 1024, 0),
                                       (5000, 1024, 1024, 0), (147712, 1024, 1024, 1), (147712, 4096, 1024, 1),
                                       (140001, 1024, 1024, 1), (131072, 192, 768, 1), (70000, 128, 1536, 1)])
def test_gemm_ln_stats_hl(M, K, N, rhl):
    """The hi/lo residual-stream epilogues (SCHED 1, split-K tail at the bench shapes M = 256 * 577;
    rhl: epi 3 on the staged-residual four-wave kernel, variant bit 128, incl. a ragged last row
    tile, K = 2 and 3 K-tiles and N = 768 / 1536): epi 3 reads resid = hi + lo and writes
    v = A W^T + b + resid as planes hi = bf16(v), lo = bf16(v - hi) plus the slab statistics; epi 4
    writes v in f32.  vs torch f32: hi is the round-to-nearest bf16 of v, hi + lo within 2^-16 |v| of
    v (f32 accumulation order aside)."""
    L = _lib.lib()
    g = torch.Generator(device="cpu").manual_seed(M + K)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    x = torch.randn(M, N, generator=g).to(DEV)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    planes = torch.stack([hi, lo]).contiguous()
    ref = A.float() @ W.float().t() + bias + (hi.float() + lo.float())
    ns = N // 64
    outp = torch.full((2, M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    part = torch.full((M, ns, 2), 7.0, device=DEV)
    prev_v = L.ce_set_gemm_variant(-1)
    L.ce_set_gemm_variant((prev_v & ~128) | (128 if rhl else 0))
    try:
        path_counts()
        _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), 0, P(planes), None, _lib.CE_F32,
                  3, P(outp), P(part), None, None)
        cnt = path_counts()
    finally:
        L.ce_set_gemm_variant(prev_v)
    assert cnt[0 + 1] == (1 if rhl else 0) and cnt[3 + 1] == (0 if rhl else 1), cnt     # W4PP / NT + LN stats
    if rhl:      # split-K tail of a last round of <= 32 tiles (M = 147,712: 2308 = 9 x 256 + 4)
        nwg = -(-M // 256) * (N // 256)
        assert cnt[6 + 1] == (1 if 0 < nwg % 256 <= 32 else 0), cnt
    out4 = torch.empty(M, N, device=DEV)
    _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), 0, P(planes), P(out4), _lib.CE_F32,
              4, None, None, None, None)
    torch.cuda.synchronize()
    scale = ref.abs().max().item()
    assert (out4 - ref).abs().max().item() <= 2e-4 * scale + 1e-5
    v = outp[0].float() + outp[1].float()
    assert (v - ref).abs().max().item() <= 2e-4 * scale + 1e-5
    assert (v - out4).abs().max().item() <= 2 ** -16 * scale
    assert torch.equal(outp[0], v.to(torch.bfloat16)) or (outp[0].float() - v).abs().max().item() <= 2 ** -8 * scale
    r3 = ref.reshape(M, ns, 64)
    mean = r3.mean(-1)
    m2 = ((r3 - mean[..., None]) ** 2).sum(-1)
    assert (part[:, :, 0] - mean).abs().max().item() <= 1e-4 * scale
    assert (part[:, :, 1] - m2).abs().max().item() <= 1e-4 * m2.abs().max().item() + 1e-4


def test_gemm_identity_asymmetric():
    """A = I with an asymmetric W catches a transposed C-write (guide §3)."""
    n = 256
    A = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    W = (torch.arange(n * n, device=DEV, dtype=torch.float32).reshape(n, n) % 97 - 48).to(torch.bfloat16)
    out = torch.empty(n, n, device=DEV, dtype=torch.float32)
    _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), n, n, n, None, 0, None, P(out), _lib.CE_F32)
    torch.cuda.synchronize()
    assert torch.equal(out, W.float().t())


QSCALE = 0.125 * 1.4426950408889634      # kAttnQScale: log2(e) / sqrt(64), ce_kernels.h


def attn_ref(qkv, B, L, H, causal):
    """softmax(q k^T / 8) v in f32 with the kernel's one input rounding applied: the kernel scores
    in log2 units from q pre-multiplied by log2(e)/8 and rounded to bf16 (in the engine that
    product is the in_proj q rows), so the reference uses the same bf16(q * QSCALE)."""
    D = H * 64
    x = qkv.float().reshape(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    q = (q * QSCALE).to(torch.bfloat16).float()
    s = (q @ k.transpose(-1, -2)) * (1.0 / 1.4426950408889634)
    if causal:
        s = s + torch.triu(torch.full((L, L), float("-inf"), device=qkv.device), 1)
    p = s.softmax(-1)
    return (p @ v).permute(0, 2, 1, 3).reshape(B * L, D)


@pytest.fixture(params=[125, 381], ids=lambda v: f"attn_var{v}")
def attn_var(request):
    """Both attention forward variants (ce_set_attn_variant) against torch f32 (causal
    launches run the general-path kernel under either)."""
    prev = _lib.lib().ce_set_attn_variant(request.param)
    yield request.param
    _lib.lib().ce_set_attn_variant(prev)


def run_attn(qkv, B, L, H, causal):
    out = torch.empty(B * L, H * 64, device=DEV, dtype=torch.bfloat16)
    _lib.call("ce_kernel_attention", S(), P(qkv), P(out), B, L, H, 1 if causal else 0)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("B,L,H,causal", [(2, 577, 16, False), (3, 77, 12, True), (1, 1, 16, False),
                                          (2, 64, 4, False), (2, 65, 4, True), (1, 129, 2, False),
                                          (1, 300, 12, True), (5, 577, 1, False), (1, 257, 2, False),
                                          (2, 289, 3, False), (1, 97, 2, False)])
def test_attention(B, L, H, causal, attn_var):
    g = torch.Generator(device="cpu").manual_seed(B * 1000 + L + H)
    qkv = (torch.randn(B * L, 3 * H * 64, generator=g) * 1.5).to(torch.bfloat16).to(DEV)
    out = run_attn(qkv, B, L, H, causal)
    ref = attn_ref(qkv, B, L, H, causal)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


def test_attention_spike_rescale(attn_var):
    """Force the online-softmax rescale: a late key dominates one query (guide §5.4 rule 26).  On
    the fixed-offset variants the score (~184 in log2 units) overflows the fast tile's check, so
    the tile is redone with the exact max and the wave returns to the general path."""
    B, L, H = 1, 577, 2
    g = torch.Generator(device="cpu").manual_seed(3)
    qkv = torch.randn(B * L, 3 * H * 64, generator=g) * 0.5
    D = H * 64
    qkv[10, 0:64] = 4.0                 # query 10, head 0
    qkv[500, D:D + 64] = 4.0            # key 500 -> huge score for query 10 at the 8th key tile
    qkv = qkv.to(torch.bfloat16).to(DEV)
    out = run_attn(qkv, B, L, H, False)
    ref = attn_ref(qkv, B, L, H, False)
    assert (out.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("key", [3, 100, 576])
def test_attention_spike_positions(key, attn_var):
    """A dominant key in tile 0 (row max > 64: the wave never takes the fixed offset), inside a
    fast tile (overflow redo), and the single-key last tile (general path with a fixed offset)."""
    B, L, H = 2, 577, 2
    g = torch.Generator(device="cpu").manual_seed(key)
    qkv = torch.randn(B * L, 3 * H * 64, generator=g) * 0.5
    D = H * 64
    for q in (5, 200, 570):
        qkv[q, 0:64] = 4.0
    qkv[L + 7, 64:128] = -4.0
    qkv[key, D:D + 64] = 4.0
    qkv[L + key, D + 64:D + 128] = -4.0
    qkv = qkv.to(torch.bfloat16).to(DEV)
    out = run_attn(qkv, B, L, H, False)
    ref = attn_ref(qkv, B, L, H, False)
    assert (out.float() - ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("scale", [3.0, 4.5])
def test_attention_wide_scores(scale, attn_var):
    """Scores spread over tens of log2 units (p up to ~2^60 on the fixed offset, no overflow), and
    beyond (scale 4.5: some rows overflow the check)."""
    B, L, H = 2, 577, 4
    g = torch.Generator(device="cpu").manual_seed(int(scale * 10))
    qkv = (torch.randn(B * L, 3 * H * 64, generator=g) * scale).to(torch.bfloat16).to(DEV)
    out = run_attn(qkv, B, L, H, False)
    ref = attn_ref(qkv, B, L, H, False)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err
    prev = _lib.lib().ce_set_attn_variant(125 if attn_var == 381 else 381)
    try:
        base = run_attn(qkv, B, L, H, False)
    finally:
        _lib.lib().ce_set_attn_variant(prev)
    err0 = (out.float() - base.float()).abs().max().item()
    assert err0 < 2e-2 * max(1.0, ref.abs().max().item()), err0


def attn_ref_f32(qkv, B, L, H, causal):
    """softmax(q k^T / 8) v in plain f32 on the bf16 inputs, no kernel rounding restated."""
    x = qkv.float().reshape(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = (x[0] @ x[1].transpose(-1, -2)) / 8.0
    if causal:
        s = s + torch.triu(torch.full((L, L), float("-inf"), device=qkv.device), 1)
    return (s.softmax(-1) @ x[2]).permute(0, 2, 1, 3).reshape(B * L, H * 64)


@pytest.mark.parametrize("scale,causal", [(3.0, False), (4.5, False), (3.0, True)])
def test_attention_wide_scores_vs_unrounded_f32(scale, causal):
    """The default kernel against attention in f32 WITHOUT the kernel's bf16(q * log2(e)/8) input
    rounding (attn_ref restates it): bounds that rounding's effect at kernel level, on score spreads
    of tens of log2 units (the bound of the rounding-free reference before it was restated)."""
    B, L, H = 2, (577 if not causal else 77), 4
    g = torch.Generator(device="cpu").manual_seed(int(scale * 10) + causal)
    qkv = (torch.randn(B * L, 3 * H * 64, generator=g) * scale).to(torch.bfloat16).to(DEV)
    out = run_attn(qkv, B, L, H, causal)
    ref = attn_ref_f32(qkv, B, L, H, causal)
    err = (out.float() - ref).abs().max().item()
    assert err < 6e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("rows,D,bf16", [(1000, 1024, True), (1000, 1024, False), (77, 768, True), (3, 768, False)])
def test_layernorm(rows, D, bf16):
    g = torch.Generator(device="cpu").manual_seed(rows + D)
    x = (torch.randn(rows, D, generator=g) * 3 + 1).to(DEV)
    w = (1 + 0.1 * torch.randn(D, generator=g)).to(DEV)
    b = (0.1 * torch.randn(D, generator=g)).to(DEV)
    out = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16 if bf16 else torch.float32)
    _lib.call("ce_kernel_layernorm", S(), P(x), P(out), _lib.CE_BF16 if bf16 else _lib.CE_F32, P(w), P(b), rows, D)
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x, (D,), w, b, 1e-5)
    err = (out.float() - ref).abs().max().item()
    assert err < (3e-2 if bf16 else 1e-4), err


@pytest.mark.parametrize("var", [381])
@pytest.mark.parametrize("s0", [6.0, -6.0, 0.0])
@pytest.mark.parametrize("L", [577, 65, 129])
def test_attention_cls_key_first(L, s0, var):
    """Variant 381 (key 0 folded in before the key tiles, tiles over keys 1..L-1) with key 0 dominant
    (s0 = +6: every query's score with it ~ +6 * 64 * 4 -> far past the fixed offset's +-64), far below
    (-6) and ordinary: vs f32 attention and vs the default variant."""
    B, H = 2, 4
    g = torch.Generator(device="cpu").manual_seed(L + int(s0 * 10))
    qkv = torch.randn(B * L, 3 * H * 64, generator=g) * 0.8
    D = H * 64
    if s0 != 0.0:
        for b in range(B):
            qkv[b * L:(b + 1) * L, 0:64] = qkv[b * L:(b + 1) * L, 0:64].abs() * 0 + 1.0   # head 0 queries
            qkv[b * L, D:D + 64] = s0                                                        # key 0, head 0
    qkv = qkv.to(torch.bfloat16).to(DEV)
    ref = attn_ref(qkv, B, L, H, False)
    prev = _lib.lib().ce_set_attn_variant(var)
    try:
        out = run_attn(qkv, B, L, H, False)
    finally:
        _lib.lib().ce_set_attn_variant(prev)
    base = run_attn(qkv, B, L, H, False)
    scale = max(1.0, ref.abs().max().item())
    assert (out.float() - ref).abs().max().item() < 2e-2 * scale
    assert (out.float() - base.float()).abs().max().item() < 2e-2 * scale
