"""SCHED 14 (gemm_w2b, csrc/gemm_w2b.hip): two independent 256 x 128-tile workgroups per CU.  Checked
against plain PyTorch f32 references of the same op (bias / GELU / QuickGELU, null bias, LN-folded
consumer), with a ragged last M tile, the shortest K (2 K-steps: the prologue's two in flight), step
counts 4, 6 and 10 (the 3-slot ring and the 6-step unroll's tails), K = 4096, grids below the CU count; rows
past M must stay untouched; and against SCHED 11 on the QKV shape."""
import ctypes

import pytest
import torch

from clipembed import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
W2 = 10          # ce_gemm_path_counts: the two-workgroup kernels (SCHED 12 / 14), + epi


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def path_counts():
    c = (ctypes.c_int64 * 13)()
    _lib.call("ce_gemm_path_counts", c, 13, 1)
    return list(c)


def run14(fn):
    L = _lib.lib()
    prev = L.ce_set_gemm_schedule(14)
    try:
        path_counts()
        fn()
        torch.cuda.synchronize()
        return path_counts()
    finally:
        L.ce_set_gemm_schedule(prev)


def _ref_act(ref, act):
    if act == 1:
        return torch.nn.functional.gelu(ref)
    if act == 2:
        return ref * torch.sigmoid(1.702 * ref)
    return ref


SHAPES = [(20000, 3072, 1024), (2308, 4096, 1024), (17000, 1024, 4096), (300, 1024, 1024), (5, 768, 1024),
          (1000, 256, 64), (700, 128, 128), (4100, 512, 192), (300, 384, 320)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_w2b_bias_act(M, N, K, act):
    g = torch.Generator(device="cpu").manual_seed(M + N + K + act)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    out = torch.full((M + 64, N), 7.0, device=DEV, dtype=torch.bfloat16)
    cnt = run14(lambda: _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, P(bias), act, None, P(out),
                                  _lib.CE_BF16))
    assert cnt[W2] == 1, cnt
    ref = _ref_act(A.float() @ W.float().t() + bias, act)
    err = (out[:M].float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item() + 1e-5, err
    assert bool((out[M:] == 7.0).all())


def test_gemm_w2b_null_bias():
    M, N, K = 3000, 1024, 512
    g = torch.Generator(device="cpu").manual_seed(3)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    cnt = run14(lambda: _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, None, 0, None, P(out),
                                  _lib.CE_BF16))
    assert cnt[W2] == 1, cnt
    ref = A.float() @ W.float().t()
    assert (out.float() - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()


@pytest.mark.parametrize("M,N", [(20000, 3072), (20000, 4096), (4252, 4096), (300, 1024), (77, 2304)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_w2b_ln_fold(M, N, act):
    """out = act(rstd_m (A W^T - mu_m c_n) + d_n), the QKV / c_fc epilogue of the folded tower."""
    K = 1024
    g = torch.Generator(device="cpu").manual_seed(M + N + act + 13)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    mu = (torch.randn(M, generator=g) * 0.2).to(DEV)
    rstd = (torch.rand(M, generator=g) * 1.5 + 0.5).to(DEV)
    stats = torch.stack([mu, rstd], 1).contiguous()
    fold_c = W.float().sum(1).contiguous()
    out = torch.full((M + 64, N), 7.0, device=DEV, dtype=torch.bfloat16)
    cnt = run14(lambda: _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), act, None, P(out),
                                  _lib.CE_BF16, 2, None, None, P(stats), P(fold_c)))
    assert cnt[W2 + 2] == 1, cnt
    ref = _ref_act(rstd[:, None] * (A.float() @ W.float().t() - mu[:, None] * fold_c[None, :]) + bias, act)
    err = (out[:M].float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item() + 1e-5, err
    assert bool((out[M:] == 7.0).all())


def test_gemm_w2b_matches_sched11_and_is_deterministic():
    """Same inputs through SCHED 11 and SCHED 14 (QKV shape at B = 32): both f32-accumulate each
    output over K in the same order, so the bf16 outputs agree to the epilogue's rounding; two
    SCHED 14 launches are bitwise equal."""
    M, N, K = 32 * 577, 3072, 1024
    g = torch.Generator(device="cpu").manual_seed(5)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    outs = []
    L = _lib.lib()
    for sc in (11, 14, 14):
        prev = L.ce_set_gemm_schedule(sc)
        try:
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            _lib.call("ce_kernel_gemm_bf16", S(), P(A), P(W), M, N, K, P(bias), 1, None, P(out), _lib.CE_BF16)
            torch.cuda.synchronize()
            outs.append(out.float())
        finally:
            L.ce_set_gemm_schedule(prev)
    d = (outs[0] - outs[1]).abs().max().item()
    assert d <= 1e-2 * outs[0].abs().max().item(), d
    assert torch.equal(outs[1], outs[2])


@pytest.mark.parametrize("M,N,K", [(256 * 577, 1024, 1024), (256 * 577, 1024, 4096), (1000, 768, 1024), (77, 1536, 256),
                                   (5, 1024, 64)])
def test_gemm_w2b_ln_stats_hl(M, N, K):
    """The hi/lo residual-stream epilogue (epi 3: out-proj / c_proj of the folded towers) on SCHED 14:
    resid = hi + lo planes, v = A W^T + b + resid written as planes hi = bf16(v), lo = bf16(v - hi) plus
    per-64-column slab (mean, M2); vs torch f32 (hi + lo within 2^-16 |v| of the f32 value up to the
    accumulation order) and rows past M untouched."""
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    A = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    x = torch.randn(M, N, generator=g).to(DEV)
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    planes = torch.stack([hi, lo]).contiguous()
    ref = A.float() @ W.float().t() + bias + (hi.float() + lo.float())
    ns = N // 64
    outp = torch.full((2, M + 64, N), 7.0, device=DEV, dtype=torch.bfloat16)
    part = torch.full((M + 64, ns, 2), 7.0, device=DEV)
    # planes of M rows each: the output planes are written at xb and xb + M * N (hl_plane = M * N)
    outv = outp.view(-1)[: 2 * M * N].view(2, M, N)
    cnt = run14(lambda: _lib.call("ce_kernel_gemm_bf16_epi", S(), P(A), P(W), M, N, K, P(bias), 0, P(planes), None,
                                  _lib.CE_F32, 3, P(outv), P(part), None, None))
    assert cnt[W2 + 1] == 1, cnt
    scale = ref.abs().max().item()
    v = outv[0].float() + outv[1].float()
    assert (v - ref).abs().max().item() <= 2e-4 * scale + 1e-5
    assert (outv[0].float() - v).abs().max().item() <= 2 ** -8 * scale
    assert bool((outp.view(-1)[2 * M * N:] == 7.0).all())
    r3 = ref.reshape(M, ns, 64)
    mean = r3.mean(-1)
    m2 = ((r3 - mean[..., None]) ** 2).sum(-1)
    assert (part[:M, :, 0] - mean).abs().max().item() <= 1e-4 * scale
    assert (part[:M, :, 1] - m2).abs().max().item() <= 1e-4 * m2.abs().max().item() + 1e-4
    assert bool((part[M:] == 7.0).all())
