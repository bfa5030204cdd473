"""The MN-major weight-gradient GEMM (gemm_tn.hip, ce_kernel_gemm_tn_bf16) against a plain PyTorch
fp32 reference of the same product, C = diag(scale) A^T B, and the text-tower backward with it against
the transposed-copy path it replaces (autograd of transformer.py:228-239).

Tolerance: bf16 operands are exact in f32, products are exact, and the kernel accumulates in f32
(over split-K chunks summed in fixed order), so it differs from torch's f32 GEMM only by summation
order: |C - ref| <= 1e-5 * sum_k |A[k][m] B[k][n]| (K up to 118k) is asserted elementwise."""
import ctypes

import numpy as np
import pytest
import torch

from clipembed import _lib

pytestmark = pytest.mark.gpu

DEV = "cuda"


def P(t):
    return ctypes.c_void_p(t.data_ptr())


def S():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run_tn(A, B, M, N, K, scale_rows=0, scale=1.0, ldc=None):
    ldc = ldc or N
    C = torch.full((M, ldc), float("nan"), device=DEV)
    _lib.call("ce_kernel_gemm_tn_bf16", S(), P(A), A.stride(0), P(B), B.stride(0), M, N, K, P(C), ldc, scale_rows,
              ctypes.c_float(scale))
    torch.cuda.synchronize()
    return C


def check(C, A, B, M, N, K, scale_rows=0, scale=1.0):
    a, b = A[:K, :M].float(), B[:K, :N].float()
    ref = a.t() @ b
    bound = a.abs().t() @ b.abs()
    sc = torch.ones(M, 1, device=DEV)
    sc[:scale_rows] = scale
    ref, bound = ref * sc, bound * sc.abs()
    err = (C[:, :N] - ref).abs()
    assert torch.isfinite(C[:, :N]).all()
    worst = float((err / (bound + 1e-30)).max())
    assert bool((err <= 1e-5 * bound + 1e-30).all()), worst


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 512, 1), (512, 256, 100), (768, 768, 462),
                                   (768, 3072, 4096), (3072, 768, 9240), (2304, 768, 77 * 64),
                                   (4096, 4096, 512)])
def test_gemm_tn(M, N, K):
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(K, M, generator=g).to(torch.bfloat16).to(DEV)
    B = torch.randn(K, N, generator=g).to(torch.bfloat16).to(DEV)
    check(run_tn(A, B, M, N, K), A, B, M, N, K)


def test_gemm_tn_strides_and_row_scale():
    """lda > M, ldb > N (a column slice of a wider activation), ldc > N, q-row scale on the first rows"""
    M, N, K = 512, 256, 777
    g = torch.Generator(device="cpu").manual_seed(5)
    Aw = torch.randn(K, M + 256, generator=g).to(torch.bfloat16).to(DEV)
    Bw = torch.randn(K, N + 64, generator=g).to(torch.bfloat16).to(DEV)
    C = run_tn(Aw, Bw, M, N, K, scale_rows=256, scale=0.18, ldc=N + 128)
    check(C, Aw, Bw, M, N, K, scale_rows=256, scale=0.18)
    assert torch.isnan(C[:, N:]).all()          # columns past N untouched


def test_gemm_tn_one_chunk_direct_store():
    """256 tiles = one workgroup per CU: no split, the kernel stores C itself and applies the row
    scale there (scale_rows not a multiple of the tile)"""
    M, N, K = 4096, 4096, 320
    g = torch.Generator(device="cpu").manual_seed(9)
    A = torch.randn(K, M, generator=g).to(torch.bfloat16).to(DEV)
    B = torch.randn(K, N, generator=g).to(torch.bfloat16).to(DEV)
    check(run_tn(A, B, M, N, K, scale_rows=1000, scale=0.5), A, B, M, N, K, scale_rows=1000, scale=0.5)


def test_gemm_tn_full_size_deterministic():
    """the NegCLIP text batch (1,536 captions x 77 tokens) at the c_fc weight shape, twice: bitwise equal"""
    M, N, K = 3072, 768, 1536 * 77
    g = torch.Generator(device=DEV).manual_seed(11)
    A = (torch.randn(K, M, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    B = torch.randn(K, N, generator=g, device=DEV).to(torch.bfloat16)
    C1 = run_tn(A, B, M, N, K)
    C2 = run_tn(A, B, M, N, K)
    assert torch.equal(C1, C2)
    rows = torch.tensor([0, 1, 1535, 3071], device=DEV)
    ref = A[:, rows].float().t() @ B.float()
    bound = A[:, rows].float().abs().t() @ B.float().abs()
    assert bool(((C1[rows] - ref).abs() <= 1e-5 * bound).all())


def test_gemm_tn_rejects_bad_shapes():
    A = torch.zeros(64, 256, dtype=torch.bfloat16, device=DEV)
    C = torch.zeros(256, 256, device=DEV)
    with pytest.raises(_lib.ClipEmbedError, match="multiples of 256"):
        _lib.call("ce_kernel_gemm_tn_bf16", S(), P(A), 256, P(A), 256, 256, 192, 64, P(C), 256, 0, ctypes.c_float(1))


def test_train_backward_tn_matches_transpose_path():
    """one NegCLIP gradient computation with the MN-major dW GEMMs and with the transposed copies"""
    import clipembed
    from clipembed import weights as W
    from clipembed.config import get_model_config
    from clipembed.train import TextTowerTrainer

    cfg = get_model_config("ViT-L-14-336").with_depth(1, 2)
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    m.to(DEV)
    tr = TextTowerTrainer(m, lr=1e-4, weight_decay=0.1, usehardtext=True)
    imgs = torch.from_numpy(W.synthetic_images(4, seed=3)).cuda()
    rng = np.random.default_rng(0)
    caps = torch.from_numpy(rng.integers(1, 49000, size=(6, 77))).cuda()
    caps[:, 0] = 49406
    caps[np.arange(6), rng.integers(5, 70, size=6)] = 49407
    grads = {}
    prev = _lib.lib().ce_set_train_dw_tn(1)
    try:
        for on in (1, 0):
            _lib.lib().ce_set_train_dw_tn(on)
            tr.compute_grads(imgs, caps)
            torch.cuda.synchronize()
            grads[on] = {n: v.detach().clone() for n, v in tr.gviews.items()}
    finally:
        _lib.lib().ce_set_train_dw_tn(prev)
    for n, a in grads[1].items():
        b = grads[0][n]
        tol = 1e-4 * float(b.abs().max()) + 1e-12
        assert float((a - b).abs().max()) <= tol, n
