"""Time torch.matmul (hipBLASLt) on the bench's GEMM shapes — a library reference point for the
hand-written kernel (run under rocprofv3 --kernel-trace to see which library kernel it picks)."""
import torch

B = 256
Mv, Mt = B * 577, B * 77
for name, (M, N, K) in {"qkv_v": (Mv, 3072, 1024), "fc_v": (Mv, 4096, 1024), "out_v": (Mv, 1024, 1024),
                        "proj_v": (Mv, 1024, 4096)}.items():
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        torch.matmul(A, W.t())
    torch.cuda.synchronize()
    print(name, "done", flush=True)
