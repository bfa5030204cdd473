"""Per-workgroup (per-tile for the persistent SCHED 11) timeline of a GEMM launch (ce_set_gemm_trace, s_memrealtime at 100 MHz):
K-loop and epilogue durations and how many workgroups are in their epilogue at once.

    python tools/gemm_trace.py --shape out --scheds 1,1s4,12
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO, os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from clipembed import _lib  # noqa: E402
from bench_gemm_epi import P, parse  # noqa: E402

SHAPES = {"qkv": (3072, 1024, 0, 2, False, True), "out": (1024, 1024, 0, 1, True, False),
          "fc": (4096, 1024, 1, 2, False, True), "proj": (1024, 4096, 0, 1, True, False),
          "fc_plain": (4096, 1024, 0, 0, False, True), "fc_fold": (4096, 1024, 0, 2, False, True),
          "out_hl": (1024, 1024, 0, 3, True, False), "proj_hl": (1024, 4096, 0, 3, True, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="out")
    ap.add_argument("--scheds", default="1,11")
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    M = args.batch * 577
    N, K, act, epi, resid, ob = SHAPES[args.shape]
    g = torch.Generator(device="cuda").manual_seed(0)
    A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    bias = torch.rand(N, device="cuda", generator=g)
    R = torch.rand(M, N, device="cuda", generator=g) if resid else None
    O = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if ob else torch.float32) if epi != 3 else None
    xb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
    part = torch.empty(M, N // 64, 2, device="cuda") if epi in (1, 3) else None
    if epi == 3:     # hi/lo planes
        R = torch.stack([R.to(torch.bfloat16), torch.zeros_like(R, dtype=torch.bfloat16)]).contiguous()
        xb = torch.empty(2, M, N, device="cuda", dtype=torch.bfloat16)
    st = torch.stack([torch.rand(M, device="cuda", generator=g) * 0.1,
                      torch.rand(M, device="cuda", generator=g) + 0.5], 1).contiguous() if epi == 2 else None
    fc = W.float().sum(1).contiguous() if epi == 2 else None
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = _lib.lib()
    nb = 20000
    tr = torch.zeros(nb, 4, dtype=torch.int64, device="cuda")

    def run():
        _lib.call("ce_kernel_gemm_bf16_epi", stream, P(A), P(W), M, N, K, P(bias), act, P(R), P(O),
                  _lib.CE_BF16 if ob else _lib.CE_F32, epi, P(xb), P(part), P(st), P(fc))

    for tok in args.scheds.split(","):
        sc, gm, auto, split, stag, var = parse(tok)
        L.ce_set_gemm_variant(var)
        L.ce_set_gemm_schedule(sc | (gm << 8) | (stag << 24))
        L.ce_set_gemm_auto(auto)
        L.ce_set_gemm_splitk(split)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        tr.zero_()
        L.ce_set_gemm_trace(P(tr), nb)
        run()
        torch.cuda.synchronize()
        L.ce_set_gemm_trace(None, 0)
        t = tr.cpu().numpy()
        t = t[t[:, 0] > 0]
        t0 = t[:, 0].min()
        s0, s1, s2 = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, (t[:, 2] - t0) / 100.0   # us
        main, epi_t = s1 - s0, s2 - s1
        span = s2.max()
        flops = 2.0 * M * N * K
        print(f"== {args.shape} s{tok}: {len(t)} blocks, span {span:.1f} us ({flops / span / 1e6:.0f} TFLOP/s), "
              f"K-loop mean {main.mean():.2f} us (p10 {np.percentile(main, 10):.2f} p90 {np.percentile(main, 90):.2f}), "
              f"epilogue mean {epi_t.mean():.2f} us (p10 {np.percentile(epi_t, 10):.2f} p90 {np.percentile(epi_t, 90):.2f})")
        # concurrency histogram: how many blocks are in K-loop / epilogue at each microsecond
        grid = np.arange(0, span, 1.0)
        in_main = ((s0[None, :] <= grid[:, None]) & (grid[:, None] < s1[None, :])).sum(1)
        in_epi = ((s1[None, :] <= grid[:, None]) & (grid[:, None] < s2[None, :])).sum(1)
        step = max(1, len(grid) // 40)
        print("   t(us)  K-loop  epilogue")
        for i in range(0, len(grid), step):
            print(f"   {grid[i]:6.0f} {in_main[i]:6d} {in_epi[i]:8d}")
        first = t[:256]
        hw = first[:, 3] & 0xffffffff
        cu = (hw >> 8) & 0xf
        sh = (hw >> 12) & 0x1
        se = (hw >> 13) & 0x7
        xcc = first[:, 3] >> 32
        print("   first 16 blocks (block, xcc, se, sh, cu):", [(i, int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i])) for i in range(16)])


if __name__ == "__main__":
    main()
