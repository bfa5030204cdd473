"""Kernel micro-benchmarks at the ViT-L/14-336 bench shapes (B = 256 per GPU), random data,
interleaved A/B of GEMM schedules in one process (guide §5.4 rule 24).

    python tools/bench_kernels.py [--batch 256] [--reps 10] [--rounds 3]
"""
import argparse
import ctypes
import json
import time
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]

import torch  # noqa: E402

from clipembed import _lib  # noqa: E402


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, reps):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scheds", default="0,1")
    ap.add_argument("--warm-s", type=float, default=2.0)
    ap.add_argument("--torch-ref", action="store_true", help="also time torch.matmul (hipBLASLt) per shape")
    ap.add_argument("--only", default="", help="comma list of shape names to run (default all)")
    ap.add_argument("--attn-vars", default="1", help="comma list of attention variants (ce_set_attn_variant) to A/B")
    args = ap.parse_args()
    B = args.batch
    Mv, Mt = B * 577, B * 77
    shapes = {  # name: (M, N, K, act, resid, out_bf16)
        "qkv_v": (Mv, 3072, 1024, 0, False, True), "out_v": (Mv, 1024, 1024, 0, True, False),
        "fc_v": (Mv, 4096, 1024, 1, False, True), "proj_v": (Mv, 1024, 4096, 0, True, False),
        "qkv_t": (Mt, 2304, 768, 0, False, True), "fc_t": (Mt, 3072, 768, 1, False, True),
        # diagnostics: A resident in L2/MALL (M = 8192) and a square 4096^3 reference point
        "qkv_m8k": (8192, 3072, 1024, 0, False, True), "sq4096": (4096, 4096, 4096, 0, False, True),
        # epilogue ablations: the vision shapes with a plain bf16 store (no GELU / residual / f32 out)
        "fc_v_plain": (Mv, 4096, 1024, 0, False, True), "out_v_plain": (Mv, 1024, 1024, 0, False, True),
        "proj_v_plain": (Mv, 1024, 4096, 0, False, True),
        "out_v_f32": (Mv, 1024, 1024, 0, False, False), "proj_v_f32": (Mv, 1024, 4096, 0, False, False),
    }
    if args.only:
        keep = set(args.only.replace("+", ",").split(","))
        shapes = {k: v for k, v in shapes.items() if k in keep}
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    # bring the clocks up before the first timed shape (~2 s of dense bf16 matmul)
    xw = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < args.warm_s:
        for _ in range(20):
            xw @ xw
        torch.cuda.synchronize()
    del xw
    g = torch.Generator(device="cuda").manual_seed(0)
    res = {}
    bufs = {}
    for name, (M, N, K, act, resid, ob) in shapes.items():
        A = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        bias = torch.rand(N, device="cuda", generator=g)
        R = torch.rand(M, N, device="cuda", generator=g) if resid else None
        O = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if ob else torch.float32)
        bufs[name] = (A, W, bias, R, O)
    for rnd in range(args.rounds):
        for sched in args.scheds.split(","):   # "1", "1g4" (tile-order M-group 4), "1r3" (resid ring 3),
            # "1n" (split-K tail off)
            # suffix "n": split-K tail off
            _lib.lib().ce_set_gemm_splitk(0 if sched.endswith("n") else 1)
            sc, _, rg = sched.rstrip("n").partition("r")
            sc, _, gm = sc.partition("g")
            _lib.lib().ce_set_gemm_schedule(int(sc) | (int(gm or 0) << 8) | (int(rg or 0) << 16))
            for name, (M, N, K, act, resid, ob) in shapes.items():
                A, W, bias, R, O = bufs[name]

                def fn():
                    _lib.call("ce_kernel_gemm_bf16", stream, P(A), P(W), M, N, K, P(bias), act, P(R), P(O),
                              _lib.CE_BF16 if ob else _lib.CE_F32)
                ms = timeit(fn, args.reps)
                tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
                res.setdefault(f"{name}/s{sched}", []).append(tf)
    if args.torch_ref:
        # library reference point: torch.matmul (hipBLASLt) on the same shapes, bf16 out, no epilogue
        for name, (M, N, K, act, resid, ob) in shapes.items():
            A, W, bias, R, O = bufs[name]
            Ob = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            for rnd in range(args.rounds):
                ms = timeit(lambda: torch.matmul(A, W.t(), out=Ob), args.reps)
                res.setdefault(f"{name}/torch", []).append(2.0 * M * N * K / (ms * 1e-3) / 1e12)
            del Ob
    attns = {"attn_v": (577, 16, 0, B), "attn_t": (77, 12, 1, B),
             # diagnostics: the same FLOPs at longer sequences (fewer, longer key loops per q-block)
             "attn_v1153": (1153, 16, 0, B // 4), "attn_v2305": (2305, 16, 0, B // 16),
             # the image shape at smaller batches (K / V of every head within the 256-MB MALL)
             "attn_v_b64": (577, 16, 0, B // 4), "attn_v_b32": (577, 16, 0, B // 8)}
    if args.only:
        attns = {k: v for k, v in attns.items() if k in keep}
    else:
        attns = {k: v for k, v in attns.items() if k in ("attn_v", "attn_t")}
    for attn, (L, H, causal, Bx) in attns.items():
        qkv = (torch.randn(Bx * L, 3 * H * 64, device="cuda", generator=g)).to(torch.bfloat16)
        out = torch.empty(Bx * L, H * 64, device="cuda", dtype=torch.bfloat16)
        for rnd in range(args.rounds):
            for var in [int(v) for v in args.attn_vars.replace("+", ",").split(",")]:
                _lib.lib().ce_set_attn_variant(var)
                ms = timeit(lambda: _lib.call("ce_kernel_attention", stream, P(qkv), P(out), Bx, L, H, causal),
                            args.reps)
                res.setdefault(f"{attn}/var{var}", []).append(4.0 * Bx * H * L * L * 64 / (ms * 1e-3) / 1e12)
        _lib.lib().ce_set_attn_variant(-1)
    for rows, D in (((Mv, 1024),) if not args.only or "ln_v" in keep else ()):
        x = torch.randn(rows, D, device="cuda", generator=g)
        w = torch.ones(D, device="cuda")
        o = torch.empty(rows, D, device="cuda", dtype=torch.bfloat16)
        for rnd in range(args.rounds):
            ms = timeit(lambda: _lib.call("ce_kernel_layernorm", stream, P(x), P(o), _lib.CE_BF16, P(w), P(w), rows, D),
                        args.reps)
            res.setdefault("ln_v (GB/s)", []).append(rows * D * 6 / (ms * 1e-3) / 1e9)
    for k, v in res.items():
        print(f"{k:<16} " + " ".join(f"{x:8.1f}" for x in v) + f"   best {max(v):8.1f}")
    print(json.dumps({k: round(max(v), 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
