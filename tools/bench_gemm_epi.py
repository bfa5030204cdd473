"""GEMM A/B at the ViT-L/14-336 bench shapes (B = 256) with the epilogues the model runs
(LN fold on QKV / c_fc, LN stats on out-proj / c_proj), schedules interleaved in one process
(guide §5.4 rule 24), random data.

    python tools/bench_gemm_epi.py --scheds 1,11 [--rounds 3] [--reps 10] [--only fc,qkv]
    (':' also separates schedule tokens: tools/gpu_run.sh turns ',' into spaces)
A schedule token: <sched>[g<groupm>][a<auto>][s<stagger>][v<variant bits>][n]  (n: split-K tail off; a0: auto policy off;\ns<k>: first-round stagger of k x s_sleep 127 for half the CUs).
"""
import argparse
import ctypes
import json
import os
import sys
import time

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


def parse(tok):
    """<sched>[g<groupm>][a<auto>][s<stagger>][v<variant bits>][n], modifiers in any order."""
    import re
    m = re.fullmatch(r"(\d+)((?:[gasv]\d+)*)(n?)", tok)
    if not m:
        raise ValueError(f"bad schedule token {tok!r}")
    mods = {k: int(v) for k, v in re.findall(r"([gasv])(\d+)", m.group(2))}
    split = 0 if m.group(3) else 1
    stag = mods.get("s", 0) + 1          # always explicit (0 would keep the previous value)
    return int(m.group(1)), mods.get("g", 0), mods.get("a", 1), split, stag, mods.get("v", -1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--scheds", default="1,11")
    ap.add_argument("--only", default="")
    ap.add_argument("--warm-s", type=float, default=2.0)
    args = ap.parse_args()
    M = args.batch * 577
    # name: (N, K, act, epi, resid, out_bf16)
    shapes = {"qkv": (3072, 1024, 0, 2, False, True), "out": (1024, 1024, 0, 1, True, False),
              "fc": (4096, 1024, 1, 2, False, True), "proj": (1024, 4096, 0, 1, True, False),
              "fc_plain": (4096, 1024, 0, 0, False, True), "proj_plain": (1024, 4096, 0, 0, False, True), "fc_fold": (4096, 1024, 0, 2, False, True), "sq": (4096, 4096, 0, 0, False, True),
              # hi/lo residual stream (epi 3: resid and xb are [2][M][N] bf16 planes, no f32 output)
              "out_hl": (1024, 1024, 0, 3, True, False), "proj_hl": (1024, 4096, 0, 3, True, False)}
    if args.only:
        shapes = {k: v for k, v in shapes.items() if k in args.only.replace(":", ",").split(",")}
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    xw = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < args.warm_s:
        for _ in range(20):
            xw @ xw
        torch.cuda.synchronize()
    del xw
    g = torch.Generator(device="cuda").manual_seed(0)
    bufs = {}
    for name, (N, K, act, epi, resid, ob) in shapes.items():
        m = 4096 if name == "sq" else M
        A = (torch.rand(m, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        bias = torch.rand(N, device="cuda", generator=g)
        R = torch.rand(m, N, device="cuda", generator=g) if resid else None
        O = torch.empty(m, N, device="cuda", dtype=torch.bfloat16 if ob else torch.float32) if epi != 3 else None
        xb = torch.empty(m, N, device="cuda", dtype=torch.bfloat16) if epi == 1 else None
        part = torch.empty(m, N // 64, 2, device="cuda") if epi in (1, 3) else None
        if epi == 3:
            R = torch.stack([R.to(torch.bfloat16), torch.zeros(m, N, device="cuda", dtype=torch.bfloat16)]).contiguous()
            xb = torch.empty(2, m, N, device="cuda", dtype=torch.bfloat16)
        st = torch.stack([torch.rand(m, device="cuda", generator=g) * 0.1,
                          torch.rand(m, device="cuda", generator=g) + 0.5], 1).contiguous() if epi == 2 else None
        fc = W.float().sum(1).contiguous() if epi == 2 else None
        bufs[name] = (m, A, W, bias, R, O, xb, part, st, fc)
    res = {}
    L = _lib.lib()
    for _ in range(args.rounds):
        for tok in args.scheds.replace(":", ",").split(","):
            sc, gm, auto, split, stag, var = parse(tok)
            L.ce_set_gemm_variant(var)
            L.ce_set_gemm_schedule(sc | (gm << 8) | (stag << 24))
            L.ce_set_gemm_auto(auto)
            L.ce_set_gemm_splitk(split)
            for name, (N, K, act, epi, resid, ob) in shapes.items():
                m, A, W, bias, R, O, xb, part, st, fc = bufs[name]

                def fn():
                    _lib.call("ce_kernel_gemm_bf16_epi", stream, P(A), P(W), m, N, K, P(bias), act, P(R), P(O),
                              _lib.CE_BF16 if ob else _lib.CE_F32, epi, P(xb), P(part), P(st), P(fc))
                ms = timeit(fn, args.reps)
                res.setdefault(f"{name}/s{tok}", []).append(2.0 * m * N * K / (ms * 1e-3) / 1e12)
    for k, v in res.items():
        print(f"{k:<16} " + " ".join(f"{x:8.1f}" for x in v) + f"   best {max(v):8.1f}", flush=True)
    print(json.dumps({k: round(max(v), 1) for k, v in res.items()}))


if __name__ == "__main__":
    main()
