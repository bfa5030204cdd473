"""Per-wave timeline of the image-tower attention (variant 1405 = 381 + s_memrealtime stamps,
ce_set_attn_trace) at the bench shape: where a 32-query wave's time goes outside its key-tile loop.

    python tools/attn_trace.py [--batch 256] [--L 577]

Prints per-phase averages (µs, 100-MHz clock) over all waves of the last of a few launches: prologue
(entry -> Q and key 0 done), tile-0 wait (-> first barrier passed), key-tile loop, epilogue (loop end ->
stores retired), and how many waves were resident per CU over time."""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from clipembed import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--L", type=int, default=577)
    ap.add_argument("--H", type=int, default=16)
    ap.add_argument("--var", type=int, default=1405, help="1405 (381 + stamps), 3453 (2429 + stamps), 1917 / 10109 (893 / 9085 + phase sums)")
    args = ap.parse_args()
    B, L, H = args.batch, args.L, args.H
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * L, 3 * H * 64, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(B * L, H * 64, device="cuda", dtype=torch.bfloat16)
    nblk = ((L + 127) // 128) * H * B
    buf = torch.zeros(nblk * 4 * 8, device="cuda", dtype=torch.int64)
    lib = _lib.lib()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    prev = lib.ce_set_attn_variant(args.var)
    try:
        def launch():
            _lib.call("ce_kernel_attention", stream, ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                      B, L, H, 0)
        for _ in range(20):       # clocks up
            launch()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(20):
            launch()
        ev1.record()
        ev1.synchronize()
        ms = ev0.elapsed_time(ev1) / 20
        print(f"untraced launches of variant {args.var}: {ms:.4f} ms, "
              f"{4.0 * B * H * L * L * 64 / (ms * 1e-3) / 1e12:.1f} TF/s")
        _lib.call("ce_set_attn_trace", ctypes.c_void_p(buf.data_ptr()), nblk * 4)
        _lib.call("ce_kernel_attention", stream, ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                  B, L, H, 0)
        torch.cuda.synchronize()
        _lib.call("ce_set_attn_trace", None, 0)
    finally:
        lib.ce_set_attn_variant(prev)
    if args.var in (1917, 10109):
        # persistent kernel: per wave {time in block starts, key-tile loops, epilogues, blocks}
        q = buf.view(-1, 8).cpu().numpy().astype(np.int64)
        q = q[q[:, 3] > 0]
        t0 = q[:, 4].min()
        st, en = (q[:, 4] - t0) / 100.0, (q[:, 5] - t0) / 100.0
        print(f"wave first stamp: p0 {st.min():.1f} p50 {np.percentile(st, 50):.1f} p90 {np.percentile(st, 90):.1f} "
              f"max {st.max():.1f} us; last stamp: min {en.min():.1f} p50 {np.percentile(en, 50):.1f} "
              f"p90 {np.percentile(en, 90):.1f} max {en.max():.1f} us")
        xc = (q[:, 6] >> 32) & 0xf
        allq = buf.view(-1, 8)[:, 3].cpu().numpy()
        bid = np.nonzero(allq > 0)[0] // 4
        for x in range(8):
            m = xc == x
            if m.any():
                print(f"  XCC {x}: waves {int(m.sum())}, bid%8 == XCC {float(np.mean(bid[m] % 8 == x)):.2f}, "
                      f"end p50 {np.percentile(en[m], 50):.1f} max {en[m].max():.1f} us, "
                      f"loop per block {float(np.mean(q[m, 1] / 100.0 / q[m, 3])):.2f} us")
        nb = q[:, 3].astype(np.float64)
        print(f"persistent waves {len(q)}, blocks per wave {nb.mean():.2f} (min {nb.min():.0f}, max {nb.max():.0f})")
        for k, name in enumerate(("block_start", "loop", "epilogue")):
            per = q[:, k] / 100.0 / nb
            print(f"  {name:<11} per block mean {per.mean():7.2f} us  p10 {np.percentile(per, 10):7.2f}  "
                  f"p90 {np.percentile(per, 90):7.2f}")
        return
    r = buf.view(-1, 8).cpu().numpy().astype(np.int64)
    r = r[r[:, 0] > 0]
    t0 = r[:, 0].min()
    t = (r[:, :5] - t0) / 100.0          # µs
    span = t[:, 4].max()
    ph = {"prologue": t[:, 1] - t[:, 0], "tile0_wait": t[:, 2] - t[:, 1], "loop": t[:, 3] - t[:, 2],
          "epilogue": t[:, 4] - t[:, 3], "wave_total": t[:, 4] - t[:, 0]}
    print(f"waves {len(r)}  kernel span {span:.1f} us  (L = {L}, B = {B}, H = {H})")
    for k, v in ph.items():
        print(f"  {k:<11} mean {v.mean():7.2f} us  p10 {np.percentile(v, 10):7.2f}  p50 {np.percentile(v, 50):7.2f}  "
              f"p90 {np.percentile(v, 90):7.2f}")
    # waves per CU over time (resident = entry <= t < exit), CU = (XCC, SE, CU) from the id word
    hw = r[:, 5] & 0xffffffff
    xcc = r[:, 5] >> 32
    cu = (xcc << 16) | (((hw >> 13) & 0x7) << 8) | ((hw >> 8) & 0xf)
    ncu = len(np.unique(cu))
    grid = np.linspace(0, span, 200)
    res = [(np.sum((t[:, 0] <= x) & (t[:, 4] > x))) / ncu for x in grid]
    print(f"  CUs seen {ncu}; resident waves per CU: mean {np.mean(res):.2f}, max {np.max(res):.2f}")
    # busy fraction of the loop phase: waves in their tile loop per CU over time
    lp = [(np.sum((t[:, 2] <= x) & (t[:, 3] > x))) / ncu for x in grid]
    print(f"  waves in the tile loop per CU: mean {np.mean(lp):.2f}")


if __name__ == "__main__":
    main()
