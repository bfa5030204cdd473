"""Per-step timeline of a rocprofv3 kernel trace (rocpd SQLite db) of bench.py: the image tower's
stream vs the text tower's, how much of the step only text kernels occupy, and the per-stream busy
time.  python tools/trace_overlap.py gpurun_out/<tag>_prof<n>/run_results.db"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    suf = [r[0] for r in c.execute("select name from sqlite_master where type='table'")
           if r[0].startswith("rocpd_kernel_dispatch_")][0][len("rocpd_kernel_dispatch_"):]
    names = {r[0]: r[1] for r in c.execute(f"select id, display_name from rocpd_info_kernel_symbol_{suf}")}
    rows = [(s, e, names[k].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0], st)
            for s, e, k, st in c.execute(f"select start, end, kernel_id, stream_id from rocpd_kernel_dispatch_{suf}")]
    rows = [r for r in rows if not r[2].startswith("__amd")]
    rows.sort()
    img_stream = [r[3] for r in rows if r[2].startswith("ce::im2col")][0]
    starts = [r[0] for r in rows if r[2].startswith("ce::im2col")]
    for i, t0 in enumerate(starts[:-1]):
        t1 = starts[i + 1]
        ks = [r for r in rows if t0 <= r[0] < t1]
        img = [(s, e) for s, e, n, st in ks if st == img_stream]
        txt = [(s, e) for s, e, n, st in ks if st != img_stream]
        img_busy = sum(e - s for s, e in img) / 1e6
        txt_busy = sum(e - s for s, e in txt) / 1e6
        # gaps on the image stream (between consecutive image kernels)
        gaps = sum(max(0, img[j + 1][0] - img[j][1]) for j in range(len(img) - 1)) / 1e6
        print(f"step {i}: span {(t1 - t0) / 1e6:7.2f} ms  image busy {img_busy:7.2f}  gaps {gaps:5.2f}  "
              f"text busy {txt_busy:5.2f} ({len(txt)} kernels)")
    # per-kernel average over the trace
    agg = {}
    for s, e, n, st in rows:
        a = agg.setdefault((n[:58], st == img_stream), [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
    print(f"{'kernel':<60} {'img':>4} {'n':>5} {'avg ms':>8} {'total':>8}")
    for (n, im), (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:24]:
        print(f"{n:<60} {int(im):>4} {cnt:5d} {tot / cnt:8.4f} {tot:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
