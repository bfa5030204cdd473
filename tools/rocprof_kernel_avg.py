"""Average duration per (kernel, grid size) from a rocprofv3 --kernel-trace csv: separates the image
tower's persistent GEMM launches (256 workgroups) from the text tower's one-tile launches of the same
template, which run_kernel_stats.csv averages together.

    python tools/rocprof_kernel_avg.py gpurun_out/<tag>_prof<n>/run_kernel_trace.csv [name-prefix]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    pref = sys.argv[2] if len(sys.argv) > 2 else ""
    g = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if pref in r["Kernel_Name"]:
                g[(r["Kernel_Name"], int(r["Grid_Size_X"]))].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for (k, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"{k[:80]:<80} grid {grid:9d} n {len(v):5d} avg {sum(v) / len(v):9.4f} ms total {sum(v):9.2f} ms")


if __name__ == "__main__":
    main()
