"""Effective clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass (tools/gpu_run.sh clock step):
clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time (MI355X_MICROARCH.md 'DVFS give-back').
    python tools/clock_summary.py gpurun_out/<tag>_clk<n>/run_counter_collection.csv"""
import collections
import csv
import sys


def main(path):
    rows = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            if dur <= 0:
                continue
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            name = name.split("(")[0][:60]
            rows[name].append((float(r["Counter_Value"]), dur))
    out = []
    for name, v in rows.items():
        cyc = sum(c for c, _ in v)
        t = sum(d for _, d in v)
        out.append((t, name, len(v), cyc / 8 / t / 1e9))
    out.sort(reverse=True)
    print(f"{'kernel':<62} {'n':>5} {'total ms':>9} {'GHz':>6}")
    for t, name, n, ghz in out[:25]:
        print(f"{name:<62} {n:5d} {t * 1e3:9.3f} {ghz:6.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
