"""Summarise rocprofv3 --pmc CSV passes (tools/pmc_gemm.sh) per kernel dispatch class.

    python tools/summarize_pmc.py gpurun_out/pmc  [--json out.json]

Kernel class = short kernel name + grid size (one class per GEMM shape / attention shape).
FETCH_SIZE is doubled for the gfx950 under-count of wide streaming reads (MI355X_MICROARCH.md
§HBM: FETCH_SIZE reports exactly 1/2 of a wide coalesced stream); WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Both are KB per dispatch.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(gemm_bf16_\w+|attn_fwd|layernorm_k|fgemm_k|pacl_pool_k|im2col_k)[^(]*", name)
    return m.group(0) if m else name[:40]


def main():
    root = sys.argv[1]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    per = defaultdict(lambda: defaultdict(list))   # class -> counter -> [values per dispatch]
    dur = defaultdict(list)
    for path in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
        seen = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if not k.startswith(("gemm", "attn", "layernorm", "pacl", "fgemm", "im2col")):
                    continue
                cls = f"{k} grid={row['Grid_Size']}"
                per[cls][row["Counter_Name"]].append(float(row["Counter_Value"]))
                key = (path, row["Dispatch_Id"])
                if key not in seen:
                    seen[key] = 1
                    dur[cls].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    summary = {}
    for cls in sorted(per):
        c = {k: sum(v) / len(v) for k, v in per[cls].items()}
        d = {"dispatches": len(dur[cls]), "avg_ms_profiled": round(sum(dur[cls]) / max(1, len(dur[cls])), 4)}
        if "FETCH_SIZE" in c:
            d["fetch_MB_corrected"] = round(2 * c["FETCH_SIZE"] / 1024, 1)
        if "WRITE_SIZE" in c:
            d["write_MB"] = round(c["WRITE_SIZE"] / 1024, 1)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["hbm_bytes_per_launch"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
            act = c["SQ_LDS_IDX_ACTIVE"] - c["SQ_LDS_BANK_CONFLICT"]
            d["lds_conflict_ratio"] = round(c["SQ_LDS_BANK_CONFLICT"] / max(1.0, act), 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # GRBM_GUI_ACTIVE is summed over 8 XCDs; 1024 SIMDs
            d["mfma_busy_pct"] = round(100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 1)
            d["clock_GHz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (d["avg_ms_profiled"] * 1e-3) / 1e9, 3)
        if "SQ_WAVE_CYCLES" in c:
            w = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if k in c:
                    d[k.lower() + "_pct"] = round(100 * c[k] / w, 1)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            d["l2_hit_pct"] = round(100 * c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 1)
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAVES"):
            if k in c:
                d[k] = c[k]
        summary[cls] = d
        print(cls)
        for k, v in d.items():
            print(f"    {k:<28} {v}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump(summary, f, indent=1)


if __name__ == "__main__":
    main()
