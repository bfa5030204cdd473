"""MFMA utilisation per engine kernel from one rocprofv3 --pmc pass over bench.py (tools/gpu_run.sh
pmcs:SQ_VALU_MFMA_BUSY_CYCLES+GRBM_GUI_ACTIVE+...).

    python tools/summarize_mfma.py gpurun_out/<tag>_pmcsN/run_counter_collection.csv --out profiles/r04/mfma

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the fraction of the matrix
pipes' cycles spent on MFMAs while the kernel ran (GRBM_GUI_ACTIVE sums the 8 XCDs; the busy count sums
every SIMD's MFMA cycles: c_fc's 75.6 M v_mfma_f32_16x16x32_bf16 x 16 cycles = 1.21e9 per launch, as
counted).  clock = GRBM_GUI_ACTIVE / 8 / duration.  `frac_at_nominal` = mfma_busy x clock / 2.4 GHz,
comparable with bench.py's event-timed FLOP fraction of the 2.5 PF/s (2.4 GHz) peak.
Kernel classes map to the engine's tags by name, grid and duration (out-proj and c_proj share the
staged-residual kernel and grid; c_proj's K = 4096 launches run ~2x longer; the thresholds are the
B = 256 inference bench's, so over a NegCLIP run only dW_tn and attn_v are clean classes)."""
import argparse
import collections
import csv
import json
import os
import re


def tag_of(name, grid, ms):
    if "gemm_tn_w4" in name:
        return "dW_tn"
    if "gemm_w4_resid_hl" in name and grid == 65536:
        return "gemm_proj_v" if ms > 0.6 else "gemm_out_v"
    if "gemm_bf16_w4pp<1" in name and grid == 65536:
        return "gemm_fc_v"
    if "gemm_bf16_w4pp<0" in name and grid == 65536:
        return "gemm_qkv_v"
    if re.search(r"attn_fwd<false", name):
        return "attn_v"
    if re.search(r"attn_fwd<true", name):
        return "attn_t"
    if "gemm_w4_resid_hl" in name:
        return "gemm_resid_t"
    if "gemm_bf16_w4pp" in name:
        return "gemm_fold_t"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = {}
    for r in csv.DictReader(open(a.csv)):
        key = (r["Dispatch_Id"], r["Kernel_Name"], int(r["Grid_Size"]))
        disp[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for key, c in per.items():
        tag = tag_of(key[1], key[2], disp[key])
        if tag is None or "GRBM_GUI_ACTIVE" not in c or "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
            continue
        t = acc[tag]
        t["n"] += 1
        t["ms"] += disp[key]
        t["busy"] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        t["gui8"] += c["GRBM_GUI_ACTIVE"] / 8
        t["wave"] += c.get("SQ_WAVE_CYCLES", 0.0)
        t["lds_conf"] += c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        t["lds_act"] += c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    out = {}
    lines = [f"{'kernel':<14} {'launches':>8} {'avg ms':>8} {'clock GHz':>9} {'mfma_busy':>9} {'at 2.4 GHz':>10} "
             f"{'LDS conflict':>12}"]
    for tag, t in sorted(acc.items(), key=lambda kv: -kv[1]["ms"]):
        busy = t["busy"] / (t["gui8"] * 1024)
        clk = t["gui8"] / (t["ms"] * 1e-3) / 1e9
        d = {"launches": int(t["n"]), "avg_ms_profiled": round(t["ms"] / t["n"], 4), "clock_GHz": round(clk, 3),
             "mfma_busy": round(busy, 4), "frac_at_nominal": round(busy * clk / 2.4, 4),
             "lds_conflict_frac": round(t["lds_conf"] / t["lds_act"], 4) if t["lds_act"] else None}
        out[tag] = d
        lines.append(f"{tag:<14} {d['launches']:>8} {d['avg_ms_profiled']:>8.4f} {clk:>9.3f} {busy:>9.4f} "
                     f"{d['frac_at_nominal']:>10.4f} {d['lds_conflict_frac'] if d['lds_conflict_frac'] is not None else '-':>12}")
    print("\n".join(lines))
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out + ".json", "w") as f:
            json.dump({"source": a.csv, "method": __doc__.split("\n\n")[1].strip(), "kernels": out}, f, indent=1)
        with open(a.out + ".txt", "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
