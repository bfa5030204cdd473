"""Aggregate tools/pmc_traffic.sh into profiles/pmc_traffic.json (read by bench.py's roofline).

    python tools/pmc_traffic.py gpurun_out/pmct profiles/pmc_traffic.json

hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes), averaged over the dispatches of
the shape's kernel (gfx950: FETCH_SIZE counts half of a wide coalesced stream, MI355X_MICROARCH.md
§HBM; WRITE_SIZE is exact for 16-B-per-lane stores and approximate for the 8-B stores of the GEMM
bf16 epilogue and the attention output).
"""
import csv
import glob
import json
import os
import sys

KERNEL = {"attn_v": "attn_fwd", "attn_t": "attn_fwd", "ln_v": "layernorm_k"}
# tools/pmc_traffic2.sh shapes (bench_gemm_epi names): the main GEMM kernel of the launch (the
# persistent four-wave kernel for qkv / fc, the 4-phase kernel for out / proj)
KERNEL2 = {"qkv": "gemm_bf16_w4pp", "fc": "gemm_bf16_w4pp", "out": "gemm_bf16_nt", "proj": "gemm_bf16_nt",
           # the hi/lo residual GEMMs on the staged-residual four-wave kernel (default since r02)
           "out_hl": "gemm_w4_resid_hl", "proj_hl": "gemm_w4_resid_hl"}


def avg_counter(d, counter, kname):
    vals = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kname in row["Kernel_Name"] and row["Counter_Name"] == counter:
                    vals.append(float(row["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    root, out = sys.argv[1], sys.argv[2]
    res = {}
    if os.path.exists(out):          # merge: keep the entries of shapes not measured in this run
        with open(out) as f:
            res = json.load(f)
    shapes = sorted({os.path.basename(p).rsplit("_", 2)[0] for p in glob.glob(os.path.join(root, "*_FETCH_SIZE"))})
    for s in shapes:
        kname = KERNEL.get(s, KERNEL2.get(s, "gemm_bf16_nt"))
        fetch, nf = avg_counter(os.path.join(root, f"{s}_FETCH_SIZE"), "FETCH_SIZE", kname)
        write, nw = avg_counter(os.path.join(root, f"{s}_WRITE_SIZE"), "WRITE_SIZE", kname)
        if fetch is None or write is None:
            continue
        tag = s if s in KERNEL else "gemm_" + (s + "_v" if s in KERNEL2 else s)
        res[tag] = {"hbm_bytes_per_launch": round((2 * fetch + write) * 1024),
                    "fetch_bytes_corrected": round(2 * fetch * 1024), "write_bytes": round(write * 1024),
                    "dispatches": [nf, nw], "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, {root}"}
        print(f"{tag:<12} fetch {2 * fetch / 1024:9.1f} MB  write {write / 1024:8.1f} MB  ({nf}/{nw} dispatches)")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
