"""HBM bytes per launch of the bench's kernels from two rocprofv3 --pmc passes over bench.py itself
(tools/gpu_run.sh steps pmc:FETCH_SIZE and pmc:WRITE_SIZE; MI355X_MICROARCH.md §HBM: separate
passes, FETCH_SIZE doubled on gfx950, counters in KB).  Dispatches are grouped by kernel name and
grid size (the image tower's persistent GEMMs run 256 workgroups, the text tower's one-tile GEMMs
one per tile), so a bench tag maps to one group.

    python tools/pmc_bench_traffic.py gpurun_out/<tag>_pmc1_FETCH_SIZE gpurun_out/<tag>_pmc2_WRITE_SIZE \
        [profiles/pmc_traffic.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench tag -> (kernel-name prefix(es), grid size in threads) of the image tower at B = 256 (clip
# workload) and of the PACL pooling at B = 512 (pacl workload: its two passes sum to one launch)
TAGS = {"gemm_fc_v": ("void ce::(anonymous namespace)::gemm_bf16_w4pp<1, false, true, 2", 65536),
        "gemm_qkv_v": ("void ce::(anonymous namespace)::gemm_bf16_w4pp<0, false, true, 2", 65536),
        "attn_v": ("void ce::(anonymous namespace)::attn_fwd<false", None),
        "gemm_out_v": ("resid_hl:out", 65536),
        "gemm_proj_v": ("resid_hl:proj", 65536),
        "pacl_pool": (("void ce::(anonymous namespace)::pacl_pool_part_k", "ce::(anonymous namespace)::pacl_pool_finish_k"),
                      None)}


RESID_HL = "void ce::(anonymous namespace)::gemm_w4_resid_hl<"


def load(d, counter):
    """{(kernel, grid): [value per dispatch]}; the staged-residual kernel's dispatches (out-proj and
    c_proj share its name and grid) are split by dispatch order: each image block launches out-proj
    before c_proj, so in dispatch order they alternate out, proj, out, proj ..."""
    g = defaultdict(list)
    hl = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                key = (row["Kernel_Name"], int(row["Grid_Size"]))
                if key[0].startswith(RESID_HL) and key[1] == 65536:
                    hl.append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"])))
                else:
                    g[key].append(float(row["Counter_Value"]))
    hl.sort()
    for i, (_, v) in enumerate(hl):
        g[("resid_hl:" + ("out" if i % 2 == 0 else "proj"), 65536)].append(v)
    return g


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    fetch, write = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    for (k, grid), v in sorted(fetch.items(), key=lambda kv: -sum(kv[1]))[:16]:
        w = write.get((k, grid), [])
        print(f"{k[:70]:<70} grid {grid:8d} n {len(v):3d}/{len(w):3d} fetch x2 {2 * sum(v) / len(v) / 1024:9.1f} MB"
              f"  write {sum(w) / max(1, len(w)) / 1024:8.1f} MB")
    if not out:
        return
    res = {}
    if os.path.exists(out):
        with open(out) as f:
            res = json.load(f)
    for tag, (prefs, grid) in TAGS.items():
        prefs = prefs if isinstance(prefs, tuple) else (prefs,)
        f2 = wr = 0.0
        n = []
        for pref in prefs:
            fs = [v for (k, g), vs in fetch.items() if k.startswith(pref) and (grid is None or g == grid) for v in vs]
            ws = [v for (k, g), vs in write.items() if k.startswith(pref) and (grid is None or g == grid) for v in vs]
            if not fs or not ws:
                break
            f2 += 2 * sum(fs) / len(fs) * 1024
            wr += sum(ws) / len(ws) * 1024
            n += [len(fs), len(ws)]
        else:
            pass
        if len(n) != 2 * len(prefs):
            continue
        res[tag] = {"hbm_bytes_per_launch": round(f2 + wr), "fetch_bytes_corrected": round(f2),
                    "write_bytes": round(wr), "dispatches": n,
                    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over bench.py, {fd}, {wd}"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
