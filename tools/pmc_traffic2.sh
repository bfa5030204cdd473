#!/bin/bash
# HBM-side traffic per launch (FETCH_SIZE, WRITE_SIZE in separate rocprofv3 --pmc passes) of the
# bench's vision GEMMs on the default policy, via tools/bench_gemm_epi.py (the model's epilogues).
# Output: gpurun_out/pmc2/<shape>_<counter>/ ; aggregate: tools/pmc_traffic.py gpurun_out/pmc2 <json>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPES=${1:-qkv,fc,out,proj}
OUT=${2:-gpurun_out/pmc2}
mkdir -p $OUT
for s in ${SHAPES//,/ }; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/${s}_${c}
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $c -d $d -o run --output-format csv -- \
      python3 tools/bench_gemm_epi.py --rounds 1 --reps 3 --warm-s 0 --scheds 1 --only $s > $d.log 2>&1 || exit 1
  done
done
echo pmc done
