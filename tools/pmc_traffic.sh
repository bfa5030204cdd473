#!/bin/bash
# HBM traffic per launch for the bench's dominant kernels: one rocprofv3 --kernel-trace --pmc run
# per (shape, counter) so every dispatch in a directory belongs to one bench tag, FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md: they cannot share a pass).
# Output: gpurun_out/pmct/<shape>_<fetch|write>/ ; aggregate with tools/pmc_traffic.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPES=${1:-qkv_v,fc_v,out_v,proj_v,attn_v,ln_v}
OUT=${2:-gpurun_out/pmct}   # e.g. run with CE_GEMM_GROUPM=8 into another directory
mkdir -p $OUT
for s in ${SHAPES//,/ }; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/${s}_${c}
    timeout -k 10 180 rocprofv3 --kernel-trace --pmc $c -d $d -o run --output-format csv -- \
      python3 tools/bench_kernels.py --rounds 1 --reps 3 --warm-s 0 --scheds 1 --only $s > $d.log 2>&1
  done
done
