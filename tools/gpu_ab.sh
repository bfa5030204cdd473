#!/bin/bash
# bench_gemm_epi A/B only: bash tools/gpu_ab.sh <tag> <sched tokens> <shapes> [rounds]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_gemm_epi.py --scheds $2 --rounds ${4:-3} --only $3 > gpurun_out/$1_bench.log 2>&1 &&
echo "bench ok" && tail -1 gpurun_out/$1_bench.log
