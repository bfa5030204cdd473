#!/bin/bash
# GEMM A/B on the GPU box: persistent-GEMM tests, then bench_gemm_epi over the given schedule tokens.
#   bash tools/gpu_epi_ab.sh <tag> <sched tokens> [shapes]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-ab}
S=${2:-1a0,11v0,11v1}
O=${3:-qkv,out,fc,proj,fc_plain}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "persistent or (test_gemm and 11)" \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_kern.log 2>&1 && echo "kern ok" && tail -1 gpurun_out/${T}_kern.log &&
timeout -k 10 400 python -u tools/bench_gemm_epi.py --scheds $S --rounds 3 --only $O > gpurun_out/${T}_bench.log 2>&1 &&
echo "bench ok" && cat gpurun_out/${T}_bench.log
