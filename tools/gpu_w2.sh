#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-w2}
S=${2:-1,12}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "test_gemm and 12" --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_kern.log 2>&1 && echo "kern ok" &&
timeout -k 10 400 python -u tools/bench_gemm_epi.py --scheds $S --rounds 2 --only qkv,out,fc,proj > gpurun_out/${T}_bench.log 2>&1 && echo "bench ok" && cat gpurun_out/${T}_bench.log
