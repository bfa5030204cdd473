#!/bin/bash
# Persistent-GEMM tests + A/B over all four vision GEMM shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-w4ab}
S=${2:-1a0,11v1,11v3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "persistent or (test_gemm and 11)" \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_kern.log 2>&1 && echo "kern ok" && tail -1 gpurun_out/${T}_kern.log &&
timeout -k 10 500 python -u tools/bench_gemm_epi.py --scheds $S --rounds 3 --only qkv,out,fc,proj > gpurun_out/${T}_bench.log 2>&1 &&
echo "bench ok" && tail -1 gpurun_out/${T}_bench.log
