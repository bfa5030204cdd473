#!/bin/bash
# Persistent-GEMM tests + per-tile timelines + epilogue A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-tr11}
S=${2:-11v1,11v3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "persistent or (test_gemm and 11)" \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_kern.log 2>&1 && echo "kern ok" && tail -1 gpurun_out/${T}_kern.log &&
for sh in fc fc_fold fc_plain; do
  timeout -k 10 200 python -u tools/gemm_trace.py --shape $sh --scheds $S > gpurun_out/${T}_${sh}.log 2>&1 || exit 1
  grep "==" gpurun_out/${T}_${sh}.log
done &&
timeout -k 10 400 python -u tools/bench_gemm_epi.py --scheds 1a0,$S --rounds 3 --only qkv,fc,fc_fold,fc_plain > gpurun_out/${T}_bench.log 2>&1 &&
echo "bench ok" && tail -1 gpurun_out/${T}_bench.log
