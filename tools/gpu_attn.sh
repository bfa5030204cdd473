#!/bin/bash
# Attention-variant pass: kernel tests, kernel A/B, in-model A/B (same box).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-attn}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q --timeout 120 --timeout-method thread -k attention \
  > gpurun_out/${TAG}_pytest.log 2>&1; tail -3 gpurun_out/${TAG}_pytest.log;
timeout -k 10 240 python -u tools/bench_kernels.py --only attn_v,attn_t --attn-vars ${VARS:-0,1,2,5,9,13} --rounds 4 \
  > gpurun_out/${TAG}_kernels.log 2>&1 && echo "kernel ab ok" &&
for v in ${BVARS:-0 1 5 9 13}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --attn-var $v > gpurun_out/${TAG}_bench$v.log 2>&1 || exit 1
done
echo "bench ab ok" && tail -1 gpurun_out/${TAG}_bench*.log && cat gpurun_out/${TAG}_kernels.log
