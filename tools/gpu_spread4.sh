#!/bin/bash
# DMA split A/B (10+6 default vs 12+4 vs 8+8) on the four-wave persistent GEMM + in-model.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-spread3}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -k "persistent" \
  > gpurun_out/${TAG}_pytest.log 2>&1; tail -2 gpurun_out/${TAG}_pytest.log; grep -q " passed" gpurun_out/${TAG}_pytest.log || exit 1
grep -q "failed" gpurun_out/${TAG}_pytest.log && exit 1
timeout -k 10 300 python -u tools/bench_gemm_epi.py --only qkv,fc --scheds 11v899,11v4995 --rounds 4 \
  > gpurun_out/${TAG}_gemm.log 2>&1 && echo "gemm ab ok" && tail -1 gpurun_out/${TAG}_gemm.log &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_def.log 2>&1 &&
CE_GEMM_VARIANT=4995 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench_4995.log 2>&1 &&
echo "bench ab ok" && tail -1 gpurun_out/${TAG}_bench_def.log
