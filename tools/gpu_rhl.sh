#!/bin/bash
# Staged-residual four-wave kernel (variant bit 128) for the hi/lo residual GEMMs: kernel tests, then
# A/B vs SCHED 1 at the bench shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-rhl}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "ln_stats_hl" -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 && echo "pytest ok" && tail -3 gpurun_out/${TAG}_pytest.log &&
timeout -k 10 300 python -u tools/bench_gemm_epi.py --only out_hl,proj_hl --scheds 1v3,1v131 --rounds 3 \
  > gpurun_out/${TAG}_ab.log 2>&1 && echo "ab ok" && cat gpurun_out/${TAG}_ab.log
