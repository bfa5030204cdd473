#!/bin/bash
# GPU tests, then in-model A/B of the hi/lo residual stream and the SCHED 11 split-K tail.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r02e}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/${T}_pytest.log &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_hl.log 2>&1 && tail -1 gpurun_out/${T}_bench_hl.log | cut -c1-200 &&
CE_RESID_HL=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_f32.log 2>&1 && tail -1 gpurun_out/${T}_bench_f32.log | cut -c1-200 &&
CE_GEMM_VARIANT=35 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_bench_tail.log 2>&1 && tail -1 gpurun_out/${T}_bench_tail.log | cut -c1-200
