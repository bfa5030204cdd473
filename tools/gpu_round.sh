#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, bench, rocprofv3 kernel stats.  Each step has its
# own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && echo "bench ok" &&
tail -1 gpurun_out/${TAG}_bench.log
