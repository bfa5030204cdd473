#!/bin/bash
# Round-2 GPU pass: GPU parity tests, bench (clip), rocprofv3 kernel stats of the bench.
# Each step has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-r02c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/${TAG}_pytest.log &&
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 && echo "bench ok" &&
tail -1 gpurun_out/${TAG}_bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 && echo "prof ok"
