#!/bin/bash
# Round-2 first GPU pass: the new bench-path tests first (verbose), then the whole GPU suite, then the
# benchmark legs.  Every GPU step has its own limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-r02a}
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_path.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/${T}_benchpath.log 2>&1 && echo "benchpath ok" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 && echo "pytest ok" &&
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 && echo "bench ok" && tail -1 gpurun_out/${T}_bench.log &&
timeout -k 10 300 python -u bench.py --workload pacl --no-cpu-baseline --steps 5 > gpurun_out/${T}_pacl.log 2>&1 && echo "pacl ok" &&
timeout -k 10 300 python -u bench.py --workload sparc --no-cpu-baseline --steps 5 > gpurun_out/${T}_sparc.log 2>&1 && echo "sparc ok" &&
timeout -k 10 300 python -u bench.py --workload negclip --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${T}_negclip.log 2>&1 && echo "negclip ok"
