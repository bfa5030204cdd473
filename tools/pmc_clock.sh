#!/bin/bash
# Effective clock per kernel under the bench step (MI355X_MICROARCH.md 'DVFS give-back': clock ~
# GRBM_GUI_ACTIVE / 8 / kernel wall time), one rocprofv3 --pmc pass.  Args: TAG [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-clk}; shift
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG} -o run --output-format csv -- \
  python3 -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-timing "$@" > gpurun_out/${TAG}.log 2>&1
