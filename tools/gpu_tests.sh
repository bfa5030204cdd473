#!/bin/bash
# Full GPU test suite (verbose on the files given first), one process, each step time-limited.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-t}
shift
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_new.log 2>&1 && echo "new ok" || { echo "new FAILED"; exit 1; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_all.log 2>&1 && echo "all ok"; tail -3 gpurun_out/${T}_all.log
