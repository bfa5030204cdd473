#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-tw}
for r in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_conc$r.log 2>&1 && tail -1 gpurun_out/${T}_conc$r.log | cut -c1-120 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --tower-priority > gpurun_out/${T}_prio$r.log 2>&1 && tail -1 gpurun_out/${T}_prio$r.log | cut -c1-120 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --serial-towers > gpurun_out/${T}_serial$r.log 2>&1 && tail -1 gpurun_out/${T}_serial$r.log | cut -c1-120 || exit 1
done
