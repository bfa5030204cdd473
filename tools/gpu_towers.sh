#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-tw}
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_conc.log 2>&1 && tail -1 gpurun_out/${T}_conc.log | cut -c1-160 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --serial-towers > gpurun_out/${T}_serial.log 2>&1 && tail -1 gpurun_out/${T}_serial.log | cut -c1-160 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${T}_conc2.log 2>&1 && tail -1 gpurun_out/${T}_conc2.log | cut -c1-160
