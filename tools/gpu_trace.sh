#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-tr}
timeout -k 10 200 python -u tools/gemm_trace.py --shape out --scheds 1,1s4,12,12s2 > gpurun_out/${T}_out.log 2>&1 && echo "out ok" &&
timeout -k 10 200 python -u tools/gemm_trace.py --shape fc --scheds 1,12 > gpurun_out/${T}_fc.log 2>&1 && echo "fc ok"
