#!/bin/bash
# In-model A/B: default GEMM variant bits vs + split-K tail on the four-wave schedule (bit 5).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-tail}
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_def1.log 2>&1 &&
CE_GEMM_VARIANT=931 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_931a.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_def2.log 2>&1 &&
CE_GEMM_VARIANT=931 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_931b.log 2>&1 &&
echo "tail ab ok"
