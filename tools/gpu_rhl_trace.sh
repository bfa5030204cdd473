#!/bin/bash
# Per-tile timelines of the hi/lo residual GEMMs: SCHED 1 vs the staged-residual kernel (v131) with
# and without a de-synchronised start; then the A/B of the same tokens.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-rhlt}
S=${2:-1v3,1v131,1v131s4,1v131s8}
for sh in out_hl proj_hl; do
  timeout -k 10 200 python -u tools/gemm_trace.py --shape $sh --scheds $S > gpurun_out/${T}_${sh}.log 2>&1 || exit 1
  grep "==" gpurun_out/${T}_${sh}.log
done &&
timeout -k 10 300 python -u tools/bench_gemm_epi.py --only out_hl,proj_hl --scheds $S --rounds 3 \
  > gpurun_out/${T}_ab.log 2>&1 && echo "ab ok" && tail -1 gpurun_out/${T}_ab.log
