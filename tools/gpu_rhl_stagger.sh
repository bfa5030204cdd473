#!/bin/bash
# First-round stagger sweep of the staged-residual kernel (hi/lo residual GEMMs at B = 256).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-rhls}
timeout -k 10 400 python -u tools/bench_gemm_epi.py --only out_hl,proj_hl --scheds ${2:-1v131,1v131s2,1v131s4,1v131s6,1v131s8,1v131s12,1v131s16} --rounds 3 \
  > gpurun_out/${T}_ab.log 2>&1 && echo "ab ok" && cat gpurun_out/${T}_ab.log
