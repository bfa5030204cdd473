#!/bin/bash
# Staged-residual kernel tests + A/B (hi/lo residual GEMMs, c_fc with the GELU epilogue).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-rhl}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "ln_stats_hl or persistent or (test_gemm and gelu)" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 && echo "pytest ok" && tail -1 gpurun_out/${T}_pytest.log &&
timeout -k 10 400 python -u tools/bench_gemm_epi.py --only out_hl,proj_hl,fc,qkv --scheds 1v3,1v131 --rounds 3 \
  > gpurun_out/${T}_ab.log 2>&1 && echo "ab ok" && tail -1 gpurun_out/${T}_ab.log &&
timeout -k 10 200 python -u tools/gemm_trace.py --shape out_hl --scheds 1v131,1v135,1v139 > gpurun_out/${T}_trace.log 2>&1 && grep "==" gpurun_out/${T}_trace.log
