#!/bin/bash
# PMC passes over the kernel micro-benchmark (one counter group per rocprofv3 run, --kernel-trace
# only; never combined with sys/runtime tracing).  Output: ${PMCDIR:-gpurun_out/pmc}/<pass>/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ONLY=${1:-qkv_v,fc_v,out_v,proj_v,attn_v}
run() {
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc "$@" -d ${PMCDIR:-gpurun_out/pmc}/$name -o run --output-format csv -- \
    python3 tools/bench_kernels.py --rounds 1 --reps 2 --warm-s 0 --scheds ${SCHEDS:-1} --attn-vars ${ATTN_VARS:-381} --only "$ONLY" > ${PMCDIR:-gpurun_out/pmc}/$name.log 2>&1
}
mkdir -p ${PMCDIR:-gpurun_out/pmc}
timeout -k 10 60 rocprofv3 -L > ${PMCDIR:-gpurun_out/pmc}/counters.txt 2>&1 || true
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run l2 TCC_HIT_sum TCC_MISS_sum
