cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "splitk or test_gemm" > gpurun_out/t_split.log 2>&1 &&
timeout -k 10 300 python3 tools/bench_kernels.py --scheds 1,1n --rounds 3 --only qkv_v,fc_v,out_v,proj_v > gpurun_out/abl_split.log 2>&1 &&
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/b_split.log 2>&1
