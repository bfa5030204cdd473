cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 300 env CLIPEMBED_LIB=$PWD/gpurun_ab/libclipembed_a7b4537.so python -u bench.py --no-cpu-baseline > gpurun_out/r05aj_old1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r05aj_new1.log 2>&1 && \
timeout -k 10 300 env CLIPEMBED_LIB=$PWD/gpurun_ab/libclipembed_a7b4537.so python -u bench.py --no-cpu-baseline > gpurun_out/r05aj_old2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r05aj_new2.log 2>&1
