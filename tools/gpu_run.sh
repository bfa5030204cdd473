#!/bin/bash
# One parameterised GPU-box pass.  Usage: tools/gpu_run.sh TAG STEP...  where STEP is one of
#   tests:<pytest args, comma-separated>   verbose pytest on the given files / -k filters
#   gputests                               the whole -m gpu suite
#   smoke                                  __graft_entry__.smoke()
#   bench:<bench.py args, comma-separated> one bench.py run (JSON line -> gpurun_out/TAG_benchN.log)
#   envbench:<VAR=VAL>,<bench.py args>    one bench.py run with one environment setting (A/B)
#   rocprof:<bench.py args>                rocprofv3 --kernel-trace --stats of one bench.py run
#   clock:<bench.py args>                  GRBM_GUI_ACTIVE pass (effective clock per kernel)
#   pmc:<counter>,<bench.py args>          one --pmc pass with one counter over a short bench run
#   pmcs:<c1+c2+...>,<bench.py args>       one --pmc pass with several counters (within one pass's limits)
#   py:<script>,<args>                     any python script (kernel A/B: tools/bench_gemm_epi.py,
#                                          tools/bench_kernels.py; timelines: tools/gemm_trace.py)
#   envpy:<VAR=VAL>,<script>,<args>        the same with one environment setting (e.g. CLIPEMBED_LIB=...)
# Every step has its own time limit; the chain stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  args=${arg//,/ }
  case $kind in
    tests)   timeout -k 10 900 python -u -m pytest $args -v --timeout 300 --timeout-method thread \
               > gpurun_out/${TAG}_tests$n.log 2>&1 ;;
    gputests) timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
               > gpurun_out/${TAG}_gputests.log 2>&1 ;;
    smoke)   timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1 ;;
    bench)   timeout -k 10 400 python -u bench.py $args > gpurun_out/${TAG}_bench$n.log 2>&1 ;;
    envbench) ev=${args%% *}; rest=${args#* }
             timeout -k 10 400 env $ev python -u bench.py $rest > gpurun_out/${TAG}_bench$n.log 2>&1 ;;
    rocprof) timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof$n -o run --output-format csv -- \
               python3 -u bench.py --no-cpu-baseline $args > gpurun_out/${TAG}_prof$n.log 2>&1 ;;
    clock)   timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/${TAG}_clk$n \
               -o run --output-format csv -- python3 -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-timing $args \
               > gpurun_out/${TAG}_clk$n.log 2>&1 ;;
    pmc)     cnt=${args%% *}; rest=${args#* }; [ "$rest" = "$args" ] && rest=""
             timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $cnt -d gpurun_out/${TAG}_pmc${n}_$cnt \
               -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing $rest \
               > gpurun_out/${TAG}_pmc${n}.log 2>&1 ;;
    pmcs)    cnt=${args%% *}; rest=${args#* }; [ "$rest" = "$args" ] && rest=""; cnt=${cnt//+/ }
             timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $cnt -d gpurun_out/${TAG}_pmcs$n \
               -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing $rest \
               > gpurun_out/${TAG}_pmcs${n}.log 2>&1 ;;
    py)      timeout -k 10 600 python -u $args > gpurun_out/${TAG}_py$n.log 2>&1 ;;
    envpy)   ev=${args%% *}; rest=${args#* }
             timeout -k 10 600 env $ev python -u $rest > gpurun_out/${TAG}_py$n.log 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "step $n $step: rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
