cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && for m in 0 1 2; do for l in 0 1; do timeout -k 10 120 tools/handout_probe $m $l 5000 2000 >> gpurun_out/r06j_handout.log 2>&1 || exit $?; done; done
