#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports that NOTHING ran (no box / no
# slot / back-off: gpurun's status=transient, nothing charged).  A call that ran, whatever
# its exit status, is never repeated.  Usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient" "$out"; then
    w=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-120} > 60 ? ${w:-120} : 60 ))
    continue
  fi
  exit $rc
done
exit 3
