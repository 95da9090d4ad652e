#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool answers "no slot / no box free" (exit 3 or a
# transient status: nothing ran, nothing was charged).  Any other outcome -- success or a failing GPU
# step -- ends it; a failing GPU command is never re-run.
#   tools/gpurun_queue.sh OUT_FILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "nothing was charged" "$out"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
