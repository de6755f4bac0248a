#!/bin/bash
# Run GPU steps in sequence on the gpurun box; each step has its own time limit.
# A step that ends in a fault (abort 134, segfault 139, timeout 124/137, or any
# signal) stops the session: nothing else touches the GPU after it.  Ordinary
# failures (e.g. pytest rc=1) are recorded and the session continues.
#   usage: tools/gpu_steps.sh "<secs>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 4 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) [ $rc -ne 0 ] && status=$rc ;;
    *) echo "=== [$name] ended abnormally (rc=$rc): stopping the session"; exit $rc ;;
  esac
done
exit $status
