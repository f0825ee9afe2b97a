#!/bin/bash
# Run GPU steps in order, each under its own time limit, logs under gpurun_out/<tag>/ (dev tool).
# A step's failure with an ordinary exit status (1: test failures) lets the next step run; a time
# limit, abort, segfault or kill (124, 134, 137, 139, >128) ends the call there.
#   tools/gpu_steps.sh TAG "name|seconds|command" ...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - start )) s"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
