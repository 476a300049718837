#!/bin/bash
# Runs GPU steps one after the other on the box, each under its own time limit, and stops at the first
# step that timed out, aborted or crashed (exit status 124, 134, 137, 139 or above 128): an ordinary
# failure (a red test, status 1) does not stop the chain.
#   bash tools/gpu_steps.sh gpurun_out/TAG "name|seconds|command" ...
# Each step's output goes to OUT/name.log; OUT/steps.txt lists "name status seconds".
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  t0=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name $rc $(( $(date +%s) - t0 ))" >> "$OUT/steps.txt"
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then
    echo "stopping after $name (status $rc)" >> "$OUT/steps.txt"
    exit $rc
  fi
done
exit 0
