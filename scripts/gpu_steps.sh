#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that times out,
# aborts or crashes (124 / 134 / 137 / 139 / >128) — ordinary test failures (rc 1) continue.
# usage: scripts/gpu_steps.sh <secs> "<cmd>" [<secs> "<cmd>" ...]   (logs: gpurun_out/steps.log)
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  secs=$1; cmd=$2; shift 2
  echo "=== [$(date +%T)] $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ge 124 ]; then
    echo "stopping: step rc=$rc" >> gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
