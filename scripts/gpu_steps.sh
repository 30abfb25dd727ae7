#!/bin/bash
# Run GPU steps in sequence on the gpurun box; each step has its own time limit.
# A step that faults / aborts / times out (124 134 137 139) ends the whole job: nothing
# more touches the GPU after that.  Ordinary failures (e.g. a failing test) continue.
# usage: scripts/gpu_steps.sh "SECONDS|name|command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== step $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== step $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139) echo "=== fatal rc=$rc in $name: stopping"; exit $rc;;
  esac
done
exit 0
