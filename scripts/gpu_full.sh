#!/bin/bash
# Full GPU pass without stopping at the first failing test: the suite (all failures listed),
# then smoke and the default bench (they run unless a step faulted / timed out).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_suite.log; grep -E "^FAILED|^ERROR" gpurun_out/gpu_suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
exit $rc
