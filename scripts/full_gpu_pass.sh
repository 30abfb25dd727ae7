#!/bin/bash
# The driver's round-end GPU tiers in one call: every GPU test (one process, per-test timeout),
# smoke(), then the headline bench in the driver's shape.  Output under gpurun_out/full/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/full
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
tail -1 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-300
exit $rc
