#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_hop_engine.py tests/test_gpu_transformer.py -k "hop_engine or whisper_small or world1" -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --parallel pp --steps 20 --warmup 5 --write-element-times $O/element_times.json > $O/pp.log 2>&1 || { tail -20 $O/pp.log; exit 1; }
tail -1 $O/pp.log | cut -c1-300; cat $O/element_times.json
