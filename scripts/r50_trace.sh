#!/bin/bash
# ResNet-50 kernel traces at batch $1 (default 320): tiles tuned once, then (a) a one-lane eager
# trace whose last forward is listed kernel by kernel (isolated per-launch times) and (b) the
# two-lane trace of the default shape.  Output under gpurun_out/r50trace_<tag>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B=${1:-320}; TAG=${2:-r4}
O=$R/gpurun_out/r50trace_$TAG
mkdir -p $O
timeout -k 10 200 python $R/scripts/r50_profile.py --batch $B --tune $O/tiles.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/l1 -o run -- python3 $R/scripts/r50_profile.py --batch $B --load $O/tiles.json --iters 6 --lanes 1 > $O/l1.log 2>&1 || { tail -20 $O/l1.log; exit 1; }
db=$(find $O/l1 -name "*.db" | head -1)
python3 $R/scripts/rocprof_summary.py "$db" --sequence 75 > $O/seq_l1.md 2>&1
tail -3 $O/seq_l1.md
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/l2 -o run -- python3 $R/scripts/r50_profile.py --batch $B --load $O/tiles.json --iters 20 --lanes 2 > $O/l2.log 2>&1 || { tail -20 $O/l2.log; exit 1; }
grep "frames/s" $O/l1.log $O/l2.log
db=$(find $O/l2 -name "*.db" | head -1)
python3 $R/scripts/rocprof_summary.py "$db" > $O/summary_l2.md 2>&1
rm -rf $O/l1 $O/l2
exit 0
