set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python3 -u scripts/model_layers.py --batch 320 > $O/layers_resnet50.txt 2>&1 || { tail -5 $O/layers_resnet50.txt; exit 1; }
tail -3 $O/layers_resnet50.txt
