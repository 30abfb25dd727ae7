# Infinity-Cache blocking sweep for the ResNet-50 bench (AIKO_RESNET_MALL_CHUNK / _BLOCKS);
# usage: bash scripts/mall_experiment.sh [extra bench args]
set -o pipefail
mkdir -p gpurun_out
run() { echo "== $* $EXTRA" >> gpurun_out/mall.log; env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 6 $EXTRA >> gpurun_out/mall.log 2>&1; }
EXTRA="$*"
run AIKO_RESNET_MALL_CHUNK=0 && run AIKO_RESNET_MALL_CHUNK=64 AIKO_RESNET_MALL_BLOCKS=3 && run AIKO_RESNET_MALL_CHUNK=32 AIKO_RESNET_MALL_BLOCKS=3 && run AIKO_RESNET_MALL_CHUNK=64 AIKO_RESNET_MALL_BLOCKS=7 && run AIKO_RESNET_MALL_CHUNK=128 AIKO_RESNET_MALL_BLOCKS=3 && run AIKO_RESNET_MALL_CHUNK=128 AIKO_RESNET_MALL_BLOCKS=7
