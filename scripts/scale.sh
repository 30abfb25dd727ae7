#!/bin/bash
# Scaling sweep of BASELINE configs 2, 3 and 4 on one node (1/2/4/8 GPUs, one rank per GPU via
# torch.distributed.run over RCCL).  Emits one SCALE-format JSON object per config on stdout:
#   {"config": "...", "runs": [<bench.py line for N=1>, ... N=8], "efficiency": {N: value_N / (N * value_1)}}
# config 2 (ResNet-50 DP) and 4 (YOLOv8-n DP) are weak scaling, config 3 (ResNet-50 actor
# pipeline, balanced stages + replicas) strong scaling: efficiency is then value_N / value_1 / N.
#   bash scripts/scale.sh [max_gpus] > gpurun_out/scale.jsonl
MAX=${1:-8}
STEPS=${STEPS:-30}
WARMUP=${WARMUP:-8}
run() {   # $1 = n, rest = bench args
  local n=$1; shift
  local port=$((29500 + RANDOM % 1000))
  if [ "$n" = 1 ]; then
    timeout -k 10 300 python3 bench.py --gpus 1 --steps $STEPS --warmup $WARMUP "$@" 2>/dev/null | grep '^{'
  else
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n --steps $STEPS --warmup $WARMUP "$@" 2>/dev/null | grep '^{'
  fi
}
for cfg in "config2-resnet50-dp|" "config3-resnet50-pp|--parallel pp" "config4-yolov8n-dp|--model yolov8n"; do
  name=${cfg%%|*}; args=${cfg#*|}
  lines=()
  for n in 1 2 4 8; do
    [ $n -gt $MAX ] && break
    l=$(run $n $args) || { echo "{\"config\": \"$name\", \"error\": \"N=$n failed\"}"; break; }
    lines+=("$l")
  done
  python3 - "$name" "${lines[@]}" <<'PY'
import json, sys
name, runs = sys.argv[1], [json.loads(l) for l in sys.argv[2:]]
base = runs[0]["value"] if runs else None
eff = {r["n_gpus"]: round(r["value"] / (r["n_gpus"] * base), 4) for r in runs} if base else {}
print(json.dumps({"config": name, "runs": runs, "efficiency": eff}))
PY
done
