#!/bin/bash
# conv variants per layer: scripts/conv_cmp.sh "layers" "tiles"
for l in ${1//,/ }; do
  for t in $2; do echo -n "$t "; python scripts/layer_bench.py --layers $l --tile $t --iters 20 2>&1 | grep -v amdgpu.ids || exit $?; done
done
