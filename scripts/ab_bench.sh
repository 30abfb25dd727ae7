#!/bin/bash
# A/B the headline bench on ONE box: each arm runs bench.py in its own process with an env
# override, arms interleaved twice.  usage: scripts/ab_bench.sh "NAME:ENV=V ENV2=V" ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for round in 1 2; do
  for arm in "$@"; do
    name="${arm%%:*}"; envs="${arm#*:}"
    out=$(env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 8 2>/dev/null | tail -1) || exit $?
    v=$(echo "$out" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
    echo "round $round $name: $v"
  done
done
