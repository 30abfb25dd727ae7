#!/bin/bash
# PMC counter passes over one op of scripts/op_bench.py:
#   scripts/pmc_op.sh <op> <tile "bm,bn,v" | -> <kernel-name substring> <tag>  -> gpurun_out/pmcop_<tag>.txt
op=$1; tile=$2; kname=$3; tag=$4
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
targ=""; [ "$tile" != "-" ] && targ="--tile $tile"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE TCP_TCC_READ_REQ_sum" "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcop_${tag}_${i} -o run --output-format csv -- \
    python3 $R/scripts/op_bench.py $op $targ --iters 5 --reps 1 > /dev/null 2>&1 || exit $?
done
KN="$kname" TAG="$tag" python3 - <<'PY' | tee $R/gpurun_out/pmcop_${tag}.txt
import csv, collections, glob, os
R, kn, tag = os.environ["GRAFT_REPO_ROOT"], os.environ["KN"], os.environ["TAG"]
agg, n, dur = collections.defaultdict(float), collections.Counter(), []
for f in sorted(glob.glob(f"{R}/gpurun_out/pmcop_{tag}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kn not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
print(f"# {tag}: kernels matching '{kn}', mean per dispatch")
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:.4g}")
if dur:
    print("dispatch us (median, under pmc):", sorted(dur)[len(dur) // 2])
g = {k: agg[k] / n[k] for k in agg}
if "SQ_VALU_MFMA_BUSY_CYCLES" in g and "GRBM_GUI_ACTIVE" in g:
    print("MFMA busy (MFMA_BUSY / (GUI_ACTIVE * CUs 256)):", g["SQ_VALU_MFMA_BUSY_CYCLES"] / (g["GRBM_GUI_ACTIVE"] * 256))
PY
