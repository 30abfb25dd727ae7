#!/bin/bash
# PMC counter passes over any python command:  scripts/pmc_cmd.sh <tag> <kernel substring> <python args...>
#   -> gpurun_out/pmccmd_<tag>.txt (mean per matching dispatch; SQ_*CYCLES in quad-cycles)
tag=$1; kname=$2; shift 2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE TCP_TCC_READ_REQ_sum" "WRITE_SIZE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmccmd_${tag}_${i} -o run --output-format csv -- \
    python3 "$@" > /dev/null 2>&1 || exit $?
done
KN="$kname" TAG="$tag" python3 - <<'PY' | tee $R/gpurun_out/pmccmd_${tag}.txt
import csv, collections, glob, os
R, kn, tag = os.environ["GRAFT_REPO_ROOT"], os.environ["KN"], os.environ["TAG"]
agg, n, dur = collections.defaultdict(float), collections.Counter(), []
for f in sorted(glob.glob(f"{R}/gpurun_out/pmccmd_{tag}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kn not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
g = {k: agg[k] / n[k] for k in agg}
print(f"# {tag}: kernels matching '{kn}', mean per dispatch")
for k in sorted(g):
    print(f"{k:28s} {g[k]:.4g}")
if dur:
    d = sorted(dur)[len(dur) // 2]
    print("dispatch us (median, under pmc):", d)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in g:
        print("MFMA busy vs 1024 SIMDs x duration @2.4GHz:", round(g["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * d * 2400), 3))
    if "SQ_WAIT_INST_ANY" in g and "SQ_WAVE_CYCLES" in g:
        print("wait share of wave time:", round(g["SQ_WAIT_INST_ANY"] / g["SQ_WAVE_CYCLES"], 3))
PY
