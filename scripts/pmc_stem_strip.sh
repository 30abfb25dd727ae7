#!/bin/bash
# PMC passes over one u8 stem variant: scripts/pmc_stem_strip.sh <variant>
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
V=${1:-2}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_stem${V}_${i} -o run --output-format csv -- \
    python3 $R/scripts/stem_pool_bench.py 256 u8v$V > /dev/null 2>&1 || exit $?
done
python3 - "$V" <<'PY'
import csv, collections, glob, os, sys
R = os.environ["GRAFT_REPO_ROOT"]
V = sys.argv[1]
agg, n, dur = collections.defaultdict(float), collections.Counter(), []
for f in sorted(glob.glob(f"{R}/gpurun_out/pmc_stem{V}_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "stem_pool" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:.4g}")
print("dispatch us (median, under pmc):", sorted(dur)[len(dur) // 2])
PY
