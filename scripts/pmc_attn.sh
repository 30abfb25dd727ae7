#!/bin/bash
# PMC counter passes over the flash-attention kernel at Whisper-small shapes (op_bench attn)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_attn_${i} -o run --output-format csv -- \
    python3 $R/scripts/op_bench.py attn --iters 5 > /dev/null 2>&1 || exit $?
done
python3 - <<'PY'
import csv, collections, glob, os
R = os.environ["GRAFT_REPO_ROOT"]
agg, n, dur = collections.defaultdict(float), collections.Counter(), []
for f in sorted(glob.glob(f"{R}/gpurun_out/pmc_attn_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "attn_fwd" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
        dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k in sorted(agg):
    print(f"{k:28s} {agg[k] / n[k]:.4g}")
print("dispatch us (median, under pmc):", sorted(dur)[len(dur) // 2])
PY
