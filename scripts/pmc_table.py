#!/usr/bin/env python3
"""Markdown table of rocprofv3 --pmc passes (scripts/pmc_bench.sh) for the top kernels:
per (kernel, grid) — dispatches, mean duration (serialised under --pmc), MFMA busy share,
LDS bank-conflict rate, HBM fetch / write (FETCH_SIZE / WRITE_SIZE, KB) and the bandwidth
they imply.

    python scripts/pmc_table.py gpurun_out/pmcb_r2_1 ... [--top 12] [--clock-ghz 2.4]
MFMA busy share = SQ_VALU_MFMA_BUSY_CYCLES / (duration cycles x 256 CUs x 4 SIMDs)."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--lds", action="store_true",
                    help="add LDS-array utilisation (SQ_LDS_IDX_ACTIVE / (cycles x 256 CUs)) and per-wave counts")
    a = ap.parse_args()
    cnt = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                key = (name[-58:], int(r["Grid_Size"]))
                cnt[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[key][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    rows = []
    for key, cs in cnt.items():
        ds = list(dur[key].values())
        us = sum(ds) / len(ds)
        calls = max(len(v) for v in cs.values())
        m = lambda c: (sum(cs[c]) / len(cs[c])) if cs.get(c) else float("nan")  # noqa: E731
        cyc = us * 1e-6 * a.clock_ghz * 1e9
        mfma = m("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024) if cyc else float("nan")
        conf = m("SQ_LDS_BANK_CONFLICT") / m("SQ_LDS_IDX_ACTIVE") if m("SQ_LDS_IDX_ACTIVE") else 0.0
        fetch, write = m("FETCH_SIZE"), m("WRITE_SIZE")
        bw = (fetch + write) * 1e3 / (us * 1e-6) / 1e12 if us else float("nan")
        waves = max(1.0, m("SQ_WAVES")) if cs.get("SQ_WAVES") else float("nan")
        extra = (m("SQ_LDS_IDX_ACTIVE") / (cyc * 256) if cyc else float("nan"),
                 m("SQ_INSTS_LDS") / waves, m("SQ_INSTS_MFMA") / waves, m("SQ_INSTS_VALU") / waves)
        rows.append((us * calls, key, calls, us, mfma, conf, fetch / 1e3, write / 1e3, bw,
                     m("SQ_INSTS_VALU") / max(1.0, m("SQ_INSTS_MFMA")), extra))
    rows.sort(reverse=True)
    hdr = "| kernel | grid | n | us | MFMA busy | LDS conflict | fetch MB | write MB | TB/s | VALU/MFMA |"
    if a.lds:
        hdr += " LDS active | LDS/wave | MFMA/wave | VALU/wave |"
    print(hdr)
    print("|---" * (hdr.count("|") - 1) + "|")
    for tot, (name, grid), n, us, mf, cf, fe, wr, bw, vm, ex in rows[:a.top]:
        line = f"| `{name}` | {grid} | {n} | {us:.1f} | {mf:.2f} | {cf:.3f} | {fe:.1f} | {wr:.1f} | {bw:.2f} | {vm:.2f} |"
        if a.lds:
            line += f" {ex[0]:.2f} | {ex[1]:.0f} | {ex[2]:.0f} | {ex[3]:.0f} |"
        print(line)


if __name__ == "__main__":
    main()
