#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (run_counter_collection.csv).

    python scripts/pmc_summary.py gpurun_out/pmc_dir [gpurun_out/pmc_dir2 ...] [--filter gemm]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if a.filter and a.filter not in name:
                    continue
                short = name.split("(")[0][-60:] + f" [g{r['Grid_Size']}]"
                vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
