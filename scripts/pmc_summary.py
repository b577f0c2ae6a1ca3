#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel (name prefix) and counter, the mean
over dispatches of the per-dispatch sum across dimensions.  Usage: pmc_summary.py DIR [DIR...]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    for d in sys.argv[1:]:
        per = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r.get("Kernel_Name", "?")[:70]
                    per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        print(f"== {d}")
        for k, cs in per.items():
            n = max(1, len(disp[k]))
            if "gemm" not in k and "Cijk" not in k:
                continue
            print(f"  {k} ({n} dispatches)")
            for c, v in sorted(cs.items()):
                print(f"    {c:28s} {v / n:16.0f}")


if __name__ == "__main__":
    main()
