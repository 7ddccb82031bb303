#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc counter_collection.csv files per kernel (sum over dispatches)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
ndisp = collections.defaultdict(set)
for f in sorted(glob.glob(f"{root}/p*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        ndisp[k].add((f, r["Dispatch_Id"]))
for k, v in agg.items():
    if "rocclr" in k:
        continue
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:.4g}")
    if "SQ_INSTS_VALU" in v and "SQ_BUSY_CYCLES" in v:
        pass
