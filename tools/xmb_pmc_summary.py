#!/usr/bin/env python3
"""Per-kernel summary of tools/gpu_pmc_xmb.sh's rocprofv3 passes: median per
dispatch of every counter (summed over XCDs), kernel-trace average duration,
and the HBM traffic per MB (FETCH_SIZE doubled for the wide streaming reads,
MI355X_MICROARCH.md HBM section; WRITE_SIZE as is; both KiB).
usage: xmb_pmc_summary.py DIR [KERNEL_SUBSTRING [UNITS]]  ->  JSON on stdout
(defaults: xform_mb, 256 x 8160 MBs; tools/gpu_pmc_dec.sh passes dec_recon|loopfilter)"""
import collections
import csv
import glob
import json
import statistics
import sys

root = sys.argv[1]
MBS = int(sys.argv[3]) if len(sys.argv) > 3 else 256 * 8160  # the xmb_bench launch: 256 1080p frames
PATS = (sys.argv[2] if len(sys.argv) > 2 else "xform_mb").split("|")


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n


per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/*/*counter_collection.csv")):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        acc[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in acc.items():
        per[k][c].append(v)
dur = {}
for f in glob.glob(f"{root}/trace/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        dur[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
out = {}
for k, cs in per.items():
    if not any(p in k for p in PATS):
        continue
    d = {c: statistics.median(v) for c, v in cs.items()}
    e = {"counters_median_per_dispatch": d, "trace": dur.get(k)}
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        rd, wr = 2 * d["FETCH_SIZE"] * 1024, d["WRITE_SIZE"] * 1024
        e.update({"hbm_read_bytes": rd, "hbm_write_bytes": wr, "traffic_bytes": rd + wr, "units": MBS,
                  "traffic_bytes_per_mb": (rd + wr) / MBS})
    if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
        e["valu_insts_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        e["valu_insts_per_unit"] = d["SQ_INSTS_VALU"] / MBS
    out[k] = e
json.dump(out, sys.stdout, indent=1)
