#!/usr/bin/env python3
"""Per-launch VALU-issue figures of the encode kernels from rocprofv3 --pmc passes.

usage: encode_pmc_summary.py DIR FRAMES [WIDTH HEIGHT]
Counters are summed over the device per dispatch (rocprofv3 aggregates the SE /
XCD instances); the median dispatch of each kernel is reported.
  valu_insts_per_mb  SQ_INSTS_VALU / MBs of the launch (wave64 instructions)
  kernel_cycles      GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs; MI355X_MICROARCH.md, DVFS item)
  dispatch_ms        End_Timestamp - Start_Timestamp of the same dispatch (pass 1 of the counters)
  clock_ghz          kernel_cycles / dispatch time: the clock the chip ran that dispatch at
  valu_issue_frac    SQ_INSTS_VALU / (kernel_cycles x 256 CUs x 2): the VALU issue peak is one
                     wave64 instruction per 2 cycles on each of a CU's 4 SIMD32
  valu_active_frac   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both quad-cycles): share of a wave's
                     lifetime in which it issued VALU
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

root, frames = sys.argv[1], int(sys.argv[2])
w = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
h = int(sys.argv[4]) if len(sys.argv) > 4 else 1080
nmb = ((w + 15) // 16) * ((h + 15) // 16)
per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, pass, dispatch) -> counter
span = {}  # (kernel, pass, dispatch) -> ns
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    pas = os.path.basename(os.path.dirname(os.path.relpath(f, root)).split(os.sep)[0] or "?")  # p1 / p2
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_encode_pass" not in k:
            continue
        key = (k.split("(")[0], pas, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            span[key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
out = {}
for kern in sorted({k for k, _, _ in per}):
    vals = collections.defaultdict(list)
    for (k, _, _), c in per.items():
        if k != kern:
            continue
        for name, v in c.items():
            vals[name].append(v)
    med = {n: statistics.median(v) for n, v in vals.items()}
    mbs = frames * nmb
    d = {"frames_per_launch": frames, "mbs_per_launch": mbs, "counters_median": med}
    if "SQ_INSTS_VALU" in med:
        d["valu_insts_per_mb"] = med["SQ_INSTS_VALU"] / mbs
        d["salu_insts_per_mb"] = med.get("SQ_INSTS_SALU", 0) / mbs
        d["lds_insts_per_mb"] = med.get("SQ_INSTS_LDS", 0) / mbs
    if "GRBM_GUI_ACTIVE" in med:
        cyc = med["GRBM_GUI_ACTIVE"] / 8
        d["kernel_cycles"] = cyc
        if "SQ_INSTS_VALU" in med:
            d["valu_issue_frac"] = med["SQ_INSTS_VALU"] / (cyc * 256 * 2)
        # the clock of the dispatches that carried SQ_INSTS_VALU and GRBM_GUI_ACTIVE together
        pairs = [(c["GRBM_GUI_ACTIVE"] / 8, span[key]) for key, c in per.items()
                 if key[0] == kern and "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c and span.get(key)]
        if pairs:
            d["dispatch_ms"] = statistics.median(t for _, t in pairs) / 1e6
            d["clock_ghz"] = statistics.median(cy / t for cy, t in pairs)
    if "SQ_ACTIVE_INST_VALU" in med and "SQ_WAVE_CYCLES" in med:
        d["valu_active_frac"] = med["SQ_ACTIVE_INST_VALU"] / med["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in med and "SQ_WAVE_CYCLES" in med:
        d["wait_any_frac"] = med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"]
        d["wait_inst_any_frac"] = med.get("SQ_WAIT_INST_ANY", 0) / med["SQ_WAVE_CYCLES"]
        d["active_inst_any_frac"] = med.get("SQ_ACTIVE_INST_ANY", 0) / med["SQ_WAVE_CYCLES"]
    out[kern] = d
print(json.dumps(out, indent=1))
