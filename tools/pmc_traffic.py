#!/usr/bin/env python3
"""Per-dispatch HBM traffic of one kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE/WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the bytes
of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM/rocprofv3
section), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
usage: pmc_traffic.py DIR KERNEL_SUBSTRING FRAMES"""
import csv
import glob
import json
import statistics
import sys

root, kname, frames = sys.argv[1], sys.argv[2], int(sys.argv[3])
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    per = {}
    for r in csv.DictReader(open(f)):
        if kname not in r["Kernel_Name"] or r["Counter_Name"] not in vals:
            continue
        key = (r["Counter_Name"], r["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    for (c, _), v in per.items():
        vals[c].append(v)
fetch_kib = statistics.median(vals["FETCH_SIZE"])
write_kib = statistics.median(vals["WRITE_SIZE"])
blocks = frames * 8160 * 24
read_b, write_b = 2 * fetch_kib * 1024, write_kib * 1024
alg = blocks * 80
print(json.dumps({"kernel": kname, "frames": frames, "blocks": blocks, "dispatches": len(vals["FETCH_SIZE"]),
                  "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
                  "hbm_read_bytes": read_b, "hbm_write_bytes": write_b, "traffic_bytes": read_b + write_b,
                  "alg_bytes": alg, "traffic_over_alg": (read_b + write_b) / alg}, indent=1))
