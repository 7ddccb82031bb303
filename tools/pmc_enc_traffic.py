#!/usr/bin/env python3
"""Per-dispatch HBM traffic of the encode kernels from FETCH_SIZE / WRITE_SIZE passes.

usage: pmc_enc_traffic.py DIR FRAMES [WIDTH HEIGHT]
FETCH_SIZE / WRITE_SIZE are KiB summed over the device per dispatch; the gfx950
correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of wide
reads) doubles FETCH_SIZE, as tools/pmc_traffic.py does for k_xform_mb.  Per
kernel the median dispatch; units = the launch's MBs."""
import collections
import csv
import glob
import json
import statistics
import sys

root, frames = sys.argv[1], int(sys.argv[2])
w = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
h = int(sys.argv[4]) if len(sys.argv) > 4 else 1080
nmb = ((w + 15) // 16) * ((h + 15) // 16)
per = collections.defaultdict(float)  # (kernel, counter, dispatch) -> KiB
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("k_encode_pass"):
            continue
        per[(k, r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
out = {}
for k in sorted({x[0] for x in per}):
    fetch = [v for (kk, c, _), v in per.items() if kk == k and c == "FETCH_SIZE"]
    write = [v for (kk, c, _), v in per.items() if kk == k and c == "WRITE_SIZE"]
    if not fetch or not write:
        continue
    fk, wk = statistics.median(fetch), statistics.median(write)
    units = frames * nmb if k.endswith("_fp") else min(frames, 256) * nmb
    rb, wb = 2 * fk * 1024, wk * 1024
    out[k] = {"frames": frames, "units": units, "unit": "MB", "dispatches": len(fetch), "fetch_size_kib_raw": fk,
              "write_size_kib": wk, "hbm_read_bytes": rb, "hbm_write_bytes": wb, "traffic_bytes": rb + wb,
              "traffic_bytes_per_mb": (rb + wb) / units}
print(json.dumps(out, indent=1))
