#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace: kernels (>= min ms) and GPU idle gaps.

usage: tools/trace_timeline.py kernel_trace.csv [t_from_ms t_to_ms] [min_ms]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = float(sys.argv[3]) if len(sys.argv) > 3 else 1e18
mn = float(sys.argv[4]) if len(sys.argv) > 4 else 0.1
end = None
busy = 0.0
for r in rows:
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    if not (lo <= s <= hi):
        continue
    if end is not None and s > end + 0.05:
        print(f"          ---- idle {s - end:7.3f} ms")
    if end is None or e > end:
        busy += e - max(s, end if end is not None else s)
        end = e
    if e - s >= mn:
        print(f"{s:9.3f} {e:9.3f} {e - s:8.3f} q{r['Queue_Id']:>3} {r['Kernel_Name'][:34]}")
print(f"busy {busy:.2f} ms")
