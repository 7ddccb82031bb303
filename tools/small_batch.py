#!/usr/bin/env python3
"""Small-batch encode latency: batch kernels (one 12-wave workgroup per frame)
against the row-parallel kernels (one wave per MB row), per batch size.

usage: tools/small_batch.py [w h] [sizes, comma-separated]
Prints one JSON line per (n, rows): wall ms per batch (encode + outputs) and
the pass-1 / pass-2 kernel ms of the last batch.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

w = int(sys.argv[1]) if len(sys.argv) > 1 else 1920
h = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
sizes = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8,16,32").split(",")]
ctx = zwebp.Context(0)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
for n in sizes:
    for rows in ("0", "1"):
        os.environ["ZW_ENC_ROWS"] = rows
        p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
        for i in range(n):
            p.upload(i, imgs[i % 4])
        p.encode()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            p.encode()
            for i in range(n):
                p.output(i)
        ms = (time.perf_counter() - t0) / reps * 1e3
        k = p.kernel_times()
        outs = [p.output(i) for i in range(min(n, 4))]
        p.close()
        print(json.dumps({"w": w, "h": h, "n": n, "rows": int(rows), "wall_ms": round(ms, 2),
                          "encodes_per_s": round(n / ms * 1e3, 1), "pass1_ms": round(k[2], 2),
                          "pass2_ms": round(k[3], 2), "analysis_ms": round(k[1], 2),
                          "out_bytes": [len(o) for o in outs]}), flush=True)
os.environ.pop("ZW_ENC_ROWS", None)
