#!/usr/bin/env python3
"""Single-frame latency through the seam (zw_encode_frame_lossy, 1080p RGBA Q75
m4) of the library ZWEBP_LIB names, with the row-parallel kernels' times.
usage: ZWEBP_LIB=... python tools/single_frame.py [reps]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.shard import frame_seed  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
w, h = 1920, 1080
ctx = zwebp.Context(0)
img = synth_rgba(w, h, frame_seed(0))
out = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
best = 1e9
for _ in range(reps):
    t0 = time.perf_counter()
    zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    best = min(best, time.perf_counter() - t0)
p = zwebp.Pipeline(1, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
p.upload(0, img)
p.run_device()
k = p.kernel_times()
o2 = p.output(0)
p.close()
with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
    want = json.load(f)["digests"].get(f"{w}x{h}/q75m4/{frame_seed(0):#010x}")
print(json.dumps({"lib": os.path.basename(os.environ.get("ZWEBP_LIB", "libzwebp.so")), "best_ms": best * 1e3,
                  "pass1_ms": k[2], "pass2_ms": k[3], "verified": hashlib.sha256(o2).hexdigest() == want,
                  "frame_bytes": len(out), "pipe_bytes": len(o2)}))
