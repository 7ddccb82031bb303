#!/usr/bin/env python3
"""One-lane encode kernel times of the library ZWEBP_LIB names (for A/B runs):
KAB_FRAMES (256) 1080p frames per chunk, best of R runs (ms per launch).
usage: ZWEBP_LIB=... python tools/kab.py [R] [W H]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
os.environ["ZW_PIPE_LANES"] = "1"
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(os.environ.get("KAB_FRAMES", "256"))  # frames per launch (512: pass 2 in frame pairs)
os.environ.setdefault("ZW_PIPE_CHUNK", str(n))
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
ctx = zwebp.Context(0)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
for i in range(n):
    p.upload(i, imgs[i % 4])
p.run_device()
best = None
for _ in range(R):
    p.run_device()
    k = p.kernel_times()
    best = list(k[:4]) if best is None else [min(a, b) for a, b in zip(best, k[:4])]
p.encode()
import hashlib  # noqa: E402
dig = hashlib.sha256(b"".join(p.output(i) for i in range(4))).hexdigest()[:16]
print(json.dumps({"lib": os.path.basename(os.environ.get("ZWEBP_LIB", "libzwebp.so")), "size": f"{w}x{h}", "rgb2yuv": best[0],
                  "analysis": best[1], "pass1": best[2], "pass2": best[3], "digest4": dig}), flush=True)
