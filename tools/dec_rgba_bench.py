#!/usr/bin/env python3
"""Decode batches to YUV planes and to packed RGBA (256 1080p frames): wall
time per batch; with ZW_DEC_TIMING=1 the library prints per-chunk host phases."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
w, h = 1920, 1080
ctx = zwebp.Context(0)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
streams = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
vp8 = [streams[i % 4] for i in range(F)]
import numpy as np  # noqa: E402
bufs = [np.empty(w * h * 4, np.uint8) for _ in range(F)]
for name, fn in (("rgba_into", lambda: zwebp.decode_rgb_batch_into(vp8, bufs, 4, ctx=ctx)),
                 ("yuv", lambda: zwebp.decode_batch(vp8, ctx=ctx)),
                 ("rgba", lambda: zwebp.decode_rgb_batch(vp8, bpp=4, ctx=ctx)),
                 ("rgb", lambda: zwebp.decode_rgb_batch(vp8, bpp=3, ctx=ctx))):
    fn()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        out = fn()
        best = min(best, time.perf_counter() - t0)
        del out
    print(f"{name}: {F} frames {best * 1e3:.1f} ms = {F / best:.0f} decodes/s", flush=True)
