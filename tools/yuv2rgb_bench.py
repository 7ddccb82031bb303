#!/usr/bin/env python3
"""k_yuv2rgb (fancy upsampling, RGBA) timing on 256 decoded 1080p frames:
the library's kernel time over the batch's chunks, best of 3, and the HBM
fraction at 5.5 algorithmic bytes per pixel (Y 1 + U, V 0.5 read, RGBA 4 written)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import numpy as np  # noqa: E402
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

F, w, h = 256, 1920, 1080
ctx = zwebp.Context(0)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
streams = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
vp8 = [streams[i % 4] for i in range(F)]
bufs = [np.empty(w * h * 4, np.uint8) for _ in range(F)]
zwebp.decode_rgb_batch_into(vp8, bufs, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
ref = [bufs[i].copy() for i in range(4)]
best = 1e9
for _ in range(3):
    zwebp.decode_rgb_batch_into(vp8, bufs, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    best = min(best, zwebp.decode_rgb_kernel_ms(ctx=ctx))
same = all(np.array_equal(bufs[i], ref[i % 4]) for i in range(F))
gbs = 5.5 * w * h * F / (best * 1e-3) / 1e9
print(f"k_yuv2rgb RGBA fancy: {F} frames {best:.3f} ms = {gbs:.0f} GB/s = {gbs / 8000:.3f} of 8 TB/s; stable {same}")
