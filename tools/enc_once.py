#!/usr/bin/env python3
"""Encode a batch once (after one warm-up encode) -- a small target for rocprofv3 runs."""
import os

# Two pipeline lanes x (kernel + copy stream) plus the runtime's own streams:
# ask HIP for 8 hardware queues (default 4) so no two busy streams share one.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
p = zwebp.Pipeline(F, w, h, zwebp.ColorType.Rgba8, 75, 4)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
for i in range(F):
    p.upload(i, imgs[i % 4])
p.encode()
p.encode()
print("kernel ms", p.kernel_times())
