#!/usr/bin/env python3
"""Host-resident (PCIe-inclusive) encode rate: zw_pipe_encode_host over 1024
1080p frames x 3 batches, pageable frames and pinned frames, per uploader count.
usage: python tools/host_res.py [frames] [batches] [hip]
Legs: RGBA frames packed to RGB on the host (ZW_UPLOAD_PACK=1, the default) or sent as RGBA."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 3
w, h = 1920, 1080
torch.zeros(1, device="cuda")
ctx = zwebp.Context(0)
imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
p = zwebp.Pipeline(F, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
for i in range(F):
    p.upload(i, imgs[i % 4])
p.encode_repeat(1)
t0 = time.perf_counter()
p.encode_repeat(NB)
print(f"device-resident: {F * NB / (time.perf_counter() - t0):.0f} encodes/s", flush=True)
pageable = [np.array(imgs[i % 4], copy=True).reshape(-1) for i in range(F)]
pinned = []
for i in range(F):
    t = torch.empty(w * h * 4, dtype=torch.uint8, pin_memory=True)
    t.numpy()[:] = pageable[i]
    pinned.append(t.numpy())
legs = (("pageable packed", pageable, "1", "1"), ("pinned packed", pinned, "1", "1"),
        ("pageable rgba", pageable, "1", "0"), ("pinned rgba", pinned, "1", "0"))
if len(sys.argv) > 3 and sys.argv[3] == "hip":
    legs += (("pageable hip", pageable, "0", "0"),)
for name, frames, sd, pk in legs:
    os.environ["ZW_UPLOAD_SDMA"] = sd
    os.environ["ZW_UPLOAD_PACK"] = pk
    for u in os.environ.get("HR_UPLOADERS", "1,2,4").split(","):
        os.environ["ZW_UPLOAD_THREADS"] = u
        p.encode_host([frames])
        t0 = time.perf_counter()
        p.encode_host([frames] * NB)
        el = time.perf_counter() - t0
        bpp = 3 if pk == "1" else 4
        print(f"{name} U={u}: {F * NB / el:.0f} encodes/s ({F * NB * w * h * bpp / el / 1e9:.1f} GB/s H2D)", flush=True)
