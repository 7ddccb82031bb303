"""Writes the decode bench's kind of input for tools/parse_bench.cpp: 1080p
synthetic frames (zwebp.synth, seeds 0x5EED0000 + i) encoded at Q75 m4 by the
oracle/ C restatement, as raw VP8 frames /tmp/parse_bench_<i>.vp8.

    python tools/parse_bench_streams.py [count] [W H]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "image-webp_amd"))

import oracle_lib  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
for i in range(n):
    img = synth_rgba(w, h, 0x5EED0000 + i)
    rc, vp8, _ = oracle_lib.encode(img, w, h, 3, quality=75, method=4)  # ColorType.Rgba8
    assert rc == 0, rc
    path = f"/tmp/parse_bench_{i}.vp8"
    with open(path, "wb") as f:
        f.write(vp8)
    print(path, len(vp8))
