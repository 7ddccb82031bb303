#!/usr/bin/env python3
"""Time the streaming DCT+quant pass (k_fdct_quant) alone: python tools/xform_bench.py [frames]."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import zwebp  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = zwebp.Context(0)
r = bench.dct_quant_pass(ctx, torch, dev, frames, 8160, reps=10)
print(os.environ.get("ZW_XFORM_VARIANT", "0"), os.environ.get("ZW_XFORM_GRID", "16"),
      f"{r['ms_per_launch']:.3f} ms {r['achieved']:.0f} GB/s frac {r['frac']:.3f}")
