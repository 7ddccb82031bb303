#!/usr/bin/env python3
"""Standalone run of bench.py's k_xform_mb leg (the 8(d) roofline pass) for
rocprofv3 --kernel-trace / --pmc passes: encodes 4 synthetic 1080p frames
(Q75 m4) to get real modes and borders, then times the record-based streaming
DCT+quant pass over 256 frames, RGBA-fused and from Y/U/V planes.  Prints one
JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "image-webp_amd")]

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-i4", action="store_true", help="rewrite I4 MBs as I16 DC (cost of the I4 chains)")
    ap.add_argument("--yuv-only", action="store_true", help="only the Y/U/V-plane form (no RGBA-fused leg)")
    a = ap.parse_args()
    if a.no_i4:
        import zwebp.xmb as X
        orig = X.build_records

        def no_i4(*args, **kw):
            r = orig(*args, **kw)
            r[r[:, 0] == 4, 0] = 0
            return r
        X.build_records = no_i4
    import torch
    import zwebp
    from zwebp.shard import frame_seed
    from zwebp.synth import synth_rgba
    w, h, q, m, nd = 1920, 1080, 75, 4, 4
    ctx = zwebp.Context(0)
    dev = torch.device("cuda", 0)
    seeds = [frame_seed(i) for i in range(nd)]
    p = zwebp.Pipeline(nd, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    imgs = [synth_rgba(w, h, sd) for sd in seeds]
    for i in range(nd):
        p.upload(i, imgs[i])
    p.encode()
    r = bench.xmb_pass(ctx, torch, dev, p, nd, seeds, w, h, q, m, a.frames, a.reps, bench.load_digests(),
                       None if a.yuv_only else imgs)
    p.close()
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
