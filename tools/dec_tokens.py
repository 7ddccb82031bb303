#!/usr/bin/env python3
"""Device token parse (k_dec_tok1 + k_dec_tok2) against the host parse: the same batch
decoded with ZW_DEC_TOKENS=host and =device must give identical planes; prints
both wall times, the token kernel time and the per-stage breakdown.
usage: python tools/dec_tokens.py [frames] [reps] [modes] [distinct frames (4)]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402


def run(vp8, ctx, mode, reps):
    os.environ["ZW_DEC_TOKENS"] = mode
    best = None
    fr = None
    for _ in range(reps):
        hs = [hashlib.sha256(bytes(f.ybuf) + bytes(f.ubuf) + bytes(f.vbuf)).hexdigest() for f in fr[:8]] if fr else None
        fr = None  # the previous batch's frames go back to the library (as a decode loop frees them)
        t0 = time.perf_counter()
        fr = zwebp.decode_batch(vp8, ctx=ctx)
        el = time.perf_counter() - t0
        if best is None or el < best[0]:
            best = (el, zwebp.decode_token_ms(ctx=ctx), zwebp.decode_kernel_times(ctx=ctx),
                    zwebp.decode_stage_times(ctx=ctx), zwebp.decode_token_stages(ctx=ctx))
    hs = [hashlib.sha256(bytes(f.ybuf) + bytes(f.ubuf) + bytes(f.vbuf)).hexdigest() for f in fr[:8]]
    return best, hs


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    w, h = 1920, 1080
    ctx = zwebp.Context(0)
    D = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    streams = []
    for i0 in range(0, D, 64):
        imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(i0, min(D, i0 + 64))]
        streams += zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    vp8 = [streams[i % D] for i in range(F)]
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["host", "device", "mixed"]
    ref = None
    ok = True
    for mode in modes:
        (e, tok, k, st, ts), hs = run(vp8, ctx, mode, reps)
        ref = ref or hs
        ok = ok and hs == ref
        print(f"{F} frames, tokens={mode} (host share {os.environ.get('ZW_DEC_TOKENS_HOST', '0.5')}): "
              f"{F / e:.0f} decodes/s, token parse {tok:.1f} ms (stage 1 {ts[0]:.1f}, count {ts[1]:.1f}, "
              f"records {ts[2]:.1f}), recon/filter {k[0]:.2f}/{k[1]:.2f} ms, "
              f"stages parse/download/fanout {st[0]:.1f}/{st[1]:.1f}/{st[2]:.1f} ms; planes equal: {hs == ref}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
