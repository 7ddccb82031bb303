#!/usr/bin/env python3
"""Decode path (SURVEY config 3): host bool decoding + k_dec_recon + k_loopfilter on
a batch of 1080p frames encoded by this library (Q75 m4).
usage: python tools/dec_bench.py [frames] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

DEC_BYTES_PER_MB = 1208  # levels 800 + side info 24 + final YUV 384


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    w, h = 1920, 1080
    ctx = zwebp.Context(0)
    imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
    streams = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    vp8 = [streams[i % 4] for i in range(F)]
    zwebp.decode_batch(vp8[:8], ctx=ctx)  # warm-up
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        zwebp.decode_batch(vp8, ctx=ctx)
        el = time.perf_counter() - t0
        rk, lf = zwebp.decode_kernel_times(ctx=ctx)
        if best is None or el < best[0]:
            best = (el, rk, lf)
    el, rk, lf = best
    nmb = ((w + 15) // 16) * ((h + 15) // 16) * F
    gbs = DEC_BYTES_PER_MB * nmb / ((rk + lf) * 1e-3) / 1e9
    if os.environ.get("DEC_BATCH_ONLY"):  # (profiling runs: the batch launches only)
        print(f"{F} frames: kernels recon {rk:.2f} ms + loopfilter {lf:.2f} ms")
        return
    # single frame (SURVEY config 3): end to end, and the oracle's CPU decode of the same stream
    one = [vp8[0]]
    zwebp.decode_batch(one, ctx=ctx)
    t0 = time.perf_counter()
    for _ in range(5):
        zwebp.decode_batch(one, ctx=ctx)
    el1 = (time.perf_counter() - t0) / 5
    rk1, lf1 = zwebp.decode_kernel_times(ctx=ctx)
    cpu = None
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        t0 = time.perf_counter()
        O.decode(bytes(one[0]))
        cpu = time.perf_counter() - t0
    except Exception as e:  # noqa: BLE001 - the oracle is optional here
        print("oracle decode unavailable:", e)
    print(f"single frame: {el1 * 1e3:.2f} ms end to end (kernels {rk1:.2f} + {lf1:.2f} ms)"
          + (f"; oracle CPU decode {cpu * 1e3:.1f} ms (1 thread)" if cpu else ""))
    print(f"{F} frames: wall {el * 1e3:.1f} ms = {F / el:.0f} decodes/s (host parse + PCIe both ways); "
          f"kernels recon {rk:.2f} ms + loopfilter {lf:.2f} ms = {F / ((rk + lf) * 1e-3):.0f} frames/s, "
          f"{gbs:.0f} GB/s ({gbs / 8000:.3f} of HBM peak)")


if __name__ == "__main__":
    main()
