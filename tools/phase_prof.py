#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_encode (profiling build, make -C image-webp_amd prof).

Counters are summed over all waves (lane 0), so totals are wave-cycles.
usage: python tools/phase_prof.py [frames] [width] [height] [method]
"""
import ctypes
import os

# Two pipeline lanes x (kernel + copy stream) plus the runtime's own streams:
# ask HIP for 8 hardware queues (default 4) so no two busy streams share one.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("ZWEBP_LIB", os.path.join(ROOT, "image-webp_amd", "zwebp", "libzwebp_prof.so"))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

NAMES = {0: "wait(row above)", 1: "border+pick_i16", 2: "pick_i4", 3: "pick_uv", 4: "final_luma",
         5: "final_chroma", 6: "store/levels/publish", 8: "p1 chroma pick_uv", 9: "p1 chroma final",
         10: "  i4: values", 11: "  i4: preds+sse+rank", 12: "  i4: candidates", 13: "  i4: select+recon",
         7: "  (count of I4 MBs)", 14: "  final: I16 MBs", 15: "  final: I4 MBs",
         16: "    i16: fdct+y2", 17: "    i16: quant check+trellis", 18: "    i16: ctx resolve+gather",
         19: "  (I4 search steps run)", 20: "  (I4 searches)",
         21: "wait(above-right)+border",
         22: "  i4q: modes+pred+src", 23: "  i4q: fdct+quant+cost"}


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    m = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    L = zwebp.load_library()
    L.zw_phase_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    buf = (ctypes.c_ulonglong * 48)()
    p = zwebp.Pipeline(F, w, h, zwebp.ColorType.Rgba8, 75, m)
    imgs = [synth_rgba(w, h, 0x5EED0000 + i) for i in range(4)]
    for i in range(F):
        p.upload(i, imgs[i % 4])
    p.encode()
    L.zw_phase_cycles(buf, 1)
    t = time.perf_counter()
    p.encode()
    el = time.perf_counter() - t
    assert L.zw_phase_cycles(buf, 0) == 0
    L.zw_wave_cycles.argtypes = [ctypes.c_void_p, ctypes.c_int]
    wbuf = (ctypes.c_ulonglong * (2 * 16 * 24))()
    assert L.zw_wave_cycles(wbuf, 0) == 0
    kt = p.kernel_times()
    nmb = p.mbw * p.mbh * F
    print(f"{F} frames {w}x{h} m{m}: step {el * 1e3:.1f} ms, kernels(ms) {[round(x, 2) for x in kt[:4]]} "
          f"host(ms) fetch1/stats/fetch2/emit {[round(x, 2) for x in kt[4:8]]}")
    for ps in (0, 1):
        tot = sum(buf[ps * 24 + k] for k in list(range(10)) + [21] if k not in (7, 19, 20)) or 1
        print(f"pass {ps + 1}: total {tot / 1e9:.2f} G wave-cycles, {tot / nmb:.0f} wave-cycles/MB")
        for k in range(24):
            v = buf[ps * 24 + k]
            if v and k in (7, 19, 20):
                print(f"   {NAMES.get(k, k):24s} {v / nmb:12.3f} of MBs")
            elif v:
                print(f"   {NAMES.get(k, k):24s} {v / nmb:12.0f} cyc/MB  {100 * v / tot:5.1f}%")
        print(f"   per wave (pass {ps + 1}): total G cycles / wait G cycles / MBs(approx by I4 searches)")
        for wv in range(16):
            b = [wbuf[(ps * 16 + wv) * 24 + k] for k in range(24)]
            t = sum(b[k] for k in list(range(10)) + [21] if k not in (7,))
            if t:
                print(f"     wave {wv:2d}: {t / 1e9:8.2f}  wait {(b[0] + b[21]) / 1e9:7.2f}  ({100 * (b[0] + b[21]) / t:4.1f}%)"
                      f"  i4 searches {b[20]}")


if __name__ == "__main__":
    main()
