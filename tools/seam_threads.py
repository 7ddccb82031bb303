#!/usr/bin/env python3
"""encode_frame_lossy from T threads, one context each, on one GPU (1080p RGBA
Q75 m4), verified against the bench digests.  Prints one JSON line.
usage: python tools/seam_threads.py [seconds] [T ...]"""
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
import zwebp  # noqa: E402
from zwebp.shard import frame_seed  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402


def run(img, w, h, q, m, want, T, seconds):
    ctxs = [zwebp.Context(0) for _ in range(T)]
    for c in ctxs:
        zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=c)
    counts, good = [0] * T, [True] * T
    start = threading.Barrier(T + 1)
    stop = [False]

    def work(t):
        start.wait()
        while not stop[0]:
            b = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctxs[t])
            good[t] = good[t] and (want is None or hashlib.sha256(b).hexdigest() == want)
            counts[t] += 1

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    start.wait()
    t0 = time.perf_counter()
    time.sleep(seconds)
    stop[0] = True
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    for c in ctxs:
        c.close()
    return {"encodes_per_s": sum(counts) / el, "calls": sum(counts), "ms_per_call": T * el / max(1, sum(counts)) * 1e3,
            "verified": want is not None and all(good)}


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    Ts = [int(t) for t in sys.argv[2:]] or [1, 4, 16]
    w, h, q, m = 1920, 1080, 75, 4
    seed = frame_seed(0)
    img = synth_rgba(w, h, seed)
    try:
        with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
            want = json.load(f)["digests"].get(f"{w}x{h}/q{q}m{m}/{seed:#010x}")
    except (OSError, ValueError, KeyError):
        want = None
    out = {str(T): run(img, w, h, q, m, want, T, seconds) for T in Ts}
    print(json.dumps({"threads": out, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")}), flush=True)


if __name__ == "__main__":
    main()
