#!/usr/bin/env python3
"""Generate tests/golden/bench_digests.json: SHA-256 of the oracle's VP8
bitstream for every synthetic frame bench.py can time, so the throughput run
checks its own output without running the oracle (bench.py only reads the
digests; the oracle stays test infrastructure).

Frames covered (synth_rgba natural, RGBA8, Q75 method 4):
  * 1920x1080 (configs 2/4, default weak-scaling mode): seeds
    frame_seed(k*256 + i), k = 0..31, i = 0..3 -- the 4 distinct frames of
    every rank for per-rank batches that are multiples of 256 frames up to 8
    ranks x 1024 frames;
  * 3840x2160 (config 5, --total-frames 4096 over 1/2/4/8 ranks): seeds
    frame_seed(k*512 + i), k = 0..7, i = 0..3 (each rank's shard start).
Run in the build container: python tools/make_bench_digests.py  (~2 min, 8 threads)
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "image-webp_amd"), os.path.join(ROOT, "tests")]
import oracle_lib as O  # noqa: E402  (checker only)
from zwebp.shard import frame_seed  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
JOBS = [(1920, 1080, k * 256 + i) for k in range(32) for i in range(4)] + \
       [(3840, 2160, k * 512 + i) for k in range(8) for i in range(4)]


def one(job):
    w, h, idx = job
    seed = frame_seed(idx)
    rc, bs, _ = O.encode(synth_rgba(w, h, seed), w, h, 3, 75, 4)
    assert rc == 0
    return f"{w}x{h}/q75m4/{seed:#010x}", hashlib.sha256(bs).hexdigest(), len(bs)


def main():
    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, JOBS))
    d = {"generator": "tools/make_bench_digests.py (oracle/ C restatement of the reference encoder)",
         "key": "WxH/qQmM/seed -> sha256 of the raw VP8 frame (encode_frame_lossy output)",
         "digests": {k: v for k, v, _ in res}, "bytes": {k: n for k, _, n in res}}
    with open(OUT, "w") as f:
        json.dump(d, f, indent=0, sort_keys=True)
    print(f"{len(res)} digests -> {OUT}")


if __name__ == "__main__":
    main()
