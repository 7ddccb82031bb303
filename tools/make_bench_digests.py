#!/usr/bin/env python3
"""Generate tests/golden/bench_digests.json: SHA-256 digests of the oracle's
outputs for every synthetic workload bench.py times, so the driver-run bench
checks every leg's output without running the oracle (bench.py only reads the
digests; the oracle stays test infrastructure).

Keys (synth_rgba natural frames, RGBA8, Q75 method 4; seed = frame_seed(i)):
  WxH/q75m4/seed            raw VP8 frame (encode_frame_lossy)
      1920x1080 (configs 2/4, weak scaling): frame_seed(k*256 + i), k < 32, i < 4
      3840x2160 (config 5, --total-frames 4096 over 1/2/4/8 ranks): frame_seed(k*512 + i), k < 8
      768x512   (config 1): frame_seed(i)
  p8/1920x1080/q75m4/seed   the same frame with 8 token partitions (single_frame leg)
  riff/1920x1080/q75m4/seed RIFF + VP8X + ALPH + VP8 (WebPEncoder::encode of the RGBA frame)
  riffa/1920x1080/q75m4/seed the same for synth_rgba(..., kind="alpha") frames (a real alpha plane)
  dec_yuv/1920x1080/q75m4/seed   Y || U || V (MB-padded) of decode_frame of the VP8 frame
  dec_rgba/1920x1080/q75m4/seed  fill_rgba (fancy upsampling) of that decode
  xmb/1920x1080/q75m4/seed  levels || ry || ru || rv of the streaming DCT+quant pass
                            (or_xform_mbs) over the records of the frame's pass-2
                            modes and reconstruction, diffusion terms synthetic_derr(seed)
  for i < 4 unless stated.
Run in the build container: python tools/make_bench_digests.py  (~3 min, 8 threads)
"""
import hashlib
import json
import os
import struct
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "image-webp_amd"), os.path.join(ROOT, "tests")]
import oracle_lib as O  # noqa: E402  (checker only)
from zwebp.shard import frame_seed  # noqa: E402
from zwebp.synth import synth_rgba  # noqa: E402
from zwebp.xmb import build_records, synthetic_derr  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
JOBS = [("vp8", 1920, 1080, k * 256 + i) for k in range(32) for i in range(4)] + \
       [("vp8", 3840, 2160, k * 512 + i) for k in range(8) for i in range(4)] + \
       [("vp8", 768, 512, i) for i in range(4)] + \
       [("full", 1920, 1080, i) for i in range(4)] + \
       [("riffa", 1920, 1080, i) for i in range(4)]


def sha(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(a if isinstance(a, bytes) else np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _chunk(tag, payload):
    return tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")


def riff_rgba(w, h, vp8, alph):
    """WebPEncoder::encode with EncoderParams::lossy on an RGBA frame (encoder/api.rs:1291-1398)."""
    vp8x = _chunk(b"VP8X", bytes([0x10, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little"))
    body = b"WEBP" + vp8x + _chunk(b"ALPH", alph) + _chunk(b"VP8 ", vp8)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def one(job):
    kind, w, h, idx = job
    seed = frame_seed(idx)
    tag = f"{w}x{h}/q75m4/{seed:#010x}"
    img = synth_rgba(w, h, seed, "alpha" if kind == "riffa" else "natural")
    if kind == "riffa":
        rc, bs, _ = O.encode(img, w, h, 3, 75, 4)
        assert rc == 0
        rc, alph = O.encode_alpha(img, w, h, 3)
        assert rc == 0
        riff = riff_rgba(w, h, bs, alph)
        return [("riffa/" + tag, sha(riff), len(riff)), ("riffa_alph/" + tag, "", len(alph))]
    if kind == "vp8":
        rc, bs, _ = O.encode(img, w, h, 3, 75, 4)
        assert rc == 0
        return [(tag, sha(bs), len(bs))]
    out = []
    rc, bs, d = O.encode(img, w, h, 3, 75, 4, debug=True)
    assert rc == 0
    out.append((tag, sha(bs), len(bs)))
    rc, p8, _ = O.encode(img, w, h, 3, 75, 4, nparts=8)
    assert rc == 0
    out.append(("p8/" + tag, sha(p8), len(p8)))
    rc, alph = O.encode_alpha(img, w, h, 3)
    assert rc == 0
    riff = riff_rgba(w, h, bs, alph)
    out.append(("riff/" + tag, sha(riff), len(riff)))
    rc, r = O.decode(bs)
    assert rc == 0
    out.append(("dec_yuv/" + tag, sha(r["y"], r["u"], r["v"]), 0))
    out.append(("dec_rgba/" + tag, sha(O.yuv_to_rgb_fancy(r["y"], r["u"], r["v"], w, h, 4)), 0))
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    nmb = mbw * mbh
    p2 = d["p2_info"]
    modes = np.zeros((nmb, 20), np.uint8)
    for i in range(nmb):
        modes[i, :4] = (p2[i].luma_mode, p2[i].chroma_mode, p2[i].skip, p2[i].segment)
        modes[i, 4:20] = list(p2[i].bpred)
    recs = build_records(mbw, mbh, modes, d["recon_y"], d["recon_u"], d["recon_v"], synthetic_derr(nmb, seed))
    sq = np.array(d["seg_quant_index"], np.int32).reshape(1, 4)
    lv, ry, ru, rv = O.xform_mbs(d["src_y"], d["src_u"], d["src_v"], recs, sq, 1, mbw, mbh)
    out.append(("xmb/" + tag, sha(lv, ry, ru, rv), 0))
    return out


def main():
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None  # e.g. "riffa": add those kinds to the file
    jobs = [j for j in JOBS if only is None or j[0] in only]
    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        res = [r for rs in ex.map(one, jobs) for r in rs]
    if only is not None:
        old = json.load(open(OUT))
        old["digests"].update({k: v for k, v, _ in res if v})
        old["bytes"].update({k: n for k, _, n in res if n})
        with open(OUT, "w") as f:
            json.dump(old, f, indent=0, sort_keys=True)
        print(f"{len(res)} digests added -> {OUT}")
        return
    d = {"generator": "tools/make_bench_digests.py (oracle/ C restatement of the reference encoder)",
         "key": "see tools/make_bench_digests.py: kind/WxH/qQmM/seed -> sha256 of the oracle's output",
         "digests": {k: v for k, v, _ in res if v}, "bytes": {k: n for k, _, n in res if n}}
    with open(OUT, "w") as f:
        json.dump(d, f, indent=0, sort_keys=True)
    print(f"{len(res)} digests -> {OUT}")


if __name__ == "__main__":
    main()
