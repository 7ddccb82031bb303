#!/usr/bin/env python3
"""Generate tests/golden/ fixtures (run in the build container, not on the GPU box).

Inputs and expected outputs only -- no reference source is copied:
  * gallery1/{1..5}.webp and gallery2/{1..5}_webp_a.webp from the reference's
    tests/images (decoder goldens of tests/decode.rs): the 'VP8 ' chunk payload
    is stored as <name>.vp8.
  * Expected results:
      - rgb_sha256: SHA-256 of the reference's golden PNG pixels
        (tests/reference/gallery1/*.png, fancy upsampling), RGB rows, for gallery1;
      - rgb_nofancy_sha256: the same for tests/reference/gallery1_nofancy/*.png
        (UpsamplingMethod::Simple), gallery1;
      - yuv_sha256: SHA-256 of the cropped Y, U, V planes decoded by the system
        libwebp (WebPDecodeYUV), the independent decoder the survey pins on.
  * regression/dark.webp (a bare 1x1 'VP8 ' frame) and the four full-canvas
    VP8 keyframes of animated/random_lossy.webp (ANMF at 0,0, no ALPH, so the
    reference's composite_frame copies each frame's RGB unchanged,
    decoder/extended.rs:31-134) with their golden PNGs
    (tests/reference/regression/dark.png, animated/random_lossy-1..4.png;
    tests/decode.rs:116-149, :193-202).  Fancy upsampling only (the reference
    holds no nofancy golden for them).
  * libwebp-encoded synthetic streams (WebPEncodeRGB at several qualities) with
    their libwebp YUV digests -- different quantisers / filter levels /
    segment maps than the gallery.
The libwebp and Pillow used here exist only in this container's image; the GPU
tests read the committed files.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "image-webp_amd"))
from zwebp.synth import synth_rgba  # noqa: E402

REF = "/root/reference/tests"
OUT = os.path.join(ROOT, "tests", "golden")


def riff_vp8(data):
    assert data[:4] == b"RIFF" and data[8:12] == b"WEBP"
    off = 12
    while off + 8 <= len(data):
        tag = data[off:off + 4]
        size = int.from_bytes(data[off + 4:off + 8], "little")
        if tag == b"VP8 ":
            return data[off + 8:off + 8 + size]
        off += 8 + size + (size & 1)
    raise ValueError("no VP8 chunk")


_W = ctypes.CDLL("libwebp.so.7")
_W.WebPDecodeYUV.restype = ctypes.c_void_p
_W.WebPDecodeYUV.argtypes = [ctypes.c_char_p, ctypes.c_size_t] + [ctypes.c_void_p] * 6
_W.WebPEncodeRGB.restype = ctypes.c_size_t
_W.WebPEncodeRGB.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                             ctypes.POINTER(ctypes.c_void_p)]
_W.WebPFree.argtypes = [ctypes.c_void_p]


def anmf_vp8(data):
    """VP8 payloads of the ANMF frames of an animated RIFF, with their offsets
    and sizes (ANMF layout: 3-byte x/2, y/2, w-1, h-1, duration, flags)."""
    assert data[:4] == b"RIFF" and data[8:12] == b"WEBP"
    out, off = [], 12
    while off + 8 <= len(data):
        tag = data[off:off + 4]
        size = int.from_bytes(data[off + 4:off + 8], "little")
        if tag == b"ANMF":
            p = data[off + 8:off + 8 + size]
            x, y = 2 * int.from_bytes(p[0:3], "little"), 2 * int.from_bytes(p[3:6], "little")
            w, h = int.from_bytes(p[6:9], "little") + 1, int.from_bytes(p[9:12], "little") + 1
            assert p[16:20] == b"VP8 ", "frame is not a bare VP8 chunk"
            n = int.from_bytes(p[20:24], "little")
            out.append((x, y, w, h, p[24:24 + n]))
        off += 8 + size + (size & 1)
    return out


def libwebp_yuv_digests(riff):
    w, h, stride, uvs = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    u, v = ctypes.c_void_p(), ctypes.c_void_p()
    y = _W.WebPDecodeYUV(riff, len(riff), ctypes.byref(w), ctypes.byref(h), ctypes.byref(u), ctypes.byref(v),
                         ctypes.byref(stride), ctypes.byref(uvs))
    assert y
    W, H, cw, ch = w.value, h.value, (w.value + 1) // 2, (h.value + 1) // 2

    def plane(p, s, pw, ph):
        buf = (ctypes.c_uint8 * (s * (ph - 1) + pw)).from_address(p)
        a = np.frombuffer(buf, np.uint8)
        return np.stack([a[r * s:r * s + pw] for r in range(ph)])

    Y, U, V = plane(y, stride.value, W, H), plane(u.value, uvs.value, cw, ch), plane(v.value, uvs.value, cw, ch)
    d = [hashlib.sha256(p.tobytes()).hexdigest() for p in (Y, U, V)]
    _W.WebPFree(ctypes.c_void_p(y))
    return W, H, d


def wrap_riff(vp8):
    pad = len(vp8) & 1
    body = b"WEBP" + b"VP8 " + len(vp8).to_bytes(4, "little") + vp8 + b"\0" * pad
    return b"RIFF" + len(body).to_bytes(4, "little") + body


def main():
    from PIL import Image
    os.makedirs(OUT, exist_ok=True)
    manifest = {"generator": "tools/make_golden.py", "streams": []}
    for i in range(1, 6):
        riff = open(f"{REF}/images/gallery1/{i}.webp", "rb").read()
        vp8 = riff_vp8(riff)
        name = f"gallery1_{i}"
        open(os.path.join(OUT, name + ".vp8"), "wb").write(vp8)
        W, H, d = libwebp_yuv_digests(riff)
        png = np.asarray(Image.open(f"{REF}/reference/gallery1/{i}.png").convert("RGB"))
        assert png.shape == (H, W, 3)
        # UpsamplingMethod::Simple goldens (tests/decode.rs:168-190 reftest_nofancy)
        png_nf = np.asarray(Image.open(f"{REF}/reference/gallery1_nofancy/{i}.png").convert("RGB"))
        assert png_nf.shape == (H, W, 3)
        manifest["streams"].append(dict(name=name, source=f"tests/images/gallery1/{i}.webp", width=W, height=H,
                                        yuv_sha256=d, rgb_sha256=hashlib.sha256(png.tobytes()).hexdigest(),
                                        rgb_nofancy_sha256=hashlib.sha256(png_nf.tobytes()).hexdigest()))
    for i in range(1, 6):
        riff = open(f"{REF}/images/gallery2/{i}_webp_a.webp", "rb").read()
        vp8 = riff_vp8(riff)
        name = f"gallery2_{i}_a"
        open(os.path.join(OUT, name + ".vp8"), "wb").write(vp8)
        W, H, d = libwebp_yuv_digests(wrap_riff(vp8))
        manifest["streams"].append(dict(name=name, source=f"tests/images/gallery2/{i}_webp_a.webp", width=W,
                                        height=H, yuv_sha256=d))
    # regression/dark (tests/decode.rs:197): 1x1 frame
    riff = open(f"{REF}/images/regression/dark.webp", "rb").read()
    vp8 = riff_vp8(riff)
    open(os.path.join(OUT, "regression_dark.vp8"), "wb").write(vp8)
    W, H, d = libwebp_yuv_digests(riff)
    png = np.asarray(Image.open(f"{REF}/reference/regression/dark.png").convert("RGB"))
    assert png.shape == (H, W, 3)
    manifest["streams"].append(dict(name="regression_dark", source="tests/images/regression/dark.webp", width=W,
                                    height=H, yuv_sha256=d, rgb_sha256=hashlib.sha256(png.tobytes()).hexdigest()))
    # animated/random_lossy (tests/decode.rs:193, every frame :116-149)
    riff = open(f"{REF}/images/animated/random_lossy.webp", "rb").read()
    for i, (x, y, w, h, vp8) in enumerate(anmf_vp8(riff), 1):
        cw = int.from_bytes(riff[24:27], "little") + 1
        ch = int.from_bytes(riff[27:30], "little") + 1
        assert (x, y, w, h) == (0, 0, cw, ch), "not a full-canvas frame"
        name = f"random_lossy_{i}"
        open(os.path.join(OUT, name + ".vp8"), "wb").write(vp8)
        W, H, d = libwebp_yuv_digests(wrap_riff(vp8))
        png = np.asarray(Image.open(f"{REF}/reference/animated/random_lossy-{i}.png").convert("RGB"))
        assert png.shape == (H, W, 3)
        manifest["streams"].append(dict(name=name, source=f"tests/images/animated/random_lossy.webp frame {i}",
                                        width=W, height=H, yuv_sha256=d,
                                        rgb_sha256=hashlib.sha256(png.tobytes()).hexdigest()))
    for (w, h, kind, q) in [(64, 48, "natural", 75), (333, 211, "natural", 30), (256, 256, "noise", 90),
                            (200, 120, "natural", 5), (160, 96, "natural", 100)]:
        rgb = np.ascontiguousarray(synth_rgba(w, h, 0x5EED0000 + w, kind)[..., :3])
        outp = ctypes.c_void_p()
        n = _W.WebPEncodeRGB(rgb.ctypes.data, w, h, w * 3, float(q), ctypes.byref(outp))
        riff = ctypes.string_at(outp.value, n)
        _W.WebPFree(outp)
        vp8 = riff_vp8(riff)
        name = f"libwebp_{kind}_{w}x{h}_q{q}"
        open(os.path.join(OUT, name + ".vp8"), "wb").write(vp8)
        W, H, d = libwebp_yuv_digests(riff)
        manifest["streams"].append(dict(name=name, source=f"libwebp WebPEncodeRGB(synth_rgba {kind}), q={q}",
                                        width=W, height=H, yuv_sha256=d))
    with open(os.path.join(OUT, "decode_golden.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(manifest["streams"]), "streams")


if __name__ == "__main__":
    main()
