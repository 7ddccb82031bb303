"""The encoder on natural images: the reference's gallery pictures (its own
lossy test files, tests/golden/gallery*.vp8, decoded to RGB with the fancy
upsampler) as encoder input.

CPU: the published quality band.  The reference states its Q75 method-4
output at 1.045-1.135x libwebp's size with a PSNR gap of about 1.35 dB
(CLAUDE.md:37-45); no encoder golden exists, so this is the
independent check on the oracle's mode decisions that the reference itself
offers: on every gallery image the oracle's stream must sit in
[1.0, 1.15]x the system libwebp's Q75 VP8 payload and within 1.5 dB of its
PSNR.  (Measured: 1.033-1.085x, -0.8 .. +4.0 dB.)

GPU: the product's bitstreams on the same images (odd sizes, real content)
are byte-equal to the oracle's.
"""
import ctypes
import glob
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(GOLD, "gallery*.vp8")))

try:
    _W = ctypes.CDLL("libwebp.so.7")
    _W.WebPEncodeRGB.restype = ctypes.c_size_t
    _W.WebPEncodeRGB.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                 ctypes.POINTER(ctypes.c_void_p)]
    _W.WebPFree.argtypes = [ctypes.c_void_p]
except OSError:  # pragma: no cover - the GPU box image may lack it
    _W = None


def _rgb(path):
    b = open(path, "rb").read()
    rc, h = O.decode_header(b)
    assert rc == 0
    rc, r = O.decode(b)
    assert rc == 0
    return O.yuv_to_rgb_fancy(r["y"], r["u"], r["v"], h.width, h.height, 3), h.width, h.height


def _libwebp_vp8(rgb, w, h, q):
    p = ctypes.c_void_p()
    a = np.ascontiguousarray(rgb)
    n = _W.WebPEncodeRGB(a.ctypes.data, w, h, w * 3, q, ctypes.byref(p))
    assert n > 0
    riff = ctypes.string_at(p.value, n)
    _W.WebPFree(p)
    i = riff.find(b"VP8 ")
    size = int.from_bytes(riff[i + 4:i + 8], "little")
    return riff[i + 8:i + 8 + size]


def _psnr(vp8, rgb, w, h):
    rc, d = O.decode(vp8)
    assert rc == 0
    out = O.yuv_to_rgb_fancy(d["y"], d["u"], d["v"], w, h, 3).astype(np.float64)
    return 10 * np.log10(255.0 * 255.0 / np.mean((out - rgb.astype(np.float64)) ** 2))


@pytest.mark.skipif(_W is None, reason="system libwebp absent")
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_quality_band_vs_libwebp(path):
    rgb, w, h = _rgb(path)
    rc, ours, _ = O.encode(rgb, w, h, 2, 75, 4)
    assert rc == 0
    ref = _libwebp_vp8(rgb, w, h, 75)
    ratio = len(ours) / len(ref)
    assert 1.0 <= ratio <= 1.15, ratio
    assert _psnr(ours, rgb, w, h) >= _psnr(ref, rgb, w, h) - 1.5


@pytest.fixture(scope="module")
def ctx():
    import zwebp
    return zwebp.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f) for f in FILES])
def test_gpu_encode_natural_images(ctx, path):
    import zwebp
    rgb, w, h = _rgb(path)
    out = zwebp.encode_frame_lossy(rgb, w, h, zwebp.ColorType.Rgb8, 75, 4, ctx=ctx)
    rc, ref, _ = O.encode(rgb, w, h, 2, 75, 4)
    assert rc == 0
    assert out == ref
