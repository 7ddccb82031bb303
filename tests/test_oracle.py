"""Pin the CPU oracle (oracle/) against the reference's known-answer tests and
the committed golden fixtures.  CPU only; nothing here touches the product.

Reference KATs restated (values are the reference tests' own data):
  transform.rs:213-229        test_dct_inverse
  encoder/arithmetic.rs:211-271  bool encoder short / hello / tree
  encoder/cost.rs:2597-2690   test_trellis_vs_libwebp (expected -11, 0, ...)
  encoder/cost.rs:2046-2069   fixed mode costs
  decoder/yuv.rs:905-971      fancy upsampling grid + yuv_to_rgb
  tests/decode.rs             gallery goldens (tests/golden/decode_golden.json)
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from zwebp.synth import synth_rgba

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _manifest():
    with open(os.path.join(GOLD, "decode_golden.json")) as f:
        return json.load(f)["streams"]


def test_dct_inverse_kat():
    blk = np.array([38, 6, 210, 107, 42, 125, 185, 151, 241, 224, 125, 233, 227, 8, 57, 96], np.int32)
    d = O.blocks("or_fdct_c", blk)
    assert np.array_equal(O.blocks("or_idct_c", d), blk)
    assert np.array_equal(O.blocks("or_idct_scalar_c", d), blk)


def test_fdct_sse2_equals_scalar_in_residual_range():
    rng = np.random.default_rng(1)
    b = rng.integers(-255, 256, size=(20000, 16)).astype(np.int32)
    assert np.array_equal(O.blocks("or_fdct_c", b), O.blocks("or_fdct_sse2_c", b))


def test_idct_sse2_saturation_differs_only_out_of_i16():
    rng = np.random.default_rng(2)
    b = rng.integers(-2048 * 157, 2048 * 157, size=(4000, 16)).astype(np.int32)
    small = rng.integers(-2000, 2000, size=(4000, 16)).astype(np.int32)
    assert np.array_equal(O.blocks("or_idct_c", small), O.blocks("or_idct_scalar_c", small))
    # out-of-range inputs: SSE2 semantics saturate (transform_simd_intrinsics.rs:493)
    assert not np.array_equal(O.blocks("or_idct_c", b), O.blocks("or_idct_scalar_c", b))


def test_wht_roundtrip_dc_only():
    rng = np.random.default_rng(3)
    dc = rng.integers(-2000, 2000, size=(1000, 16)).astype(np.int32) * 8
    w = O.blocks("or_wht_c", dc)
    assert w.shape == dc.shape


def _bool_kat(ops):
    L = O.lib()
    flat = np.array([x for op in ops for x in op], np.int32)
    out = np.zeros(64, np.uint8)
    n = L.or_bool_encoder_kat(O._p(flat), len(ops), O._p(out), 64)
    return bytes(out[:n])


def test_bool_encoder_short():
    ops = [(2, 0, 0), (0, 1, 10), (0, 0, 250), (1, 1, 1), (1, 3, 5), (1, 8, 64), (1, 8, 185)]
    assert _bool_kat(ops) == bytes([104, 101, 107, 128])


def test_bool_encoder_hello():
    ops = [(2, 0, 0), (0, 1, 10), (0, 0, 250), (1, 1, 1), (1, 3, 5), (1, 8, 64), (1, 8, 185), (1, 8, 31),
           (1, 8, 134), (3, 2, 0x7FFF), (3, 2, 1)]
    assert _bool_kat(ops)[:5] == b"hello"


def test_bool_encoder_tree():
    assert _bool_kat([(4, 3, 0)]) == bytes([233, 64, 0, 0])  # TM_PRED


def test_trellis_vs_libwebp():
    L = O.lib()
    L.or_trellis_kat.restype = ctypes.c_int
    inp = np.array([-282, 6, 3, -4, -3, -11, -4, -2, 5, 3, 4, -1, 2, -2, -3, -1], np.int32)
    lev = np.zeros(16, np.int32)
    co = np.zeros(16, np.int32)
    L.or_trellis_kat(O._p(inp), 25, 31, 5242, 4228, 840, 3, 0, 0, 1, O._p(lev), O._p(co))
    expect = np.zeros(16, np.int32)
    expect[0] = -11
    assert np.array_equal(lev, expect)


def test_fixed_costs():
    L = O.lib()
    L.or_fixed_cost_i16.restype = ctypes.c_uint32
    L.or_fixed_cost_uv.restype = ctypes.c_uint32
    assert [L.or_fixed_cost_i16(i) for i in range(4)] == [663, 919, 872, 919]
    assert [L.or_fixed_cost_uv(i) for i in range(4)] == [302, 984, 439, 642]


def test_quality_mapping():
    L = O.lib()
    assert L.or_quality_to_quant_index(75) == 26
    assert L.or_filter_level_for_quality(75) == 6


def test_yuv_conversions_kat():
    y, u, v = (np.array([203], np.uint8), np.array([40], np.uint8), np.array([42], np.uint8))
    assert list(O.yuv_to_rgb_fancy(y, u, v, 1, 1)) == [80, 255, 40]


def test_fancy_grid_kat():
    Y = np.array([77, 162, 202, 185, 28, 13, 199, 182, 135, 147, 164, 135, 66, 27, 171, 130], np.uint8)
    U = np.array([34, 101, 123, 163], np.uint8)
    V = np.array([97, 167, 149, 23], np.uint8)
    up_u = [34, 51, 84, 101, 56, 71, 101, 117, 101, 112, 136, 148, 123, 133, 153, 163]
    up_v = [97, 115, 150, 167, 110, 115, 126, 131, 136, 117, 78, 59, 149, 118, 55, 23]
    got = O.yuv_to_rgb_fancy(Y, U, V, 4, 4)
    exp = []
    for k in range(16):
        exp += list(O.yuv_to_rgb_fancy(Y[k:k + 1], np.array([up_u[k]], np.uint8), np.array([up_v[k]], np.uint8),
                                       1, 1))
    assert list(got) == exp


def _crop(p, stride, w, h):
    return np.ascontiguousarray(p.reshape(-1, stride)[:h, :w])


@pytest.mark.parametrize("entry", _manifest(), ids=lambda e: e["name"])
def test_oracle_decoder_matches_goldens(entry):
    vp8 = open(os.path.join(GOLD, entry["name"] + ".vp8"), "rb").read()
    rc, r = O.decode(vp8)
    assert rc == 0
    w, h = entry["width"], entry["height"]
    ys, cs = r["mbw"] * 16, r["mbw"] * 8
    planes = (_crop(r["y"], ys, w, h), _crop(r["u"], cs, (w + 1) // 2, (h + 1) // 2),
              _crop(r["v"], cs, (w + 1) // 2, (h + 1) // 2))
    assert [hashlib.sha256(p.tobytes()).hexdigest() for p in planes] == entry["yuv_sha256"]
    if "rgb_sha256" in entry:
        # the reference's own RGB goldens (fancy upsampling, tests/decode.rs)
        Yc, Uc, Vc = planes
        rgb = O.yuv_to_rgb_fancy(Yc.reshape(-1), Uc.reshape(-1), Vc.reshape(-1), w, h)
        assert hashlib.sha256(rgb.tobytes()).hexdigest() == entry["rgb_sha256"]
    if "rgb_nofancy_sha256" in entry:
        # UpsamplingMethod::Simple goldens (tests/decode.rs:168-190, reference/gallery1_nofancy)
        rgb = O.yuv_to_rgb_simple(r["y"], r["u"], r["v"], w, h)
        assert hashlib.sha256(rgb.tobytes()).hexdigest() == entry["rgb_nofancy_sha256"]


def test_oracle_decoder_errors():
    vp8 = open(os.path.join(GOLD, "libwebp_natural_64x48_q75.vp8"), "rb").read()
    assert O.decode(vp8[:2])[0] != 0
    bad = bytearray(vp8)
    bad[3] = 0
    assert O.decode(bytes(bad))[0] == 10  # Vp8MagicInvalid
    inter = bytearray(vp8)
    inter[0] |= 1
    assert O.decode(bytes(inter))[0] != 0
    # truncated first partition
    assert O.decode(vp8[:12])[0] != 0


@pytest.mark.parametrize("w,h,kind,q,m", [(64, 48, "natural", 75, 4), (300, 257, "natural", 75, 4),
                                          (333, 211, "noise", 75, 6), (256, 256, "flat", 75, 4),
                                          (200, 120, "natural", 20, 2), (96, 80, "natural", 95, 0)])
def test_oracle_encoder_self_consistent(w, h, kind, q, m):
    """Encoder recon == decoder unfiltered recon; libwebp decodes identically."""
    img = synth_rgba(w, h, 0x5EED0000 + w, kind)
    rc, vp8, dbg = O.encode(img, w, h, 3, q, m, debug=True)
    assert rc == 0 and len(vp8) > 10
    rc, r = O.decode(vp8, want_unfiltered=True)
    assert rc == 0
    assert np.array_equal(r["uy"], dbg["recon_y"])
    assert np.array_equal(r["uu"], dbg["recon_u"])
    assert np.array_equal(r["uv"], dbg["recon_v"])
    try:
        W = ctypes.CDLL("libwebp.so.7")
    except OSError:
        return
    W.WebPDecodeYUV.restype = ctypes.c_void_p
    W.WebPDecodeYUV.argtypes = [ctypes.c_char_p, ctypes.c_size_t] + [ctypes.c_void_p] * 6
    pad = len(vp8) & 1
    body = b"WEBP" + b"VP8 " + len(vp8).to_bytes(4, "little") + vp8 + b"\0" * pad
    riff = b"RIFF" + len(body).to_bytes(4, "little") + body
    ww, hh, st, us = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    pu, pv = ctypes.c_void_p(), ctypes.c_void_p()
    py = W.WebPDecodeYUV(riff, len(riff), ctypes.byref(ww), ctypes.byref(hh), ctypes.byref(pu), ctypes.byref(pv),
                         ctypes.byref(st), ctypes.byref(us))
    assert py
    yb = np.ctypeslib.as_array((ctypes.c_uint8 * (st.value * h)).from_address(py)).reshape(h, st.value)[:, :w]
    assert np.array_equal(yb, r["y"].reshape(-1, r["mbw"] * 16)[:h, :w])


def test_oracle_encoder_errors():
    img = synth_rgba(16, 16)
    assert O.encode(img, 0, 16, 3)[0] != 0
    assert O.encode(img[:8], 16, 16, 3)[0] != 0
    assert O.encode(img, 16, 16, 3, quality=101)[0] != 0
