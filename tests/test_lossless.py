"""The lossless side of the container: encode_frame_lossless
(encoder/api.rs:945-1173, the VP8L coder behind EncoderParams::lossless) and
encode_alpha_lossless (:1175-1222, the ALPH chunk of every RGBA / LA lossy
encode).  CPU tests: the oracle restatement round-trips through the system
libwebp decoder exactly as the reference's own roundtrip_libwebp tests do
(api.rs tests: random 256x256 images, every color type, predictor on and off),
and the product's host coder (libzwebp.so, no device needed) is byte-identical
to the oracle."""
import ctypes
import struct

import numpy as np
import pytest

import oracle_lib as O
from zwebp.synth import synth_rgba

try:
    _W = ctypes.CDLL("libwebp.so.7")
    _W.WebPDecodeRGBA.restype = ctypes.c_void_p
    _W.WebPDecodeRGBA.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    _W.WebPFree.argtypes = [ctypes.c_void_p]
except OSError:  # pragma: no cover - the GPU box image may lack it
    _W = None

BPP = {0: 1, 1: 2, 2: 3, 3: 4}


def _chunk(tag, payload):
    return tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")


def _riff(*chunks):
    body = b"WEBP" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _libwebp_rgba(riff):
    w, h = ctypes.c_int(), ctypes.c_int()
    p = _W.WebPDecodeRGBA(riff, len(riff), ctypes.byref(w), ctypes.byref(h))
    assert p, "libwebp refused the stream"
    out = np.ctypeslib.as_array((ctypes.c_uint8 * (w.value * h.value * 4)).from_address(p)).copy()
    _W.WebPFree(p)
    return out.reshape(h.value, w.value, 4)


def _to_rgba(img, color):
    a = img.reshape(-1, BPP[color])
    if color == 0:
        return np.stack([a[:, 0], a[:, 0], a[:, 0], np.full(len(a), 255, np.uint8)], 1)
    if color == 1:
        return np.stack([a[:, 0], a[:, 0], a[:, 0], a[:, 1]], 1)
    if color == 2:
        return np.concatenate([a, np.full((len(a), 1), 255, np.uint8)], 1)
    return a


def _images():
    rng = np.random.default_rng(7)
    yield "random256", 256, 256, rng.integers(0, 256, (256, 256, 4), dtype=np.uint8)
    yield "natural333x211", 333, 211, synth_rgba(333, 211, 0x5EED0001, "natural")
    yield "flat17x9", 17, 9, np.full((9, 17, 4), 77, np.uint8)
    yield "runs", 300, 40, np.repeat(rng.integers(0, 3, (40, 300 // 50, 4), dtype=np.uint8) * 100, 50, axis=1)
    yield "tiny1x1", 1, 1, np.array([[[1, 2, 3, 4]]], np.uint8)
    # skewed histogram: deep Huffman trees (length limiting at 15)
    fib = np.concatenate([np.full(int(1.6 ** k), k, np.uint8) for k in range(24)])
    n = 512 * 64
    g = np.resize(fib, n)
    rng.shuffle(g)
    sk = np.stack([g, g, g, g], 1).reshape(64, 512, 4)
    yield "skewed512x64", 512, 64, sk
    # length limiting with tie groups split across code lengths: the symbols of
    # equal frequency that get the longer codes are chosen by the order of the
    # reference's sort_unstable_by_key (api.rs:259-260), not by symbol order
    # (checked: with a stable order instead, both predictor settings give other bytes)
    parts = [np.full(int(1.6 ** k), 100 + k, np.uint8) for k in range(22)]
    parts += [np.full(c, s, np.uint8) for s, c in zip(range(0, 90), [1, 2, 3] * 30)]
    g = np.resize(np.concatenate(parts), 640 * 256)
    rng.shuffle(g)
    yield "tied640x256", 640, 256, np.stack([g, g[::-1], g, g], 1).reshape(256, 640, 4)


IMAGES = list(_images())


@pytest.mark.skipif(_W is None, reason="system libwebp not available")
@pytest.mark.parametrize("name,w,h,img", IMAGES, ids=[i[0] for i in IMAGES])
@pytest.mark.parametrize("color", [0, 1, 2, 3])
@pytest.mark.parametrize("pred", [True, False])
def test_oracle_lossless_roundtrip_libwebp(name, w, h, img, color, pred):
    src = np.ascontiguousarray(img[..., :BPP[color]]) if color >= 2 else \
        np.ascontiguousarray(img[..., [1, 3]][..., :BPP[color]])
    rc, vp8l = O.encode_lossless(src, w, h, color, pred)
    assert rc == 0 and vp8l[0] == 0x2F
    dec = _libwebp_rgba(_riff(_chunk(b"VP8L", vp8l)))
    assert np.array_equal(dec.reshape(-1, 4), _to_rgba(src, color))


@pytest.mark.skipif(_W is None, reason="system libwebp not available")
@pytest.mark.parametrize("name,w,h,img", IMAGES[:4], ids=[i[0] for i in IMAGES[:4]])
def test_oracle_alpha_chunk_roundtrip_libwebp(name, w, h, img):
    """VP8X + ALPH + VP8: libwebp recovers the alpha plane exactly."""
    rgba = np.ascontiguousarray(img)
    rc, alph = O.encode_alpha(rgba, w, h, 3)
    assert rc == 0 and alph[0] == 1
    rc, vp8, _ = O.encode(rgba, w, h, 3, 75, 4)
    assert rc == 0
    vp8x = bytes([0x10, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little")
    dec = _libwebp_rgba(_riff(_chunk(b"VP8X", vp8x), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8)))
    assert np.array_equal(dec[..., 3], rgba[..., 3])


def _stable_order(keys):
    return np.argsort(np.asarray(keys, np.int64), kind="stable")


@pytest.mark.parametrize("n,seed,span", [(0, 0, 1), (1, 0, 1), (5, 1, 3), (20, 2, 4), (21, 3, 4), (33, 4, 5),
                                         (40, 5, 2), (64, 6, 9), (280, 7, 6), (280, 8, 1), (256, 9, 40),
                                         (1000, 10, 3), (2328, 11, 50)])
def test_rust_sort_unstable_invariants(n, seed, span):
    """The oracle's ipnsort restatement: a permutation, sorted by key, stable
    (insertion sort) up to 20 elements, and a sorted / strictly descending
    whole-slice run is returned as sorted by the run detection alone."""
    keys = np.random.default_rng(seed).integers(0, span, n).astype(np.uint32)
    idx, k = O.rust_sort_unstable_by_key(keys)
    assert sorted(idx.tolist()) == list(range(n))
    assert np.array_equal(keys[idx], k) and np.all(np.diff(k.astype(np.int64)) >= 0)
    if n <= 20:
        assert np.array_equal(idx, _stable_order(keys))
    asc = np.sort(keys)
    assert np.array_equal(O.rust_sort_unstable_by_key(asc)[0], np.arange(n))
    desc = np.arange(n, 0, -1, dtype=np.uint32)
    assert np.array_equal(O.rust_sort_unstable_by_key(desc)[0], np.arange(n)[::-1])


def test_rust_sort_unstable_is_not_stable():
    """Above the small-sort sizes the partitioning reorders equal keys, which
    is the case the length-limit reassignment depends on."""
    keys = np.random.default_rng(12).integers(0, 3, 280).astype(np.uint32)
    idx, _ = O.rust_sort_unstable_by_key(keys)
    assert not np.array_equal(idx, _stable_order(keys))


# Drift guards.  Where these came from: the oracle's restatement of
# Rust 1.92 core::slice::sort::unstable (ipnsort) at commit c7fefce, reviewed
# against that algorithm (insertion sort <= 20, run detection, limit
# 2*ilog2(len|1), small-sort cutoff 32 for (usize, u32), median3_rec, ancestor
# pivot, cyclic Lomuto partition, heapsort fallback).  No Rust toolchain exists
# here, so they pin the restatement against later edits, NOT against Rust itself:
# parity with the reference's VP8L bytes stays unpinned (no VP8L byte fixtures
# ship with the reference).
PINNED_SORT = [
    (np.array([(i * 7 + 3) % 5 for i in range(48)], np.uint32),
     [1, 6, 11, 16, 21, 26, 31, 36, 41, 46, 4, 9, 14, 19, 24, 29, 34, 39, 44, 42, 2, 22, 27, 12, 32, 37, 7, 17, 47,
      20, 10, 25, 5, 30, 35, 15, 40, 0, 45, 23, 28, 13, 33, 3, 38, 43, 18, 8]),
    (np.array([(i * i * 13 + 7) % 9 for i in range(100)], np.uint32),
     [1, 8, 10, 17, 19, 26, 28, 35, 37, 44, 46, 53, 55, 62, 64, 71, 73, 80, 82, 89, 91, 98, 52, 97, 25, 7, 29, 34, 2,
      38, 43, 11, 47, 56, 61, 65, 70, 16, 74, 79, 83, 88, 20, 92, 63, 99, 33, 48, 51, 0, 12, 54, 6, 57, 60, 27, 15, 36,
      66, 24, 9, 30, 72, 39, 75, 78, 18, 81, 84, 87, 42, 90, 21, 3, 93, 96, 45, 69, 32, 40, 67, 68, 5, 41, 13, 85, 86,
      49, 14, 31, 23, 4, 50, 58, 94, 95, 76, 77, 22, 59]),
]
# SHA-256 of the tie-split image's VP8L (predictor on / off) and ALPH payloads,
# same provenance: the oracle at c7fefce.
PINNED_TIED = {"vp8l_pred": "6cbb062244e0a3d8ecf6570b386da2e0e7f8f8b77f9fa90a9ccfee458f528e5a",
               "vp8l_nopred": "34ac80c9cc73112b21fc81bd6b6848cac38b0e8e43c566bbd952420bbfa95a0e",
               "alph": "ac975ba636b085ad030b9db4dec047dfd098e31abdcefb0b730ba50043dc83b0"}


@pytest.mark.parametrize("case", range(len(PINNED_SORT)))
def test_rust_sort_unstable_pinned(case):
    keys, want = PINNED_SORT[case]
    idx, _ = O.rust_sort_unstable_by_key(keys)
    assert idx.tolist() == want


def test_tie_split_bytes_pinned():
    """The oracle AND the product's host coder give the pinned bytes on the image
    whose length-limited trees split tie groups (so both sort restatements are
    held to the same permutation, not just to each other)."""
    import hashlib
    name, w, h, img = next(i for i in IMAGES if i[0] == "tied640x256")
    img = np.ascontiguousarray(img)
    for pred, key in ((True, "vp8l_pred"), (False, "vp8l_nopred")):
        rc, ref = O.encode_lossless(img, w, h, 3, pred)
        assert rc == 0 and hashlib.sha256(bytes(ref)).hexdigest() == PINNED_TIED[key]
        assert hashlib.sha256(bytes(zwebp.encode_frame_lossless(img, w, h, 3, pred))).hexdigest() == PINNED_TIED[key]
    rc, a = O.encode_alpha(img, w, h, 3)
    assert rc == 0 and hashlib.sha256(bytes(a)).hexdigest() == PINNED_TIED["alph"]
    assert hashlib.sha256(bytes(zwebp.encode_alpha(img, w, h, 3))).hexdigest() == PINNED_TIED["alph"]


def test_oracle_lossless_errors():
    img = np.zeros((4, 4, 4), np.uint8)
    assert O.encode_lossless(img, 4, 4, 3)[0] == 0
    assert O.encode_lossless(img, 4, 5, 3)[0] == 2          # length mismatch (the reference asserts)
    assert O.encode_lossless(np.zeros(0, np.uint8), 0, 4, 3)[0] != 0
    big = np.zeros(16385 * 4, np.uint8)
    assert O.encode_lossless(big, 16385, 1, 3)[0] == 1      # InvalidDimensions


# --------------------------------------------------------------------------
# the product's host coder (libzwebp.so; no device needed) == the oracle
# --------------------------------------------------------------------------
import zwebp  # noqa: E402


def _src(img, color):
    return np.ascontiguousarray(img[..., :BPP[color]]) if color >= 2 else \
        np.ascontiguousarray(img[..., [1, 3]][..., :BPP[color]])


@pytest.mark.parametrize("name,w,h,img", IMAGES, ids=[i[0] for i in IMAGES])
@pytest.mark.parametrize("color", [0, 1, 2, 3])
@pytest.mark.parametrize("pred", [True, False])
def test_product_lossless_matches_oracle(name, w, h, img, color, pred):
    src = _src(img, color)
    rc, ref = O.encode_lossless(src, w, h, color, pred)
    assert rc == 0
    assert zwebp.encode_frame_lossless(src, w, h, color, pred) == ref


@pytest.mark.parametrize("name,w,h,img", IMAGES, ids=[i[0] for i in IMAGES])
@pytest.mark.parametrize("color", [1, 3])
def test_product_alpha_matches_oracle(name, w, h, img, color):
    src = _src(img, color)
    rc, ref = O.encode_alpha(src, w, h, color)
    assert rc == 0
    assert zwebp.encode_alpha(src, w, h, color) == ref


def test_product_lossless_container():
    """WebPEncoder with default (lossless) params: simple VP8L container, and VP8X
    with ICCP / EXIF / XMP chunks in the reference's order and flags."""
    w, h = 64, 48
    img = synth_rgba(w, h, 0x5EED0007, "natural")
    rc, vp8l = O.encode_lossless(img, w, h, 3, True)
    enc = zwebp.WebPEncoder()
    riff = bytes(enc.encode(img, w, h, zwebp.ColorType.Rgba8))
    assert riff == _riff(_chunk(b"VP8L", vp8l))
    enc = zwebp.WebPEncoder()
    enc.set_icc_profile(b"icc-profile")
    enc.set_exif_metadata(b"exif!")
    enc.set_xmp_metadata(b"<xmp/>")
    riff = bytes(enc.encode(img, w, h, zwebp.ColorType.Rgba8))
    vp8x = bytes([0x3C, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little")
    assert riff == _riff(_chunk(b"VP8X", vp8x), _chunk(b"ICCP", b"icc-profile"), _chunk(b"VP8L", vp8l),
                         _chunk(b"EXIF", b"exif!"), _chunk(b"XMP ", b"<xmp/>"))
    if _W is not None:
        assert np.array_equal(_libwebp_rgba(riff), img)


def test_product_lossless_errors():
    img = np.zeros((4, 4, 4), np.uint8)
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossless(img, 4, 5, 3)
    assert e.value.code == 2
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossless(np.zeros(16385 * 4, np.uint8), 16385, 1, 3)
    assert e.value.code == 1
    with pytest.raises(zwebp.EncodingError):
        zwebp.encode_alpha(img, 4, 4, 2)  # no alpha channel
