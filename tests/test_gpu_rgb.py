"""GPU parity of the decoder's YUV -> RGB(A) stage (SURVEY §8(f) row 2:
fill_rgb_buffer_fancy / fill_rgb_buffer_simple, decoder/yuv.rs:82-515) and the
lossy WebP decode entry points built on it (decode_rgb / decode_rgba /
WebPDecoder::read_image, decoder/api.rs:640-993).

Pinned against the reference's own RGB goldens (tests/reference/gallery1 and
gallery1_nofancy PNG digests in tests/golden/decode_golden.json, i.e. the
reference's tests/decode.rs reftests) and bit-exact against the oracle
(oracle/or_dsp.c) on random planes of every parity of width and height."""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

import oracle_lib as O
import zwebp
from zwebp.synth import synth_rgba

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BIL, SIMPLE = zwebp.UpsamplingMethod.Bilinear, zwebp.UpsamplingMethod.Simple


@pytest.fixture(scope="module")
def ctx():
    return zwebp.Context(0)


def _manifest():
    with open(os.path.join(GOLD, "decode_golden.json")) as f:
        return json.load(f)["streams"]


def _oracle_rgb(y, u, v, w, h, bpp, up):
    fn = O.yuv_to_rgb_fancy if up == BIL else O.yuv_to_rgb_simple
    return fn(y, u, v, w, h, bpp)


def _riff(vp8):
    body = b"WEBP" + b"VP8 " + struct.pack("<I", len(vp8)) + vp8 + (b"\0" if len(vp8) & 1 else b"")
    return b"RIFF" + struct.pack("<I", len(body)) + body


@pytest.mark.parametrize("w,h", [(1, 1), (1, 2), (2, 1), (2, 2), (3, 3), (5, 4), (4, 5), (17, 9), (16, 16),
                                 (33, 31), (250, 31), (1920, 1080)])
@pytest.mark.parametrize("bpp", [3, 4])
@pytest.mark.parametrize("up", [BIL, SIMPLE])
def test_yuv_to_rgb_kernel(ctx, w, h, bpp, up):
    rng = np.random.default_rng(w * 7919 + h * 31 + bpp + 5 * up)
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    y = rng.integers(0, 256, mbw * 16 * mbh * 16, dtype=np.uint8)
    u = rng.integers(0, 256, mbw * 8 * mbh * 8, dtype=np.uint8)
    v = rng.integers(0, 256, mbw * 8 * mbh * 8, dtype=np.uint8)
    got = zwebp.yuv_to_rgb(y, u, v, w, h, mbw * 16, mbw * 8, bpp, up, ctx=ctx)
    exp = _oracle_rgb(y, u, v, w, h, bpp, up)
    assert np.array_equal(got.reshape(-1), exp)


@pytest.mark.parametrize("bpp", [3, 4])
def test_yuv_to_rgb_exhaustive(ctx, bpp):
    """Every (y, u, v) triple exactly once (yuv_to_r/g/b, yuv.rs:63-78, through the
    kernel's u16-pair arithmetic): simple upsampling of a 4096 x 4096 frame whose
    chroma sample (cx, cy) is (u, v) = (cx % 256, cy % 256) -- each pair 64 times,
    occurrence o = cx // 256 + 8 (cy // 256) -- and whose four pixels under it
    carry y = 4 o + 0..3."""
    w = h = 4096
    cy, cx = np.meshgrid(np.arange(h // 2), np.arange(w // 2), indexing="ij")
    u = (cx % 256).astype(np.uint8)
    v = (cy % 256).astype(np.uint8)
    o = (cx // 256 + 8 * (cy // 256)).astype(np.int32)
    py, px = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    y = (4 * o[py // 2, px // 2] + (px & 1) + 2 * (py & 1)).astype(np.uint8)
    triples = (y.astype(np.int64) << 16) | (u[py // 2, px // 2].astype(np.int64) << 8) | v[py // 2, px // 2]
    assert np.unique(triples).size == 1 << 24  # (the construction covers the cube)
    y, u, v = y.reshape(-1), u.reshape(-1), v.reshape(-1)
    got = zwebp.yuv_to_rgb(y, u, v, w, h, w, w // 2, bpp, SIMPLE, ctx=ctx)
    assert np.array_equal(got.reshape(-1), _oracle_rgb(y, u, v, w, h, bpp, SIMPLE))


def test_yuv_to_rgb_extremes(ctx):
    # clip both ends: every (y, u, v) corner of the cube
    w, h = 16, 16
    y = np.zeros(256, np.uint8)
    u = np.zeros(64, np.uint8)
    v = np.zeros(64, np.uint8)
    for i, (a, b, c) in enumerate([(0, 0, 0), (255, 255, 255), (0, 255, 0), (255, 0, 255), (0, 0, 255),
                                   (255, 255, 0), (128, 0, 255), (16, 240, 16)]):
        y[i * 32:(i + 1) * 32] = a
        u[i * 8:(i + 1) * 8] = b
        v[i * 8:(i + 1) * 8] = c
    for up in (BIL, SIMPLE):
        got = zwebp.yuv_to_rgb(y, u, v, w, h, 16, 8, 3, up, ctx=ctx)
        assert np.array_equal(got.reshape(-1), _oracle_rgb(y, u, v, w, h, 3, up))


@pytest.mark.parametrize("entry", [e for e in _manifest() if "rgb_sha256" in e], ids=lambda e: e["name"])
def test_decode_rgb_reference_goldens(ctx, entry):
    """The reference's own reftests (tests/decode.rs:189-202): gallery1 fancy and
    nofancy PNG pixels, regression/dark (a 1x1 frame) and every frame of
    animated/random_lossy (full-canvas opaque keyframes, which composite_frame
    copies unchanged, decoder/extended.rs:53-62 / :134), byte for byte through
    k_dec_recon / k_loopfilter / k_yuv2rgb."""
    vp8 = open(os.path.join(GOLD, entry["name"] + ".vp8"), "rb").read()
    w, h = entry["width"], entry["height"]
    rgb = zwebp.vp8_decode_rgb(vp8, 3, BIL, ctx=ctx)
    assert rgb.shape == (h, w, 3)
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == entry["rgb_sha256"]
    nofancy = entry.get("rgb_nofancy_sha256")
    if nofancy:
        rgb = zwebp.vp8_decode_rgb(vp8, 3, SIMPLE, ctx=ctx)
        assert hashlib.sha256(rgb.tobytes()).hexdigest() == nofancy
    # the container path: decode_rgb / decode_rgba / WebPDecoder
    riff = _riff(vp8)
    flat, ww, hh = zwebp.decode_rgb(riff, ctx=ctx)
    assert (ww, hh) == (w, h) and hashlib.sha256(flat.tobytes()).hexdigest() == entry["rgb_sha256"]
    rgba, ww, hh = zwebp.decode_rgba(riff, ctx=ctx)
    rgba = rgba.reshape(h, w, 4)
    assert (rgba[..., 3] == 255).all()
    assert hashlib.sha256(np.ascontiguousarray(rgba[..., :3]).tobytes()).hexdigest() == entry["rgb_sha256"]
    dec = zwebp.WebPDecoder(riff, ctx=ctx)
    assert dec.dimensions() == (w, h) and dec.is_lossy() and not dec.has_alpha()
    assert dec.output_buffer_size() == w * h * 3
    if nofancy:
        dec.set_lossy_upsampling(SIMPLE)
    buf = bytearray(dec.output_buffer_size())
    dec.read_image(buf)
    assert hashlib.sha256(bytes(buf)).hexdigest() == (nofancy or entry["rgb_sha256"])


@pytest.mark.parametrize("entry", _manifest(), ids=lambda e: e["name"])
def test_decode_rgb_matches_oracle(ctx, entry):
    vp8 = open(os.path.join(GOLD, entry["name"] + ".vp8"), "rb").read()
    rc, r = O.decode(vp8)
    assert rc == 0
    w, h = entry["width"], entry["height"]
    for bpp in (3, 4):
        for up in (BIL, SIMPLE):
            got = zwebp.vp8_decode_rgb(vp8, bpp, up, ctx=ctx)
            exp = _oracle_rgb(r["y"], r["u"], r["v"], w, h, bpp, up)
            assert np.array_equal(got.reshape(-1), exp), (bpp, up)


@pytest.mark.parametrize("chunk", [None, "2"])
def test_decode_rgb_batch(ctx, monkeypatch, chunk):
    """chunk "2": the double-buffered chunk pipeline over 3 chunks (ragged last)."""
    if chunk:
        monkeypatch.setenv("ZW_DEC_CHUNK", chunk)
    w, h = 161, 97
    streams = [O.encode(synth_rgba(w, h, 0x5EED0000 + i), w, h, 3, 20 + 15 * i, 4)[1] for i in range(5)]
    imgs = zwebp.decode_rgb_batch(streams, 4, BIL, ctx=ctx)
    assert zwebp.decode_rgb_kernel_ms(ctx=ctx) > 0
    for s, img in zip(streams, imgs):
        rc, r = O.decode(s)
        assert np.array_equal(img.reshape(-1), _oracle_rgb(r["y"], r["u"], r["v"], w, h, 4, BIL))


@pytest.mark.parametrize("bpp,pad", [(3, 0), (4, 0), (3, 13), (4, 64)])
@pytest.mark.parametrize("chunk", [None, "2"])
def test_decode_rgb_batch_into(ctx, monkeypatch, bpp, pad, chunk):
    """decode_rgba_into / decode_rgb_into semantics (api.rs:1004-1128), batched:
    the caller's buffers with a row stride; the padding bytes stay untouched."""
    if chunk:
        monkeypatch.setenv("ZW_DEC_CHUNK", chunk)
    w, h = 161, 97
    streams = [O.encode(synth_rgba(w, h, 0x5EED0200 + i), w, h, 3, 30 + 10 * i, 4)[1] for i in range(5)]
    stride = w * bpp + pad
    outs = [np.full(stride * h + 7, 0xA5, np.uint8) for _ in streams]
    dims = zwebp.decode_rgb_batch_into(streams, outs, bpp, BIL, stride_bytes=stride, ctx=ctx)
    assert dims == [(w, h)] * len(streams)
    for s, o in zip(streams, outs):
        rc, r = O.decode(s)
        rows = o[:stride * h].reshape(h, stride)
        exp = _oracle_rgb(r["y"], r["u"], r["v"], w, h, bpp, BIL).reshape(h, w * bpp)
        assert np.array_equal(rows[:, :w * bpp], exp)
        assert np.all(rows[:, w * bpp:] == 0xA5) and np.all(o[stride * h:] == 0xA5)


def test_decode_rgb_into_errors(ctx):
    vp8 = open(os.path.join(GOLD, "libwebp_natural_64x48_q75.vp8"), "rb").read()
    out = np.zeros(64 * 48 * 4, np.uint8)
    with pytest.raises(zwebp.DecodingError) as e:  # stride below width * bpp
        zwebp.decode_rgb_batch_into([vp8], [out], 4, BIL, stride_bytes=64 * 4 - 1, ctx=ctx)
    assert e.value.code == 3
    with pytest.raises(zwebp.DecodingError) as e:  # buffer below stride * height
        zwebp.decode_rgb_batch_into([vp8], [out[:-1]], 4, BIL, ctx=ctx)
    assert e.value.code == 3
    with pytest.raises(zwebp.DecodingError):
        zwebp.decode_rgba_into(_riff(vp8), out, 64 * 4 + 1, ctx=ctx)  # needs stride * height > buffer


def test_decode_rgba_into_container(ctx):
    """decode_rgba_into / decode_rgb_into of a lossy RIFF file == decode_rgba / decode_rgb."""
    vp8 = open(os.path.join(GOLD, "libwebp_natural_64x48_q75.vp8"), "rb").read()
    riff = _riff(vp8)
    for fn_into, fn, bpp in ((zwebp.decode_rgba_into, zwebp.decode_rgba, 4), (zwebp.decode_rgb_into, zwebp.decode_rgb, 3)):
        stride = 64 * bpp + 8
        out = np.zeros(stride * 48, np.uint8)
        assert fn_into(riff, out, stride, ctx=ctx) == (64, 48)
        flat, w, h = fn(riff, ctx=ctx)
        assert np.array_equal(out.reshape(48, stride)[:, :64 * bpp].reshape(-1), flat)


def test_encode_decode_rgb_roundtrip(ctx):
    """Our encoder -> RIFF -> our RGB decoder == oracle decode + oracle upsampling."""
    w, h = 333, 211
    img = np.ascontiguousarray(synth_rgba(w, h, 0x5EED0042)[..., :3])
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    riff = bytes(enc.encode(img, w, h, zwebp.ColorType.Rgb8))
    flat, ww, hh = zwebp.decode_rgb(riff, ctx=ctx)
    rc, r = O.decode(O.riff_vp8_chunk(riff))
    assert (ww, hh) == (w, h)
    assert np.array_equal(flat, _oracle_rgb(r["y"], r["u"], r["v"], w, h, 3, BIL))
    # lossy at Q75: close to the source
    assert np.abs(flat.reshape(h, w, 3).astype(int) - img.astype(int)).mean() < 8


def test_decode_rgb_errors(ctx):
    vp8 = open(os.path.join(GOLD, "libwebp_natural_64x48_q75.vp8"), "rb").read()
    with pytest.raises(zwebp.DecodingError):
        zwebp.vp8_decode_rgb(vp8[:20], 3, BIL, ctx=ctx)
    with pytest.raises(zwebp.ZwError) as e:
        zwebp.vp8_decode_rgb(vp8, 2, BIL, ctx=ctx)
    assert e.value.code == 3
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.decode_rgb(b"RIFF\0\0\0\0WEBQ", ctx=ctx)
    assert e.value.code == 19


# --------------------------------------------------------------------------
# WebPEncoder::encode, lossy with alpha (encoder/api.rs:1291-1398):
# VP8X + ALPH (encode_alpha_lossless) + "VP8 " (the GPU encoder)
# --------------------------------------------------------------------------
def _chunk(tag, payload):
    return tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")


def _riff_chunks(*chunks):
    body = b"WEBP" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


@pytest.mark.parametrize("w,h,color", [(96, 80, 3), (33, 17, 3), (64, 48, 1)])
def test_webp_encoder_lossy_with_alpha(ctx, w, h, color):
    rgba = synth_rgba(w, h, 0x5EED0100 + w, "natural").copy()
    rgba[..., 3] = (np.arange(w)[None, :] * 4 + np.arange(h)[:, None]) % 256  # non-trivial alpha
    img = rgba if color == 3 else np.ascontiguousarray(rgba[..., [1, 3]])
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    enc.set_exif_metadata(b"exif")
    riff = bytes(enc.encode(img, w, h, color))
    rc, vp8, _ = O.encode(img, w, h, color, 75, 4)
    rc2, alph = O.encode_alpha(img, w, h, color)
    assert rc == 0 and rc2 == 0
    vp8x = bytes([0x18, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little")
    assert riff == _riff_chunks(_chunk(b"VP8X", vp8x), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8),
                                _chunk(b"EXIF", b"exif"))
    # the decoder side reads the container (ALPH decoding is outside the lossy path)
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.decode_rgba(riff, ctx=ctx)
    assert e.value.code == 5
