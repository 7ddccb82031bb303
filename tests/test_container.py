"""Host logic, no GPU: the WebP container parse (WebPDecoder::new -> read_data,
decoder/api.rs:334-510) behind zw_webp_parse, on the reference's gallery1
streams (tests/golden/*.vp8, wrapped in the RIFF forms the reference reads)
and on malformed files, with the DecodingError variant each one maps to."""
import os
import struct

import pytest

import zwebp

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _vp8(name="gallery1_1"):
    return open(os.path.join(GOLD, name + ".vp8"), "rb").read()


def _chunk(tag, payload):
    return tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")


def _riff(*chunks):
    body = b"WEBP" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _vp8x(w, h, flags=0):
    return _chunk(b"VP8X", bytes([flags, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little"))


def test_simple_lossy():
    vp8 = _vp8()
    info = zwebp.webp_parse(_riff(_chunk(b"VP8 ", vp8)))
    assert (info["width"], info["height"]) == (550, 368)
    assert info["is_lossy"] and not info["has_alpha"] and not info["is_animated"]
    assert info["vp8_offset"] == 20 and info["vp8_len"] == len(vp8)


def test_extended_lossy_with_metadata_chunks():
    vp8 = _vp8()
    f = _riff(_vp8x(550, 368, flags=0x08), _chunk(b"EXIF", b"x" * 7), _chunk(b"VP8 ", vp8))
    info = zwebp.webp_parse(f)
    assert info["is_lossy"] and (info["width"], info["height"]) == (550, 368)
    assert f[info["vp8_offset"]:info["vp8_offset"] + info["vp8_len"]] == vp8


@pytest.mark.parametrize("mutate,code", [
    (lambda f: b"RIFX" + f[4:], 18),                       # ChunkHeaderInvalid(RIFF)
    (lambda f: f[:8] + b"WEBQ" + f[12:], 19),              # WebpSignatureInvalid
    (lambda f: f[:12] + b"ABCD" + f[16:], 18),             # ChunkHeaderInvalid(first chunk)
    (lambda f: f[:23] + b"\0\0\0" + f[26:], 10),            # Vp8MagicInvalid
    (lambda f: f[:20] + bytes([f[20] | 1]) + f[21:], 16),  # non-keyframe: UnsupportedFeature
    (lambda f: f[:26] + b"\0\0" + f[28:], 21),              # width 0: InconsistentImageSizes
    (lambda f: f[:10], 15),                                 # truncated: BitStreamError
])
def test_malformed(mutate, code):
    f = _riff(_chunk(b"VP8 ", _vp8()))
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.webp_parse(mutate(f))
    assert e.value.code == code


def test_out_of_scope_forms():
    vp8 = _vp8()
    # VP8L (lossless), ALPH-carrying VP8X, animation: outside the lossy block-transform path
    for f in (_riff(_chunk(b"VP8L", b"\x2f" + b"\0" * 8)),
              _riff(_vp8x(550, 368, flags=0x10), _chunk(b"ALPH", b"\0" * 9), _chunk(b"VP8 ", vp8)),
              _riff(_vp8x(550, 368, flags=0x02), _chunk(b"ANIM", b"\0" * 6))):
        with pytest.raises(zwebp.DecodingError) as e:
            zwebp.webp_parse(f)
        assert e.value.code == 5
    # VP8X with no image chunk: ChunkMissing
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.webp_parse(_riff(_vp8x(8, 8)))
    assert e.value.code == 20


def test_add_with_overflow_size():
    """decoder/api.rs:1153 add_with_overflow_size: a RIFF file whose chunk sizes
    overflow when added must be rejected with an error, not crash."""
    b = bytes([0x52, 0x49, 0x46, 0x46, 0xaf, 0x37, 0x80, 0x47, 0x57, 0x45, 0x42, 0x50, 0x6c, 0x64, 0x00, 0x00, 0xff,
               0xff, 0xff, 0xff, 0xfb, 0x7e, 0x73, 0x00, 0x06, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x05, 0x00,
               0x00, 0x00, 0x65, 0x65, 0x65, 0x65, 0x65, 0x65, 0x40, 0xfb, 0xff, 0xff, 0x65, 0x65, 0x65, 0x65, 0x65,
               0x65, 0x65, 0x65, 0x65, 0x65, 0x00, 0x00, 0x00, 0x00, 0x62, 0x00, 0x10, 0x00, 0x00, 0x00, 0x00, 0x00,
               0x00, 0x49, 0x49, 0x54, 0x55, 0x50, 0x4c, 0x54, 0x59, 0x50, 0x45, 0x33, 0x37, 0x44, 0x4d, 0x46])
    with pytest.raises(zwebp.DecodingError):
        zwebp.webp_parse(b)
    for cut in range(0, len(b), 7):  # and every truncation of it
        with pytest.raises(zwebp.DecodingError):
            zwebp.webp_parse(b[:cut])


def test_single_colour_files_parse():
    """decoder/api.rs:1166-1212 imagemagick 2x2 / 3x3 red files: WebPDecoder::new facts."""
    from test_oracle import imagemagick_red
    for n in (2, 3):
        info = zwebp.webp_parse(imagemagick_red(n))
        assert (info["width"], info["height"]) == (n, n) and info["is_lossy"] and not info["has_alpha"]
