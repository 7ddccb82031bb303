"""Token partitions ("optional 8 token partitions").

The reference encoder carries the machinery -- the frame header's
log2(partitions) field (encoder/vp8.rs:352-354) and MB row y's residual tokens
in partition y % n (:1419-1421) -- but always builds one partition (:273,
:1275).  The decoder reads n partitions (decoder/vp8.rs:421-450: the n - 1
3-byte sizes after the first partition, then the data; RFC 6386 9.5).

CPU tests pin the oracle's partitioned streams: the reference-layout decoder
restatement and the system libwebp (an independent decoder) decode every
partition count to the same pixels as the one-partition stream, and the layout
fields are where the format puts them.  GPU tests: the product's partitioned
bitstreams are byte-equal to the oracle's, on the single-frame path (partitions
coded on parallel host threads) and the batch path, and the device decoder
reads them back.
"""
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

SIZES = [(200, 152), (64, 16), (33, 70), (16, 16)]


def _riff_vp8(vp8):
    chunk = b"VP8 " + struct.pack("<I", len(vp8)) + vp8 + (b"\0" if len(vp8) & 1 else b"")
    body = b"WEBP" + chunk
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _libwebp_rgba(vp8):
    riff = _riff_vp8(vp8)
    w, h = ctypes.c_int(), ctypes.c_int()
    p = _W.WebPDecodeRGBA(riff, len(riff), ctypes.byref(w), ctypes.byref(h))
    assert p, "libwebp refused the stream"
    out = np.ctypeslib.as_array((ctypes.c_uint8 * (w.value * h.value * 4)).from_address(p)).copy()
    _W.WebPFree(p)
    return out


def _parts(vp8, n):
    tag = vp8[0] | (vp8[1] << 8) | (vp8[2] << 16)
    off = 10 + (tag >> 5)
    sizes = [int.from_bytes(vp8[off + 3 * i: off + 3 * i + 3], "little") for i in range(n - 1)]
    rest = len(vp8) - off - 3 * (n - 1) - sum(sizes)
    return sizes + [rest]


@pytest.mark.parametrize("w,h", SIZES)
def test_oracle_partitions_decode_identically(w, h):
    img = synth_rgba(w, h, 0x5EED0000 + w)
    rc, one, _ = O.encode(img, w, h, 3, 75, 4, nparts=1)
    assert rc == 0
    rc1, base = O.decode(one)
    assert rc1 == 0
    ref_px = _libwebp_rgba(one) if _W is not None else None
    for n in (2, 4, 8):
        rc, b, _ = O.encode(img, w, h, 3, 75, 4, nparts=n)
        assert rc == 0
        # the first partition differs from the one-partition stream only in the
        # 2-bit partition count, so the MB headers are the same bits
        sizes = _parts(b, n)
        assert all(s >= 0 for s in sizes) and len(sizes) == n
        rc2, r = O.decode(b)
        assert rc2 == 0
        for k in ("y", "u", "v"):
            assert np.array_equal(r[k], base[k]), (n, k)
        if _W is not None:
            assert np.array_equal(_libwebp_rgba(b), ref_px), n


def test_oracle_partition_rows():
    """MB row y's tokens sit in partition y % n: with n >= the MB rows every row
    has its own partition, and a row's partition is the same bytes whatever n is
    as long as that row is the only one in it."""
    w, h = 96, 64  # 4 MB rows
    img = synth_rgba(w, h, 0x5EED0007)
    parts = {}
    for n in (4, 8):
        rc, b, _ = O.encode(img, w, h, 3, 75, 4, nparts=n)
        assert rc == 0
        parts[n] = b
    t4 = _parts(parts[4], 4)
    t8 = _parts(parts[8], 8)
    assert t4 == t8[:4]
    # partitions 4..7 of the 8-way stream carry no rows: an empty bool-coder flush
    assert len(set(t8[4:])) == 1


def test_oracle_partition_count_checked():
    img = synth_rgba(32, 32, 1)
    for n in (0, 3, 5, 16):
        rc, _, _ = O.encode(img, 32, 32, 3, 75, 4, nparts=n)
        assert rc != 0, n


# ---------------------------------------------------------------------------
# GPU: the product against the oracle
# ---------------------------------------------------------------------------


@pytest.fixture(scope="module")
def ctx():
    import zwebp
    return zwebp.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", SIZES + [(1920, 1080)])
def test_gpu_partitions_single_frame(ctx, w, h):
    import zwebp
    img = synth_rgba(w, h, 0x5EED0000 + h)
    counts = (1, 2, 4, 8) if w < 1000 else (1, 8)
    for n in counts:
        out = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx, token_partitions=n)
        rc, ref, _ = O.encode(img, w, h, 3, 75, 4, nparts=n)
        assert rc == 0
        assert out == ref, (w, h, n)
    # the device decoder reads the partitioned stream back
    fr = zwebp.vp8_decode_frame(out, ctx=ctx)
    rc, r = O.decode(out)
    assert rc == 0
    assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])


@pytest.mark.gpu
def test_gpu_partitions_batch(ctx):
    import zwebp
    w, h = 160, 128
    imgs = [synth_rgba(w, h, 0x5EED0100 + i) for i in range(5)]
    outs = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx, token_partitions=4)
    for i, img in enumerate(imgs):
        rc, ref, _ = O.encode(img, w, h, 3, 75, 4, nparts=4)
        assert rc == 0 and outs[i] == ref, i
    # the single-frame path with one partition still gives the reference bytes
    one = zwebp.encode_frame_lossy(imgs[0], w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    assert one == O.encode(imgs[0], w, h, 3, 75, 4)[1]


@pytest.mark.gpu
def test_gpu_partition_count_checked(ctx):
    import zwebp
    img = synth_rgba(32, 32, 1)
    for n in (0, 3, 16):
        with pytest.raises(zwebp.EncodingError):
            zwebp.encode_frame_lossy(img, 32, 32, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx, token_partitions=n)
