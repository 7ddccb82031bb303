"""GPU: the encoder at the shapes the benchmark times (BASELINE configs 4 and 5),
the full WebP container for alpha inputs, and failure reporting of the
row-parallel decode.

* A 512-frame 1080p batch through zwebp.Pipeline at the default lane and chunk
  shape (256-frame launches, multi-chunk, streaming repeat) -- every output is
  compared with the oracle's bitstream of its source frame.
* A 256-frame 4K batch (one default launch of 3840x2160 frames).
* WebPEncoder::encode for RGBA8 / LA8 (api.rs:1291-1398): VP8X + ALPH + VP8
  (+ ICCP / EXIF / XMP) byte-equal to the oracle's pieces in the reference's
  chunk order; libwebp round trip when the system library is present.
"""
import os
import ctypes
import struct

import numpy as np
import pytest

import oracle_lib as O
import zwebp
from zwebp.shard import frame_seed
from zwebp.synth import synth_rgba

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    return zwebp.Context(0)


def _batch_check(ctx, n, w, h, distinct, repeat):
    imgs = [synth_rgba(w, h, frame_seed(i)) for i in range(distinct)]
    refs = []
    for im in imgs:
        rc, ref, _ = O.encode(im, w, h, 3, 75, 4)
        assert rc == 0
        refs.append(ref)
    p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    try:
        for i in range(n):
            p.upload(i, imgs[i % distinct])
        assert p.launch_frames == min(n, 256)  # default chunk = one frame per CU
        for run in range(2):
            if run == 0:
                p.encode()
            else:
                p.encode_repeat(repeat)
            bad = [i for i in range(n) if p.output(i) != refs[i % distinct]]
            assert not bad, f"run {run}: {len(bad)} of {n} frames differ, first {bad[0]}"
    finally:
        p.close()


def test_default_shape_1080p_batch_512(ctx):
    """BASELINE config 4 shape: 512 x 1920x1080, default lanes/chunks (2 launches
    of 256 frames per pass), single encode and a 2-batch streaming repeat."""
    _batch_check(ctx, 512, 1920, 1080, 4, 2)


def test_4k_batch_default_launch(ctx):
    """BASELINE config 5 frame size: one default launch of 256 x 3840x2160."""
    _batch_check(ctx, 256, 3840, 2160, 2, 1)


# --------------------------------------------------------------------------
# full container for alpha inputs
# --------------------------------------------------------------------------
def _chunk(tag, payload):
    return tag + struct.pack("<I", len(payload)) + payload + (b"\0" if len(payload) & 1 else b"")


def _riff(*chunks):
    body = b"WEBP" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _vp8x(w, h, flags):
    return _chunk(b"VP8X", bytes([flags, 0, 0, 0]) + (w - 1).to_bytes(3, "little") + (h - 1).to_bytes(3, "little"))


try:
    _W = ctypes.CDLL("libwebp.so.7")
    _W.WebPDecodeRGBA.restype = ctypes.c_void_p
    _W.WebPDecodeRGBA.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    _W.WebPFree.argtypes = [ctypes.c_void_p]
except OSError:  # the GPU box image may lack it
    _W = None


def _alpha_img(w, h, color):
    rgba = synth_rgba(w, h, 0x5EED0042)
    yy, xx = np.mgrid[0:h, 0:w]
    rgba[..., 3] = np.where((xx // 7 + yy // 5) % 3 == 0, 255, (xx * 3 + yy) & 255).astype(np.uint8)
    if color == zwebp.ColorType.La8:
        return np.ascontiguousarray(rgba[..., [0, 3]])
    return rgba


@pytest.mark.parametrize("color", [zwebp.ColorType.Rgba8, zwebp.ColorType.La8])
@pytest.mark.parametrize("w,h", [(160, 96), (333, 211), (1920, 1080)])
def test_webp_container_alpha(ctx, color, w, h):
    img = _alpha_img(w, h, color)
    rc, vp8, _ = O.encode(img, w, h, color, 75, 4)
    assert rc == 0
    rc, alph = O.encode_alpha(img, w, h, color)
    assert rc == 0
    want = _riff(_vp8x(w, h, 0x10), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8))
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    got = bytes(enc.encode(img, w, h, color))
    assert got == want
    # with metadata: VP8X flags ICC|alpha|EXIF|XMP, ICCP before ALPH, EXIF/XMP after VP8
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    enc.set_icc_profile(b"icc!")
    enc.set_exif_metadata(b"exif-data")
    enc.set_xmp_metadata(b"<x/>")
    got = bytes(enc.encode(img, w, h, color))
    assert got == _riff(_vp8x(w, h, 0x3C), _chunk(b"ICCP", b"icc!"), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8),
                        _chunk(b"EXIF", b"exif-data"), _chunk(b"XMP ", b"<x/>"))
    if _W is not None:
        ww, hh = ctypes.c_int(), ctypes.c_int()
        p = _W.WebPDecodeRGBA(got, len(got), ctypes.byref(ww), ctypes.byref(hh))
        assert p and (ww.value, hh.value) == (w, h)
        dec = np.ctypeslib.as_array((ctypes.c_uint8 * (w * h * 4)).from_address(p)).copy().reshape(h, w, 4)
        _W.WebPFree(p)
        assert np.array_equal(dec[..., 3], img[..., -1])


def _tied_alpha_img(w=640, h=256):
    """Alpha whose length-limited Huffman trees split tie groups (the order of
    the reference's sort_unstable_by_key decides which equal-frequency symbols
    get the longer codes, api.rs:259-260; the same distribution as
    test_lossless's tied640x256)."""
    rng = np.random.default_rng(7)
    parts = [np.full(int(1.6 ** k), 100 + k, np.uint8) for k in range(22)]
    parts += [np.full(c, s, np.uint8) for s, c in zip(range(0, 90), [1, 2, 3] * 30)]
    g = np.resize(np.concatenate(parts), w * h)
    rng.shuffle(g)
    img = synth_rgba(w, h, 0x5EED0077)
    img[..., 3] = g.reshape(h, w)
    return np.ascontiguousarray(img)


# SHA-256 of the oracle's ALPH payload for _tied_alpha_img() (drift guard; the
# oracle at c7fefce, parity with the reference's VP8L bytes unpinned: no fixture)
TIED_ALPH_SHA256 = "08401df9d5aa9a5b05e160fd3a4b0b8ff95c994185148dda6f22914325e6e24d"


def test_webp_container_tied_alpha(ctx):
    """WebPEncoder::encode (lossy, RGBA) on the tie-split alpha: the whole RIFF
    (VP8X + ALPH + VP8) equals the oracle's, and the ALPH payload its pinned digest."""
    import hashlib
    w, h = 640, 256
    img = _tied_alpha_img(w, h)
    rc, vp8, _ = O.encode(img, w, h, 3, 75, 4)
    assert rc == 0
    rc, alph = O.encode_alpha(img, w, h, 3)
    assert rc == 0 and hashlib.sha256(bytes(alph)).hexdigest() == TIED_ALPH_SHA256
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    got = bytes(enc.encode(img, w, h, zwebp.ColorType.Rgba8))
    assert got == _riff(_vp8x(w, h, 0x10), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8))


def test_encode_webp_rgba_entry(ctx):
    """zw_encode_webp (EncoderParams::lossy) for RGBA8 equals the _ex form."""
    w, h = 200, 120
    img = _alpha_img(w, h, zwebp.ColorType.Rgba8)
    L = zwebp.load_library()
    a = np.ascontiguousarray(img).reshape(-1)
    out = zwebp._Bytes()
    rc = L.zw_encode_webp(ctx.handle, a.ctypes.data, a.size, w, h, 3, 75, 4, ctypes.byref(out))
    assert rc == 0
    got = zwebp._take_bytes(L, out)
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    assert got == bytes(enc.encode(img, w, h, zwebp.ColorType.Rgba8))


@pytest.mark.parametrize("color", [zwebp.ColorType.Rgba8, zwebp.ColorType.La8, zwebp.ColorType.Rgb8,
                                   zwebp.ColorType.L8])
def test_encode_webp_batch(ctx, color):
    """zw_encode_webp_batch / the pipe's container mode: per frame the same
    container as WebPEncoder::encode (VP8X + ALPH for alpha inputs, built from
    the oracle's VP8 and ALPH payloads; simple RIFF otherwise)."""
    w, h = 240, 144
    imgs = []
    for i in range(5):
        im = _alpha_img(w, h, zwebp.ColorType.Rgba8) if i % 2 else synth_rgba(w, h, 0x5EED3000 + i, "noise")
        im = np.ascontiguousarray(im)
        if color == zwebp.ColorType.La8:
            im = np.ascontiguousarray(im[..., [0, 3]])
        elif color == zwebp.ColorType.Rgb8:
            im = np.ascontiguousarray(im[..., :3])
        elif color == zwebp.ColorType.L8:
            im = np.ascontiguousarray(im[..., 0])
        imgs.append(im)
    outs = zwebp.encode_webp_batch(imgs, w, h, color, 75, 4, ctx=ctx)
    for i, im in enumerate(imgs):
        rc, vp8, _ = O.encode(im, w, h, color, 75, 4)
        assert rc == 0
        if color in (zwebp.ColorType.Rgba8, zwebp.ColorType.La8):
            rc, alph = O.encode_alpha(im, w, h, color)
            assert rc == 0
            want = _riff(_vp8x(w, h, 0x10), _chunk(b"ALPH", alph), _chunk(b"VP8 ", vp8))
        else:
            want = _riff(_chunk(b"VP8 ", vp8))
        assert outs[i] == want, f"frame {i}"


@pytest.mark.parametrize("nb,lanes,chunk,up,pack,w,h", [(1, "1", "4", "1", "1", 96, 64), (3, "2", "2", "3", "0", 96, 64),
                                                         (4, "1", "3", "2", "1", 96, 64), (5, "2", "4", "1", "1", 96, 64),
                                                         (3, "1", "4", "2", "1", 101, 37)])
def test_pipe_encode_host(ctx, monkeypatch, nb, lanes, chunk, up, pack, w, h):
    """zw_pipe_encode_host: nb batches streamed from host memory (batch b+1
    uploaded into the other input buffer while batch b encodes; lanes and chunks
    forced small so the uploads wait on rgb2yuv of batch b-2 per chunk).  Every
    batch holds different frames; the last batch's bitstreams equal the oracle's.
    pack = 1 (the default): the RGBA frames cross as RGB (alpha dropped on the
    host, rgb2yuv reading 3 bytes a pixel; the 101-wide frames take its
    per-sample path); pack = 0: as RGBA."""
    monkeypatch.setenv("ZW_PIPE_LANES", lanes)
    monkeypatch.setenv("ZW_PIPE_CHUNK", chunk)
    monkeypatch.setenv("ZW_ENC_ROWS", "0")
    monkeypatch.setenv("ZW_UPLOAD_THREADS", up)
    monkeypatch.setenv("ZW_UPLOAD_PACK", pack)
    n = 16  # (two lanes need >= 8 frames each)
    batches = [[synth_rgba(w, h, 0x5EED6000 + 16 * b + i, ("natural", "noise")[(b + i) % 2]) for i in range(n)]
               for b in range(nb)]
    for b in range(nb):  # a varying alpha plane: the VP8 payload does not depend on it
        for i in range(n):
            batches[b][i].reshape(-1, 4)[:, 3] = (np.arange(w * h) * (7 + b + i)) & 255
    p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    try:
        p.encode_host(batches)
        for i in range(n):
            rc, ref, _ = O.encode(batches[-1][i], w, h, 3, 75, 4)
            assert rc == 0 and p.output(i) == ref, f"frame {i} of the last batch"
        # again on the same pipe with another uploader count, batches reversed
        monkeypatch.setenv("ZW_UPLOAD_THREADS", "2" if up != "2" else "4")
        p.encode_host(batches[::-1])
        for i in (0, n - 1):
            rc, ref, _ = O.encode(batches[0][i], w, h, 3, 75, 4)
            assert p.output(i) == ref, f"frame {i}, second call"
        # the same pipe afterwards from device-resident input (the first buffer)
        for i in range(n):
            p.upload(i, batches[0][i])
        p.encode()
        rc, ref, _ = O.encode(batches[0][3], w, h, 3, 75, 4)
        assert p.output(3) == ref
    finally:
        p.close()


@pytest.mark.parametrize("color", [zwebp.ColorType.Rgba8, zwebp.ColorType.La8])
def test_encode_webp_batch_alpha_too_large(ctx, color):
    """An alpha input taller than 16384 rows: encode_alpha_lossless returns
    InvalidDimensions (encoder/api.rs:1187), so the batch container path
    fails with ZW_EINVALID_DIMENSIONS instead of writing an empty ALPH chunk;
    the same frame without alpha (RGB8) encodes."""
    w, h = 64, 16400
    bpp = 4 if color == zwebp.ColorType.Rgba8 else 2
    img = np.full(w * h * bpp, 200, np.uint8)
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_webp_batch([img], w, h, color, 75, 0, ctx=ctx)
    assert e.value.code == 1  # ZW_EINVALID_DIMENSIONS
    rgb = np.full(w * h * 3, 200, np.uint8)
    out = zwebp.encode_webp_batch([rgb], w, h, zwebp.ColorType.Rgb8, 75, 0, ctx=ctx)
    assert out[0][:4] == b"RIFF" and out[0][12:16] == b"VP8 "


def test_rows_encode_error_reported(ctx, monkeypatch):
    """Row-parallel encode: a set launch error word (a wave that gave up
    waiting) fails the encode with ZW_EDEVICE instead of returning streams."""
    w, h = 160, 96
    img = synth_rgba(w, h, 0x5EED0077)
    monkeypatch.setenv("ZW_ENC_ROWS", "1")
    monkeypatch.setenv("ZW_ENC_FORCE_ERROR", "1")
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_batch([img, img], w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    assert e.value.code == 4  # ZW_EDEVICE
    monkeypatch.delenv("ZW_ENC_FORCE_ERROR")
    out = zwebp.encode_batch([img, img], w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    rc, ref, _ = O.encode(img, w, h, 3, 75, 4)
    assert out[0] == ref and out[1] == ref


# --------------------------------------------------------------------------
# row-parallel decode: a wave that gives up waiting fails the call
# --------------------------------------------------------------------------
def test_rows_decode_error_reported(ctx, monkeypatch):
    w, h = 320, 240
    img = synth_rgba(w, h, 0x5EED0050)
    vp8 = zwebp.encode_frame_lossy(img, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    zwebp.vp8_decode_frame(vp8, ctx=ctx)  # fine without the hook
    monkeypatch.setenv("ZW_DEC_FORCE_ERROR", "1")
    monkeypatch.setenv("ZW_DEC_ROWS", "1")
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.vp8_decode_frame(vp8, ctx=ctx)
    assert e.value.code == 4
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    y = np.zeros(mbw * mbh * 256, np.uint8)
    u = np.zeros(mbw * mbh * 64, np.uint8)
    v = np.zeros(mbw * mbh * 64, np.uint8)
    with pytest.raises(zwebp.ZwError) as e:
        zwebp.loop_filter_frame(y, u, v, mbw, mbh, np.zeros((mbw * mbh, 4), np.uint8), 0, 6, 0, ctx=ctx)
    assert e.value.code == 4
    monkeypatch.delenv("ZW_DEC_FORCE_ERROR")
    zwebp.vp8_decode_frame(vp8, ctx=ctx)


# --------------------------------------------------------------------------
# decoder/api.rs:1166-1212: the reference's single-colour imagemagick files
# --------------------------------------------------------------------------
@pytest.mark.parametrize("n", [2, 3])
def test_single_colour_files_decode(ctx, n):
    """WebPDecoder::read_image on the 2x2 / 3x3 red files: every pixel equal
    (the odd tail included) and equal to the oracle's decode."""
    from test_oracle import imagemagick_red
    f = imagemagick_red(n)
    dec = zwebp.WebPDecoder(f, ctx=ctx)
    assert dec.dimensions() == (n, n)
    rgb = dec.read_image().reshape(-1, 3)
    assert (rgb == rgb[0]).all()
    vp8 = f[20:20 + int.from_bytes(f[16:20], "little")]
    rc, r = O.decode(vp8)
    assert rc == 0
    ys, cs = r["mbw"] * 16, r["mbw"] * 8
    c = (n + 1) // 2
    ref = O.yuv_to_rgb_fancy(r["y"].reshape(-1, ys)[:n, :n].reshape(-1), r["u"].reshape(-1, cs)[:c, :c].reshape(-1),
                             r["v"].reshape(-1, cs)[:c, :c].reshape(-1), n, n).reshape(-1, 3)
    assert np.array_equal(rgb, ref)


def _hip():
    import ctypes
    import ctypes.util
    name = ctypes.util.find_library("amdhip64") or "libamdhip64.so"
    h = ctypes.CDLL(name)
    h.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    h.hipHostFree.argtypes = [ctypes.c_void_p]
    h.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    h.hipHostUnregister.argtypes = [ctypes.c_void_p]
    return h


@pytest.mark.parametrize("kind,pack", [("hostmalloc", "0"), ("registered", "0"), ("hostmalloc", "1")])
def test_pipe_encode_host_pinned(ctx, monkeypatch, kind, pack):
    """zw_pipe_encode_host from page-locked frames: with ZW_UPLOAD_PACK=0 they
    go to the DMA engines without the staging copy -- hipHostMalloc memory (what
    torch pin_memory gives) and pageable memory registered with hipHostRegister
    (the engines read it through the allocation's device pointer); packed (the
    default) they are staged as RGB like pageable frames.  Bitstreams equal the
    oracle's; every frame sits at an offset inside one allocation."""
    import ctypes
    monkeypatch.setenv("ZW_UPLOAD_PACK", pack)
    monkeypatch.setenv("ZW_PIPE_LANES", "1")
    monkeypatch.setenv("ZW_ENC_ROWS", "0")
    w, h, n, nb = 96, 64, 8, 2
    fb = w * h * 4
    hip = _hip()
    total = nb * n * fb + 4096
    if kind == "hostmalloc":
        ptr = ctypes.c_void_p()
        assert hip.hipHostMalloc(ctypes.byref(ptr), total, 0) == 0
        base = ptr.value
        keep = None
    else:
        keep = np.zeros(total, np.uint8)
        base = keep.ctypes.data
        assert hip.hipHostRegister(ctypes.c_void_p(base), total, 0) == 0
    try:
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(base))
        batches = []
        for b in range(nb):
            fr = []
            for i in range(n):
                off = 1024 + (b * n + i) * fb  # (not at the allocation's start)
                a = buf[off:off + fb]
                a[:] = synth_rgba(w, h, 0x5EED7000 + 16 * b + i, "natural").reshape(-1)
                fr.append(a)
            batches.append(fr)
        p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
        try:
            p.encode_host(batches)
            for i in range(n):
                rc, ref, _ = O.encode(np.array(batches[-1][i]).reshape(h, w, 4), w, h, 3, 75, 4)
                assert rc == 0 and p.output(i) == ref, f"frame {i}"
        finally:
            p.close()
    finally:
        if kind == "hostmalloc":
            hip.hipHostFree(ctypes.c_void_p(base))
        else:
            hip.hipHostUnregister(ctypes.c_void_p(base))


@pytest.mark.parametrize("tokens", ["auto", "device"])
def test_decode_batch_mixed_sizes(ctx, monkeypatch, tokens):
    """Frames of several sizes in one batch decode as runs of one size, each
    equal to the oracle's decode_frame (decoder/vp8.rs:1526), as a sequence of
    decode_frame calls would; RGBA batches (fresh and caller buffers) likewise.
    A damaged frame mid-batch fails the call with the oracle's variant.
    tokens=device: every run's token partitions parsed by k_dec_tokl."""
    if tokens != "auto":
        monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    sizes = [(64, 48), (64, 48), (96, 80), (33, 17), (33, 17), (33, 17), (64, 48)]
    streams = []
    for k, (w, h) in enumerate(sizes):
        rc, s, _ = O.encode(synth_rgba(w, h, 0x5EED7800 + k, "natural"), w, h, 3, 60 + k, 4)
        assert rc == 0
        streams.append(s)
    frames = zwebp.decode_batch(streams, ctx=ctx)
    for s, fr in zip(streams, frames):
        rc, r = O.decode(s)
        assert rc == 0
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])
    imgs = zwebp.decode_rgb_batch(streams, 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    stride = 4 * max(w for w, _ in sizes)  # (one row stride for every caller buffer)
    bufs = [np.zeros(stride * h, np.uint8) for (w, h) in sizes]
    zwebp.decode_rgb_batch_into(streams, bufs, 4, zwebp.UpsamplingMethod.Bilinear, stride_bytes=stride, ctx=ctx)
    for (w, h), s, im, b in zip(sizes, streams, imgs, bufs):
        rc, r = O.decode(s)
        want = np.asarray(O.yuv_to_rgb_fancy(r["y"], r["u"], r["v"], w, h, 4)).reshape(h, w * 4)
        assert bytes(im) == want.tobytes()
        assert np.array_equal(b.reshape(h, stride)[:, :w * 4], want)
    bad = list(streams)
    bad[3] = bad[3][:40]
    rc, _ = O.decode(bad[3])
    assert rc != 0
    with pytest.raises(zwebp.DecodingError) as e:
        zwebp.decode_batch(bad, ctx=ctx)
    assert e.value.code == rc


_SEAM_CHILD = r"""
import os, sys, threading
sys.path[:0] = [os.path.join(sys.argv[1], "image-webp_amd"), os.path.join(sys.argv[1], "tests")]
import numpy as np
import zwebp
import oracle_lib as O
from zwebp.synth import synth_rgba
shapes = [(96, 64, 75, 4, 1), (96, 64, 40, 2, 1), (48, 80, 75, 4, 2)]
imgs = {s: [synth_rgba(s[0], s[1], 0x5EA0 + 7 * i + s[2]) for i in range(4)] for s in shapes}
want = {}
for s in shapes:
    for i, im in enumerate(imgs[s]):
        rc, b, _ = O.encode(im, s[0], s[1], 3, s[2], s[3], nparts=s[4])
        assert rc == 0
        want[(s, i)] = b
zwebp.dbg_seam_stats(reset=True)
T, calls = 24, 6
bad, errs = [], []
def work(t):
    c = zwebp.Context(0)
    try:
        for k in range(calls):
            s = shapes[(t + k) % len(shapes)]
            i = (t * 5 + k) % 4
            got = zwebp.encode_frame_lossy(imgs[s][i], s[0], s[1], zwebp.ColorType.Rgba8, s[2], s[3], ctx=c,
                                           token_partitions=s[4])
            if bytes(got) != want[(s, i)]:
                bad.append((t, k, s, i))
    except Exception as e:
        errs.append(repr(e))
    finally:
        c.close()
th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
for x in th:
    x.start()
for x in th:
    x.join(timeout=240)
st = zwebp.dbg_seam_stats()
print("seam", st, "bad", bad[:4], "errs", errs[:4], flush=True)
assert not errs and not bad, (errs, bad[:4])
assert st[1] == T * calls and st[2] >= 2, st  # every call went through the seam, some in shared batches
# an invalid call fails on its own without joining (or stalling) a batch
c = zwebp.Context(0)
try:
    zwebp.encode_frame_lossy(imgs[shapes[0]][0].reshape(-1)[:100], 96, 64, zwebp.ColorType.Rgba8, 75, 4, ctx=c)
    raise SystemExit("an invalid call succeeded")
except zwebp.ZwError:
    pass
c.close()
print("ok", flush=True)
"""


@pytest.mark.gpu
def test_seam_batches_concurrent_calls():
    """The seam itself (zw_host.cpp seam_encode): in a fresh process with
    ZW_SEAM_SOLO=0 (read once, at the first call) every encode_frame_lossy call
    joins the seam; 24 threads with contexts of their own over three shapes
    (sizes, quality, method, partitions) form shared batches of mixed callers
    (the counters show frames per batch > 1), each caller gets exactly the
    oracle's bitstream for its own frame, and an invalid call fails alone."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ZW_SEAM_SOLO="0")
    r = subprocess.run([sys.executable, "-c", _SEAM_CHILD, root], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


@pytest.mark.gpu
def test_seam_concurrent_single_frame_calls(ctx):
    """encode_frame_lossy from 12 threads, each with a context of its own, over
    three shapes (sizes, quality, method, partitions): below ZW_SEAM_SOLO calls
    in flight each encodes on its own (the solo path), and every call returns
    exactly the oracle's bitstream for its own frame."""
    import threading
    shapes = [(96, 64, 75, 4, 1), (96, 64, 40, 2, 1), (48, 80, 75, 4, 2)]
    imgs = {s: [synth_rgba(s[0], s[1], 0x5EA0 + 7 * i + s[2]) for i in range(4)] for s in shapes}
    want = {}
    for s in shapes:
        for i, im in enumerate(imgs[s]):
            rc, b, _ = O.encode(im, s[0], s[1], 3, s[2], s[3], nparts=s[4])
            assert rc == 0
            want[(s, i)] = b
    T, calls = 12, 6
    bad, errs = [], []

    def work(t):
        c = zwebp.Context(0)
        try:
            for k in range(calls):
                s = shapes[(t + k) % len(shapes)]
                i = (t * 5 + k) % 4
                got = zwebp.encode_frame_lossy(imgs[s][i], s[0], s[1], zwebp.ColorType.Rgba8, s[2], s[3], ctx=c,
                                               token_partitions=s[4])
                if bytes(got) != want[(s, i)]:
                    bad.append((t, k, s, i))
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(repr(e))
        finally:
            c.close()

    th = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    assert not errs and not bad, (errs, bad[:4])
    # an invalid call fails on its own without joining (or stalling) a batch
    with pytest.raises(zwebp.ZwError):
        zwebp.encode_frame_lossy(imgs[shapes[0]][0].reshape(-1)[:100], 96, 64, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)


_EMIT_CHILD = r"""
import os, sys
sys.path[:0] = [os.path.join(sys.argv[1], "image-webp_amd"), os.path.join(sys.argv[1], "tests")]
import oracle_lib as O
import zwebp
from zwebp.shard import frame_seed
from zwebp.synth import synth_rgba
n, w, h, distinct = 256, 64, 48, 8
imgs = [synth_rgba(w, h, frame_seed(i)) for i in range(distinct)]
refs = []
for im in imgs:
    rc, ref, _ = O.encode(im, w, h, 3, 75, 4)
    assert rc == 0
    refs.append(ref)
ctx = zwebp.Context(0)
p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
for i in range(n):
    p.upload(i, imgs[i % distinct])
p.encode_repeat(2)
bad = [i for i in range(n) if p.output(i) != refs[i % distinct]]
assert not bad, (len(bad), bad[:4])
assert p.kernel_times()[8] > 0  # the emission workers' CPU time
p.close()
ctx.close()
print("ok")
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"ZW_CODE16": "0"}, {"ZW_EMIT_GROUP": "7"}, {"ZW_EMIT_GROUP": "16"}],
                         ids=["four_interleaved", "vector_7_lanes", "vector_16_lanes"])
def test_emission_groups_bitexact(env):
    """Host emission (zw_host.cpp chunk_emit -> zwh::emit_frames): a 256-frame
    chunk in groups of 16 frames whose coders run as the lanes of the AVX-512
    coder, in groups of 7 (9 lanes masked, and a last group of 4 on the
    interleaved coder), and with the vector coder off (four frames interleaved):
    every bitstream equals the oracle's.  A fresh process per case (the knobs
    are read once)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _EMIT_CHILD, root], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
