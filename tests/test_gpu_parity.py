"""GPU parity: the HIP product path (through the C ABI) against the CPU oracle.

Every comparison is bit-exact.  Encoder checks go stage by stage (YUV planes,
analysis alphas, pass-2 modes, quantised levels, reconstruction, bitstream) so a
failure names the first stage and macroblock that diverged.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import zwebp
from zwebp.synth import synth_rgba

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    return zwebp.Context(0)


def _img(w, h, kind, seed, color):
    rgba = synth_rgba(w, h, seed, kind)
    if color == zwebp.ColorType.Rgba8:
        return rgba
    if color == zwebp.ColorType.Rgb8:
        return np.ascontiguousarray(rgba[..., :3])
    if color == zwebp.ColorType.La8:
        return np.ascontiguousarray(rgba[..., [0, 3]])
    return np.ascontiguousarray(rgba[..., 0])


# --------------------------------------------------------------------------
# a1: RGB -> YUV 4:2:0
# --------------------------------------------------------------------------
@pytest.mark.parametrize("w,h", [(1, 1), (17, 9), (64, 48), (333, 211), (250, 31), (120, 67), (200, 75), (1920, 1080)])
@pytest.mark.parametrize("bpp", [1, 2, 3, 4])
def test_rgb_to_yuv420(ctx, w, h, bpp):
    # widths that are multiples of 8 run the row-coalesced kernel for RGB / RGBA
    # (8-pixel runs; the run at a partial-MB right edge and the padding rows
    # take the per-sample path)
    img = np.ascontiguousarray(synth_rgba(w, h, 7 + w, "noise")[..., :bpp])
    gy, gu, gv = zwebp.rgb_to_yuv420(img, w, h, bpp, ctx=ctx)
    oy, ou, ov = O.rgb_to_yuv420(img, w, h, bpp)
    assert np.array_equal(gy, oy)
    assert np.array_equal(gu, ou)
    assert np.array_equal(gv, ov)


@pytest.mark.parametrize("bpp", [3, 4])
def test_rgb_to_yuv420_exhaustive_luma(ctx, bpp):
    """rgb_to_y (yuv.rs:859-873) for every (r, g, b) exactly once: a 4096 x 4096 image
    whose pixel i is (i & 255, (i >> 8) & 255, i >> 16), through the row-coalesced
    kernel's 16-bit dot-product form; the chroma planes (2x2 sums of neighbouring
    triples) are checked as well."""
    w = h = 4096
    i = np.arange(w * h, dtype=np.uint32)
    img = np.empty((h, w, bpp), np.uint8)
    img[..., 0] = (i & 255).reshape(h, w)
    img[..., 1] = ((i >> 8) & 255).reshape(h, w)
    img[..., 2] = (i >> 16).reshape(h, w)
    if bpp == 4:
        img[..., 3] = 255
    gy, gu, gv = zwebp.rgb_to_yuv420(img, w, h, bpp, ctx=ctx)
    oy, ou, ov = O.rgb_to_yuv420(img, w, h, bpp)
    assert np.array_equal(gy, oy)
    assert np.array_equal(gu, ou)
    assert np.array_equal(gv, ov)


# --------------------------------------------------------------------------
# a2..a18: the full encoder, stage by stage
# --------------------------------------------------------------------------
ENC_CASES = [
    (64, 48, "natural", 75, 4, 3),
    (300, 257, "natural", 75, 4, 3),
    (768, 512, "natural", 75, 4, 3),
    (333, 211, "noise", 75, 4, 2),
    (256, 256, "flat", 75, 4, 3),
    (200, 120, "natural", 20, 4, 3),
    (96, 80, "natural", 95, 4, 3),
    (160, 128, "natural", 75, 0, 3),
    (160, 128, "natural", 75, 2, 3),
    (160, 128, "natural", 75, 3, 3),
    (160, 128, "natural", 75, 5, 3),
    (160, 128, "natural", 75, 6, 3),
    (123, 77, "natural", 0, 4, 0),
    (123, 77, "natural", 100, 4, 1),
    (1, 1, "natural", 75, 4, 3),
    (4000, 16, "natural", 75, 4, 3),
    (16, 1100, "natural", 60, 4, 3),
]


def _mb_rows(a, per):
    return a.reshape(-1, per)


def _plane_mb_diff(a, b, stride, mb):
    """MB indices whose (mb x mb) tile differs."""
    A = a.reshape(-1, stride)
    B = b.reshape(-1, stride)
    d = (A != B).reshape(A.shape[0] // mb, mb, stride // mb, mb).any(axis=(1, 3))
    return np.nonzero(d.reshape(-1))[0]


def _modes_of(info, nmb):
    m = np.array([[info[i].luma_mode, info[i].chroma_mode, info[i].skip, info[i].segment] + list(info[i].bpred)
                  for i in range(nmb)], np.uint8)
    m[m[:, 0] != 4, 4:] = 0
    return m


def _check_encode(ctx, w, h, kind, q, m, color, seed):
    """Stage-by-stage comparison; collects every stage's first divergence."""
    img = _img(w, h, kind, seed, color)
    rc, ref, dbg = O.encode(img, w, h, color, q, m, debug=True)
    assert rc == 0
    p = zwebp.Pipeline(1, w, h, color, q, m, ctx=ctx)
    rep = []
    try:
        p.upload(0, img)
        nmb = p.mbw * p.mbh
        ys, cs = p.mbw * 16, p.mbw * 8
        # pass 1 alone (with its reconstruction)
        p.run_pass1(True)
        y, u, v = p.planes(0, 0)
        for a, b, n in ((y, dbg["src_y"], "Y"), (u, dbg["src_u"], "U"), (v, dbg["src_v"], "V")):
            if not np.array_equal(a, b):
                rep.append(f"source plane {n} differs")
        if dbg["segments_enabled"]:
            al = p.alpha(0)
            d = np.nonzero(al != dbg["mb_alpha"])[0]
            if d.size:
                rep.append(f"alpha: {d.size} MBs differ, first {d[0]}: {al[d[0]]} vs {dbg['mb_alpha'][d[0]]}")
        m1, _ = p.mbinfo(0, 1)
        g1 = m1.copy()
        g1[g1[:, 0] != 4, 4:] = 0
        o1 = _modes_of(dbg["p1_info"], nmb)
        d = np.nonzero((g1[:, [0, 1]] != o1[:, [0, 1]]).any(axis=1) | (g1[:, 4:] != o1[:, 4:]).any(axis=1))[0]
        if d.size:
            i = int(d[0])
            rep.append(f"pass-1 modes: {d.size} MBs differ, first MB {i} (x={i % p.mbw},y={i // p.mbw}): "
                       f"{g1[i].tolist()} vs {o1[i].tolist()}")
        r1y, _, _ = p.planes(0, 1)
        d = _plane_mb_diff(r1y, dbg["recon1_y"], ys, 16)
        if d.size:
            rep.append(f"pass-1 recon Y: {d.size} MBs differ, first MB {d[0]}")
        # full encode
        p.enable_debug()
        p.encode()
        gp, gsp = p.probs(0)
        if not np.array_equal(gp, dbg["final_probs"]):
            rep.append(f"pass-2 probabilities differ in {int((gp != dbg['final_probs']).sum())} entries")
        if gsp != dbg["skip_prob"]:
            rep.append(f"skip prob {gsp} vs {dbg['skip_prob']}")
        modes, levels = p.mbinfo(0, 2)
        gm = modes.copy()
        gm[gm[:, 0] != 4, 4:] = 0
        om = _modes_of(dbg["p2_info"], nmb)
        d = np.nonzero((gm != om).any(axis=1))[0]
        if d.size:
            i = int(d[0])
            rep.append(f"pass-2 modes: {d.size} MBs differ, first MB {i} (x={i % p.mbw},y={i // p.mbw}): "
                       f"{gm[i].tolist()} vs {om[i].tolist()}")
        ol = dbg["levels"].reshape(nmb, 25, 16)
        gl = levels.astype(np.int32)
        gl[gm[:, 2] == 1] = 0
        gl[gm[:, 0] == 4, 16] = 0
        d = np.nonzero((gl != ol).reshape(nmb, -1).any(axis=1))[0]
        if d.size:
            i = int(d[0])
            blk = int(np.nonzero((gl[i] != ol[i]).any(axis=1))[0][0])
            rep.append(f"levels: {d.size} MBs differ, first MB {i} block {blk} (mode {gm[i, 0]}): "
                       f"{gl[i, blk].tolist()} vs {ol[i, blk].tolist()}")
            if gm[i, 0] == 4:
                gd = p.i4_dump(0)[i, blk]
                od = dbg["i4_dump"].reshape(nmb, 16, 34)[i, blk]
                rep.append(f"  I4 dump gpu coeffs {gd[:16].tolist()} pred {gd[16:32].tolist()} ctx0 {gd[32]} mode {gd[33]}")
                rep.append(f"  I4 dump orc coeffs {od[:16].tolist()} pred {od[16:32].tolist()} ctx0 {od[32]} mode {od[33]}")
        ry, ru, rv = p.planes(0, 1)
        for a, b, s, mb, n in ((ry, dbg["recon_y"], ys, 16, "Y"), (ru, dbg["recon_u"], cs, 8, "U"),
                               (rv, dbg["recon_v"], cs, 8, "V")):
            d = _plane_mb_diff(a, b, s, mb)
            if d.size:
                A, B = a.reshape(-1, s), b.reshape(-1, s)
                r0, c0 = (d[0] // (s // mb)) * mb, (d[0] % (s // mb)) * mb
                ta, tb = A[r0:r0 + mb, c0:c0 + mb], B[r0:r0 + mb, c0:c0 + mb]
                pos = np.argwhere(ta != tb)
                rep.append(f"recon {n}: {d.size} MBs differ, first MB {d[0]}, {len(pos)} px, first at {pos[0].tolist()}"
                           f" gpu {int(ta[tuple(pos[0])])} oracle {int(tb[tuple(pos[0])])}")
        out = p.output(0)
        if out != ref:
            rep.append(f"bitstream differs (len {len(out)} vs {len(ref)})")
    finally:
        p.close()
    assert not rep, "\n".join(rep)
    return ref


# rows "1": the row-parallel kernels (one wave per MB row, global-memory row
# hand-off; the default for single frames), "0": one 12-wave workgroup per frame
# (the batch kernels)
@pytest.mark.parametrize("rows", ["1", "0"])
@pytest.mark.parametrize("w,h,kind,q,m,color", ENC_CASES)
def test_encode_matches_oracle(ctx, monkeypatch, w, h, kind, q, m, color, rows):
    monkeypatch.setenv("ZW_ENC_ROWS", rows)
    _check_encode(ctx, w, h, kind, q, m, color, 0x5EED0000 + w * 7 + h)


def test_encode_batch_independent_frames(ctx):
    w, h = 176, 144
    imgs = [synth_rgba(w, h, 0x5EED0000 + i, "natural" if i % 3 else "noise") for i in range(5)]
    outs = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    for i, img in enumerate(imgs):
        rc, ref, _ = O.encode(img, w, h, 3, 75, 4)
        assert outs[i] == ref, f"frame {i}"


@pytest.mark.parametrize("chunk", ["2", "3"])
def test_encode_rows_multi_frame(ctx, monkeypatch, chunk):
    """Row-parallel kernels over several frames per launch (grid y = frame) and
    ragged chunks; the per-frame tickets / progress are reset per launch."""
    monkeypatch.setenv("ZW_ENC_ROWS", "1")
    monkeypatch.setenv("ZW_PIPE_CHUNK", chunk)
    w, h = 208, 144
    imgs = [synth_rgba(w, h, 0x5EED2000 + i, ("natural", "noise", "flat")[i % 3]) for i in range(5)]
    p = zwebp.Pipeline(5, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    try:
        for i, img in enumerate(imgs):
            p.upload(i, img)
        p.encode_repeat(2)
        for i, img in enumerate(imgs):
            rc, ref, _ = O.encode(img, w, h, 3, 75, 4)
            assert p.output(i) == ref, f"frame {i}"
    finally:
        p.close()


@pytest.mark.parametrize("chunk,n", [("2", 5), ("3", 7), ("4", 4)])
def test_encode_frame_pairs(ctx, monkeypatch, chunk, n):
    """Pass 2 in frame pairs (k_encode_pass2_fp: two frames per workgroup, the
    two MBs' I4 searches in one wave), forced on at small sizes: pass 2 of
    chunks (2k, 2k + 1) in one launch, odd frame counts (a workgroup with one
    frame), ragged last chunks, per-frame segments and content; several batches
    (encode_repeat).  Every frame must equal the reference's stream."""
    monkeypatch.setenv("ZW_ENC_FP", "1")
    monkeypatch.setenv("ZW_ENC_ROWS", "0")
    monkeypatch.setenv("ZW_PIPE_CHUNK", chunk)
    w, h = 208, 144
    imgs = [synth_rgba(w, h, 0x5EED3000 + i, ("natural", "noise", "flat")[i % 3]) for i in range(n)]
    p = zwebp.Pipeline(n, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    try:
        for i, img in enumerate(imgs):
            p.upload(i, img)
        p.encode_repeat(2)
        for i, img in enumerate(imgs):
            rc, ref, _ = O.encode(img, w, h, 3, 75, 4)
            assert p.output(i) == ref, f"frame {i}"
    finally:
        p.close()


@pytest.mark.parametrize("m,q", [(2, 40), (3, 90), (5, 75), (6, 30)])
def test_encode_frame_pairs_methods(ctx, monkeypatch, m, q):
    """Frame-pair pass 2 at other methods: K = 3 candidates (methods 2-3), the
    ten-candidate search (methods 5-6, each frame's own search) and trellis."""
    monkeypatch.setenv("ZW_ENC_FP", "1")
    monkeypatch.setenv("ZW_ENC_ROWS", "0")
    w, h = 144, 96
    imgs = [synth_rgba(w, h, 0x5EED4000 + i, ("natural", "noise")[i % 2]) for i in range(3)]
    outs = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, q, m, ctx=ctx)
    for i, img in enumerate(imgs):
        rc, ref, _ = O.encode(img, w, h, 3, q, m)
        assert outs[i] == ref, f"frame {i}"


def test_encode_repeat_streaming(ctx, monkeypatch):
    """encode_repeat: batch k+1's pass 1 overlaps batch k's emission (separate
    pass-1 / pass-2 pack buffers); several chunks per lane; every batch's
    output must equal the reference's."""
    monkeypatch.setenv("ZW_PIPE_CHUNK", "2")
    w, h = 160, 128
    imgs = [synth_rgba(w, h, 0x5EED1000 + i, "natural" if i % 2 else "noise") for i in range(5)]
    p = zwebp.Pipeline(5, w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    try:
        for i, img in enumerate(imgs):
            p.upload(i, img)
        p.encode_repeat(3)
        for i, img in enumerate(imgs):
            rc, ref, _ = O.encode(img, w, h, 3, 75, 4)
            assert p.output(i) == ref, f"frame {i}"
    finally:
        p.close()


def test_encode_api_errors(ctx):
    img = synth_rgba(16, 16)
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossy(img, 0, 16, 3, ctx=ctx)
    assert e.value.code == 1
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossy(img[:8], 16, 16, 3, ctx=ctx)
    assert e.value.code == 2
    with pytest.raises(zwebp.EncodingError):
        zwebp.encode_frame_lossy(img, 16, 16, 3, quality=101, ctx=ctx)
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossy(img, 20000, 1, 3, ctx=ctx)
    assert e.value.code in (1, 2)


@pytest.mark.parametrize("w,h", [(16400, 16), (16, 20000), (25088, 8)])
def test_encode_beyond_14bit_dims(ctx, w, h):
    """encode_frame_lossy accepts any u16 dimension (vp8.rs:3143-3148) and the
    header keeps the low 14 bits (vp8.rs:326-327): the product's bytes equal the
    oracle's up to the widest frame whose LDS rows fit a CU (1568 MBs)."""
    img = np.ascontiguousarray(synth_rgba(w, h, 0x5EED2000 + w)[..., :3])
    rc, ref, _ = O.encode(img, w, h, 2, 75, 4)
    assert rc == 0
    out = zwebp.encode_frame_lossy(img, w, h, 2, 75, 4, ctx=ctx)
    assert out == ref
    assert int.from_bytes(out[6:8], "little") == w & 0x3FFF and int.from_bytes(out[8:10], "little") == h & 0x3FFF


@pytest.mark.parametrize("w,h", [(25089, 1), (25600, 16), (65535, 16), (40000, 33)])
def test_encode_wide_frames(ctx, w, h):
    """encode_frame_lossy takes any u16 width (vp8.rs:3143-3148).  Frames wider
    than the batch kernels' LDS holds (1 568 MBs) run the row-parallel kernels,
    whose LDS no longer grows with the width: the bitstream equals the oracle's
    (the header keeps the low 14 bits of the width, vp8.rs:326-327).  A width of
    65 536 is not a u16: InvalidDimensions, as the reference's try_into."""
    img = np.ascontiguousarray(synth_rgba(w, h, 0x5EED7700 + w, "natural")[..., :3])
    rc, ref, _ = O.encode(img, w, h, 2, 75, 4)
    assert rc == 0
    got = zwebp.encode_frame_lossy(img, w, h, 2, 75, 4, ctx=ctx)
    assert bytes(got) == bytes(ref)
    with pytest.raises(zwebp.EncodingError) as e:
        zwebp.encode_frame_lossy(np.zeros(65536 * 3, np.uint8), 65536, 1, 2, 75, 4, ctx=ctx)
    assert e.value.code == 1


def test_webp_container(ctx):
    w, h = 48, 32
    img = np.ascontiguousarray(synth_rgba(w, h)[..., :3])
    enc = zwebp.WebPEncoder(ctx=ctx)
    enc.set_params(zwebp.EncoderParams.lossy(75, 4))
    riff = bytes(enc.encode(img, w, h, zwebp.ColorType.Rgb8))
    assert O.riff_vp8_chunk(riff) == zwebp.encode_frame_lossy(img, w, h, 2, 75, 4, ctx=ctx)


# --------------------------------------------------------------------------
# a19..a21: decoder (recon + loop filter)
# --------------------------------------------------------------------------
def _manifest():
    with open(os.path.join(GOLD, "decode_golden.json")) as f:
        return json.load(f)["streams"]


@pytest.mark.parametrize("tokens", ["host", "device"])
@pytest.mark.parametrize("rows", ["default", "0"])
@pytest.mark.parametrize("entry", _manifest(), ids=lambda e: e["name"])
def test_decode_goldens(ctx, monkeypatch, entry, rows, tokens):
    """The committed streams' planes (SHA-256 from the reference's own decode
    fixtures / libwebp).  rows=0 forces the batch kernels (one workgroup per
    frame, reconstruction -> MB tiles -> loop filter), which otherwise only run
    for batches of 128+ frames: odd sizes and the gallery1 simple-filter
    streams (chroma moved through the tiles unfiltered) go through them too.
    tokens=device: the token partition parsed by k_dec_tokl (batches of 64+
    frames otherwise), the modes on the host."""
    if rows != "default":
        monkeypatch.setenv("ZW_DEC_ROWS", rows)
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    vp8 = open(os.path.join(GOLD, entry["name"] + ".vp8"), "rb").read()
    fr = zwebp.vp8_decode_frame(vp8, ctx=ctx)
    w, h = entry["width"], entry["height"]
    assert (fr.width, fr.height) == (w, h)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    planes = (fr.ybuf.reshape(-1, fr.y_stride)[:h, :w], fr.ubuf.reshape(-1, fr.uv_stride)[:ch, :cw],
              fr.vbuf.reshape(-1, fr.uv_stride)[:ch, :cw])
    got = [hashlib.sha256(np.ascontiguousarray(p).tobytes()).hexdigest() for p in planes]
    assert got == entry["yuv_sha256"]


@pytest.mark.parametrize("tokens", ["host", "device"])
@pytest.mark.parametrize("w,h,kind,q,m", [(333, 211, "natural", 75, 4), (256, 256, "noise", 40, 6),
                                          (96, 64, "flat", 75, 4), (512, 384, "natural", 90, 2),
                                          (64, 48, "noise", 1, 4), (48, 32, "noise", 100, 6)])
def test_decode_oracle_streams(ctx, monkeypatch, w, h, kind, q, m, tokens):
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    img = synth_rgba(w, h, 0x5EED0000 + h, kind)
    rc, vp8, _ = O.encode(img, w, h, 3, q, m)
    rc, r = O.decode(vp8)
    fr = zwebp.vp8_decode_frame(vp8, ctx=ctx)
    assert np.array_equal(fr.ybuf, r["y"])
    assert np.array_equal(fr.ubuf, r["u"])
    assert np.array_equal(fr.vbuf, r["v"])


def test_decode_batch(ctx):
    w, h = 128, 96
    streams = [O.encode(synth_rgba(w, h, 0x5EED0000 + i), w, h, 3, 30 + 10 * i, 4)[1] for i in range(4)]
    frames = zwebp.decode_batch(streams, ctx=ctx)
    for s, fr in zip(streams, frames):
        rc, r = O.decode(s)
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"])


def test_decode_batch_recycled_buffers(ctx):
    """Decoded frame buffers go back to the library's pool when freed
    (zw_frame_free) and the next batch of that size fills them: a batch decoded
    into recycled buffers equals the oracle, and frames still held are never
    handed out again (a later batch leaves them unchanged)."""
    import gc
    w, h = 112, 80
    kinds = ("natural", "noise", "flat")
    sets = [[O.encode(synth_rgba(w, h, 0x5EED7000 + 16 * k + i, kinds[(i + k) % 3]), w, h, 3, 20 + 25 * i, 4)[1]
             for i in range(3)] for k in range(3)]
    first = zwebp.decode_batch(sets[0], ctx=ctx)
    del first
    gc.collect()
    held = zwebp.decode_batch(sets[1], ctx=ctx)
    copies = [(bytes(f.ybuf), bytes(f.ubuf), bytes(f.vbuf)) for f in held]
    later = zwebp.decode_batch(sets[2], ctx=ctx)
    for streams, frames in ((sets[1], held), (sets[2], later)):
        for s, fr in zip(streams, frames):
            rc, r = O.decode(s)
            assert rc == 0
            assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])
    assert [(bytes(f.ybuf), bytes(f.ubuf), bytes(f.vbuf)) for f in held] == copies
    # RGBA buffers (zw_bytes) through the same pool, beside the encoder's
    # outputs (plain malloc) freed by the same zw_bytes_free
    rgb0 = zwebp.decode_rgb_batch(sets[0], 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    del rgb0
    gc.collect()
    enc = zwebp.encode_batch([synth_rgba(w, h, 0x5EED7100)], w, h, zwebp.ColorType.Rgba8, 75, 4, ctx=ctx)
    rgb1 = zwebp.decode_rgb_batch(sets[1], 4, zwebp.UpsamplingMethod.Bilinear, ctx=ctx)
    for s, b in zip(sets[1], rgb1):
        rc, r = O.decode(s)
        assert np.array_equal(b.reshape(-1), O.yuv_to_rgb_fancy(r["y"], r["u"], r["v"], w, h, 4))
    del enc
    # release_buffers empties the pool; frames still held stay valid, later batches decode as before
    del later, rgb1
    gc.collect()
    ctx.release_buffers()
    again = zwebp.decode_batch(sets[2], ctx=ctx)
    for s, fr in zip(sets[2], again):
        rc, r = O.decode(s)
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.vbuf, r["v"])
    assert [(bytes(f.ybuf), bytes(f.ubuf), bytes(f.vbuf)) for f in held] == copies


def test_decode_batch_device_tokens(ctx, monkeypatch):
    """A batch of 80 frames of mixed content and quality, split as large batches
    are (the first chunks parsed on the host, the rest's token partitions by
    k_dec_tokl, one frame per lane, beside them) equals the oracle frame by
    frame; with one frame's token partition cut short the batch fails with the
    oracle's DecodingError variant for that frame, whichever side parses it."""
    monkeypatch.setenv("ZW_DEC_TOKENS", "mixed")  # host chunks of 16 frames beside the device's 48 (+ 16)
    monkeypatch.setenv("ZW_DEC_TOKENS_HOST", "0.4")
    monkeypatch.setenv("ZW_DEC_CHUNK", "16")
    w, h = 96, 64
    kinds = ("natural", "noise", "flat")
    streams = [O.encode(synth_rgba(w, h, 0x5EED6000 + i, kinds[i % 3]), w, h, 3, 5 + (i * 7) % 95, i % 7)[1]
               for i in range(80)]
    frames = zwebp.decode_batch(streams, ctx=ctx)
    assert zwebp.decode_token_ms(ctx=ctx) > 0.0
    for s, fr in zip(streams, frames):
        rc, r = O.decode(s)
        assert rc == 0
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])
    bad = list(streams)
    bad[17] = streams[17][: len(streams[17]) - max(8, len(streams[17]) // 3)]
    rc, _ = O.decode(bad[17])
    assert rc != 0
    for tokens in ("host", "device", "mixed"):
        monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
        with pytest.raises(zwebp.DecodingError) as e:
            zwebp.decode_batch(bad, ctx=ctx)
        assert e.value.code == rc, (tokens, e.value.code, rc)
    monkeypatch.setenv("ZW_DEC_TOKENS", "mixed")
    frames = zwebp.decode_batch(streams, ctx=ctx)  # the context stays usable
    rc, r = O.decode(streams[5])
    assert np.array_equal(frames[5].ybuf, r["y"])


def test_decode_device_tokens_edge_streams(ctx, monkeypatch):
    """Device-token batches with the streams the kernel must not mishandle: frames
    with 2 / 4 / 8 token partitions (the whole batch then stays on the host
    parse), a flat frame whose MBs are all skipped (a near-empty token
    partition), and the lowest and highest quality settings; every frame equals
    the oracle's decode."""
    monkeypatch.setenv("ZW_DEC_TOKENS", "device")
    w, h = 80, 48
    flat = np.full((h, w, 3), 128, np.uint8)
    img = np.ascontiguousarray(synth_rgba(w, h, 0x5EED7000, "noise")[..., :3])
    cases = [[O.encode(img, w, h, 2, 75, 4, nparts=k)[1] for k in (2, 4, 8)],
             [O.encode(img, w, h, 2, 75, 4, nparts=k)[1] for k in (1, 4, 1)],
             [O.encode(flat, w, h, 2, q, 4)[1] for q in (0, 75, 100)],
             [O.encode(img, w, h, 2, q, m)[1] for q, m in ((0, 0), (100, 6), (1, 2), (99, 5))]]
    for streams in cases:
        frames = zwebp.decode_batch(streams, ctx=ctx)
        for s, fr in zip(streams, frames):
            rc, r = O.decode(s)
            assert rc == 0
            assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])


@pytest.mark.parametrize("tokens", ["host", "device"])
@pytest.mark.parametrize("chunk", ["1", "2", "4"])
def test_decode_batch_chunked(ctx, monkeypatch, chunk, tokens):
    """The double-buffered chunk pipeline (ZW_DEC_CHUNK frames per chunk; the
    host parses chunk c+1 while chunk c runs): several chunks, a ragged last
    chunk, both buffer sets reused, every frame equal to the oracle."""
    monkeypatch.setenv("ZW_DEC_CHUNK", chunk)
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    w, h = 160, 112
    streams = [O.encode(synth_rgba(w, h, 0x5EED4000 + i, ("natural", "noise", "flat")[i % 3]), w, h, 3,
                        20 + 15 * i, 4)[1] for i in range(5)]
    frames = zwebp.decode_batch(streams, ctx=ctx)
    assert len(frames) == len(streams)
    for s, fr in zip(streams, frames):
        rc, r = O.decode(s)
        assert rc == 0
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])


def test_decode_batch_chunked_size_change(ctx, monkeypatch):
    """A second frame size inside a chunked batch starts a new run of that size
    (its own chunks), and every frame equals the oracle."""
    monkeypatch.setenv("ZW_DEC_CHUNK", "2")
    a = O.encode(synth_rgba(64, 48, 1), 64, 48, 3, 75, 4)[1]
    b = O.encode(synth_rgba(96, 48, 2), 96, 48, 3, 75, 4)[1]
    fr = zwebp.decode_batch([a, a, b, a, a, a], ctx=ctx)
    for s, f in zip([a, a, b, a, a, a], fr):
        rc, r = O.decode(s)
        assert rc == 0 and np.array_equal(f.ybuf, r["y"]) and np.array_equal(f.vbuf, r["v"])


@pytest.mark.parametrize("tokens", ["host", "device"])
@pytest.mark.parametrize("rows", ["1", "0"])
def test_decode_rows_and_frame_kernels(ctx, monkeypatch, rows, tokens):
    """Both reconstruction / loop-filter kernel families on the same 1080p streams
    (ZW_DEC_ROWS=1: one wave per MB row spread over the CUs, rows handed over
    through global memory; 0: one workgroup per frame) equal the oracle, with
    the tokens parsed on the host or by k_dec_tokl."""
    monkeypatch.setenv("ZW_DEC_ROWS", rows)
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    w, h = 1920, 1080
    streams = [O.encode(synth_rgba(w, h, 0x5EED3000 + i, "natural" if i else "noise"), w, h, 3, q, 4)[1]
               for i, q in enumerate((20, 75, 95))]
    frames = zwebp.decode_batch(streams, ctx=ctx)
    for s, fr in zip(streams, frames):
        rc, r = O.decode(s)
        assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])


def _header_damage_cases(vp8):
    """Streams that fail in the frame tag / key-frame header / first partition
    (decoder/vp8.rs:553-680): every DecodingError variant the header can raise."""
    out = []
    b = bytearray(vp8); b[3] = 0; out.append(bytes(b))            # start code -> Vp8MagicInvalid
    b = bytearray(vp8); b[0] |= 1; out.append(bytes(b))           # inter frame -> UnsupportedFeature
    b = bytearray(vp8); b[0] &= 0x1F; b[1] = b[2] = 0; out.append(bytes(b))  # first partition size 0
    out += [vp8[:n] for n in range(0, 12)]                        # truncated tag / start code / dims
    b = bytearray(vp8); b[10] |= 0x80; out.append(bytes(b))       # color space bit
    out.append(vp8[:40])
    return out


@pytest.mark.parametrize("tokens", ["host", "device"])
def test_decode_errors(ctx, monkeypatch, tokens):
    """Each failing header gives the oracle's DecodingError variant (codes 10-17 =
    decoder/api.rs:79-110 in declaration order)."""
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    vp8 = open(os.path.join(GOLD, "libwebp_natural_64x48_q75.vp8"), "rb").read()
    seen = set()
    for s in _header_damage_cases(vp8):
        rc, _ = O.decode(s)
        if rc == 0:
            fr = zwebp.vp8_decode_frame(s, ctx=ctx)
            continue
        with pytest.raises(zwebp.DecodingError) as e:
            zwebp.vp8_decode_frame(s, ctx=ctx)
        assert e.value.code == rc, (len(s), e.value.code, rc)
        seen.add(rc)
    assert {10, 11, 15, 16, 17}.issubset(seen), seen


@pytest.mark.parametrize("m", [0, 1, 3, 6])
def test_encode_quality_method_sweep(ctx, m):
    """encode_frame_lossy (vp8.rs:3132) over the quality range at methods the
    stage-by-stage cases visit only at Q75: the device bitstream equals the oracle's
    byte for byte (RGB and RGBA sources, a 96 x 64 natural image)."""
    for q in (1, 5, 33, 50, 66, 88, 99):
        for color in (zwebp.ColorType.Rgb8, zwebp.ColorType.Rgba8):
            img = _img(96, 64, "natural", 1000 + q, color)
            rc, ref, _ = O.encode(img, 96, 64, color, q, m)
            assert rc == 0
            got = zwebp.encode_frame_lossy(img, 96, 64, color, q, m, ctx=ctx)
            assert bytes(got) == bytes(ref), f"q={q} m={m} color={color}"


@pytest.mark.parametrize("tokens", ["host", "device"])
@pytest.mark.parametrize("name", ["libwebp_natural_64x48_q75.vp8", "gallery1_1.vp8"])
def test_decode_damaged_streams(ctx, monkeypatch, name, tokens):
    """Truncated and byte-flipped streams (the header's 10 bytes kept, so the
    dimensions stay sane): wherever the oracle decodes (decode_frame,
    decoder/vp8.rs:1526, reading zeros past the end as bit_reader.rs does), the
    device path gives the same planes; wherever it fails, the product raises
    DecodingError.  Never a crash or a silent difference."""
    monkeypatch.setenv("ZW_DEC_TOKENS", tokens)
    path = os.path.join(GOLD, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not in tests/golden")
    vp8 = open(path, "rb").read()
    rng = np.random.default_rng(len(vp8))
    cases = [vp8[:n] for n in range(10, len(vp8), max(1, len(vp8) // 24))]
    for _ in range(24):
        b = bytearray(vp8)
        for k in rng.integers(10, len(vp8), int(rng.integers(1, 4))):
            b[k] ^= int(rng.integers(1, 256))
        cases.append(bytes(b))
    agree = 0
    for s in cases:
        rc, r = O.decode(s)
        if rc != 0:
            # the DecodingError variant itself (decoder/api.rs:79-110), not just "raises"
            with pytest.raises(zwebp.DecodingError) as e:
                zwebp.vp8_decode_frame(s, ctx=ctx)
            assert e.value.code == rc, f"variant {e.value.code} != oracle {rc}"
        else:
            fr = zwebp.vp8_decode_frame(s, ctx=ctx)
            assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])
        agree += 1
    assert agree == len(cases)


@pytest.mark.parametrize("ftype,level,sharp,seg", [(0, 6, 0, 0), (0, 40, 3, 1), (1, 20, 0, 0), (0, 63, 7, 1),
                                                   (1, 63, 5, 1), (0, 15, 1, 0)])
@pytest.mark.parametrize("rows", ["1", "0"])
def test_loop_filter_frame(ctx, monkeypatch, ftype, level, sharp, seg, rows):
    """rows=1: the row-parallel kernel (one wave per MB row, cross-CU hand-off); 0: one workgroup per frame."""
    monkeypatch.setenv("ZW_DEC_ROWS", rows)
    rng = np.random.default_rng(level * 10 + sharp)
    mbw, mbh = 23, 17
    nmb = mbw * mbh
    base = synth_rgba(mbw * 16, mbh * 16, 11, "natural")[..., 0]
    y = np.ascontiguousarray((base.astype(np.int32) + rng.integers(-12, 13, base.shape)).clip(0, 255).astype(np.uint8))
    u = np.ascontiguousarray(y[::2, ::2])
    v = np.ascontiguousarray(255 - y[::2, ::2])
    flags = np.zeros((nmb, 4), np.uint8)
    flags[:, 0] = rng.integers(0, 5, nmb)
    flags[:, 1] = rng.integers(0, 4, nmb) if seg else 0
    flags[:, 2] = rng.integers(0, 2, nmb)
    flags[:, 3] = rng.integers(0, 2, nmb)
    seg_lf = (0, -5, 7, 20)
    gy, gu, gv = y.reshape(-1).copy(), u.reshape(-1).copy(), v.reshape(-1).copy()
    zwebp.loop_filter_frame(gy, gu, gv, mbw, mbh, flags, ftype, level, sharp, seg, 1, seg_lf, 1, 2, -3, ctx=ctx)
    infos = (O.MbInfo * nmb)()
    for i in range(nmb):
        infos[i].luma_mode, infos[i].segment, infos[i].skip, infos[i].non_zero_dct = (int(x) for x in flags[i])
    hdr = O.FrameHdr()
    hdr.filter_type, hdr.filter_level, hdr.sharpness = ftype, level, sharp
    hdr.segments_enabled, hdr.seg_delta_values = seg, 1
    for i in range(4):
        hdr.seg_lf_level[i] = seg_lf[i]
    hdr.lf_adj_enabled, hdr.ref_delta0, hdr.mode_delta0 = 1, 2, -3
    oy, ou, ov = y.reshape(-1).copy(), u.reshape(-1).copy(), v.reshape(-1).copy()
    import ctypes
    O.lib().or_loop_filter_c(O._p(oy), O._p(ou), O._p(ov), mbw, mbh, ctypes.addressof(infos), ctypes.byref(hdr))
    assert np.array_equal(gy, oy)
    assert np.array_equal(gu, ou)
    assert np.array_equal(gv, ov)


# --------------------------------------------------------------------------
# Full-size (BASELINE configs) properties
# --------------------------------------------------------------------------
@pytest.mark.parametrize("rows", ["1", "0"])
def test_1080p_encode_decode_roundtrip(ctx, monkeypatch, rows):
    """1920x1080 Q75 m4: GPU bitstream == oracle bitstream; GPU decode of it == oracle decode."""
    monkeypatch.setenv("ZW_ENC_ROWS", rows)
    ref = _check_encode(ctx, 1920, 1080, "natural", 75, 4, 3, 0x5EED0000)
    fr = zwebp.vp8_decode_frame(ref, ctx=ctx)
    rc, r = O.decode(ref)
    assert np.array_equal(fr.ybuf, r["y"]) and np.array_equal(fr.ubuf, r["u"]) and np.array_equal(fr.vbuf, r["v"])


@pytest.mark.parametrize("rows", ["1", "0"])
def test_4k_encode_matches_oracle(ctx, monkeypatch, rows):
    """BASELINE config 5 frame size (3840x2160, 240x135 MBs) Q75 m4: every stage
    and the bitstream equal the oracle's."""
    monkeypatch.setenv("ZW_ENC_ROWS", rows)
    _check_encode(ctx, 3840, 2160, "natural", 75, 4, 3, 0x5EED4000)


@pytest.mark.parametrize("w,h,kind,q", [(1920, 1080, "natural", 75), (1920, 1080, "noise", 95),
                                         (2048, 2048, "noise", 100), (1920, 1080, "flat", 75),
                                         (3840, 2160, "noise", 90)])
def test_device_stats_equal_host_replay(ctx, monkeypatch, w, h, kind, q):
    """k_stats (device ProbaStats pre-aggregation, including the exact replay of
    counters that pass 0xfffe decisions and halve) gives the same bitstreams as
    the host's raster replay of the pass-1 records (ZW_HOST_STATS=1), which the
    oracle-parity tests pin to the reference."""
    imgs = [synth_rgba(w, h, 0x5EED2000 + i, kind) for i in range(2)]
    dev = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, q, 4, ctx=ctx)
    monkeypatch.setenv("ZW_HOST_STATS", "1")
    host = zwebp.encode_batch(imgs, w, h, zwebp.ColorType.Rgba8, q, 4, ctx=ctx)
    for i in range(len(imgs)):
        assert dev[i] == host[i], f"frame {i}"


# --------------------------------------------------------------------------
# a7/a8: quantisation and trellis on independent blocks
# --------------------------------------------------------------------------
@pytest.mark.parametrize("ctype,first,mtype", [(3, 0, 0), (0, 1, 0), (2, 0, 2), (1, 0, 1)])
@pytest.mark.parametrize("trel", [False, True, 2])  # 2: lane-parallel trellis (trellis_g)
@pytest.mark.parametrize("qi", [0, 10, 26, 60, 127])
def test_quant_blocks(ctx, ctype, first, mtype, trel, qi):
    rng = np.random.default_rng(qi * 31 + ctype * 7 + first + trel)
    n = 3000
    scale = rng.choice([8, 40, 200, 1000, 2000], size=(n, 1))
    co = (rng.standard_normal((n, 16)) * scale / (1 + np.arange(16))).astype(np.int32)
    ctx0 = rng.integers(0, 3, n).astype(np.uint8)
    dc_q = [4, 13, 24, 50, 157][[0, 10, 26, 60, 127].index(qi)]
    ac_q = [4, 13, 30, 74, 284][[0, 10, 26, 60, 127].index(qi)]
    probs = rng.integers(1, 256, size=(4, 8, 3, 11)).astype(np.uint8)
    lam = int(rng.integers(1, 5000))
    for pr in (None, probs):
        g = zwebp.quant_blocks(co, ctx0, ctype, first, trel, lam, dc_q, ac_q, mtype, pr, ctx=ctx)
        o = O.quant_blocks(co, ctx0, ctype, first, bool(trel), lam, dc_q, ac_q, mtype, pr)
        bad = np.nonzero((g[0] != o[0]).any(axis=1))[0]
        assert bad.size == 0, f"{bad.size} blocks differ; first {co[bad[0]].tolist()} ctx {ctx0[bad[0]]}: " \
                              f"{g[0][bad[0]].tolist()} vs {o[0][bad[0]].tolist()}"
        assert np.array_equal(g[1], o[1])


# --------------------------------------------------------------------------
# a5/a7/a9/a10: the streaming DCT+quant pass (materialised prediction)
# --------------------------------------------------------------------------
@pytest.mark.parametrize("q_dc,q_ac,mtype,first", [(24, 30, 0, 0), (24, 30, 0, 1), (48, 46, 1, 0), (24, 30, 2, 0),
                                                   (4, 4, 0, 0), (157, 284, 2, 0), (13, 13, 0, 1)])
def test_transform_quant_blocks(ctx, q_dc, q_ac, mtype, first):
    rng = np.random.default_rng(q_dc * 7 + q_ac + mtype + first)
    n = 40000
    base = rng.integers(0, 256, (n, 1))
    src = np.clip(base + rng.integers(-40, 41, (n, 16)), 0, 255).astype(np.uint8)
    src[: n // 8] = rng.integers(0, 256, (n // 8, 16)).astype(np.uint8)  # full-range residuals
    pred = np.clip(base + rng.integers(-20, 21, (n, 16)), 0, 255).astype(np.uint8)
    # extreme residuals (+-255 patterns): the i16 headroom of the packed butterflies
    ext = slice(n // 8, n // 4)
    src[ext] = rng.choice(np.array([0, 255], np.uint8), (n // 8, 16))
    pred[ext] = np.where(rng.random((n // 8, 16)) < 0.9, 255 - src[ext], src[ext])
    lv, rc = zwebp.transform_quant_blocks(src, pred, q_dc, q_ac, mtype, first, ctx=ctx)
    co = O.blocks("or_fdct_c", src.astype(np.int32) - pred.astype(np.int32))
    olv, odq = O.quant_blocks(co, 0, 3, first, False, 0, q_dc, q_ac, mtype)
    orc = np.clip(pred.astype(np.int32) + O.blocks("or_idct_c", odq).reshape(n, 16), 0, 255)
    assert np.array_equal(lv.astype(np.int32), olv)
    assert np.array_equal(rc.astype(np.int32), orc)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1025, 256 * 4 * 3 + 7])
def test_transform_quant_blocks_ragged(ctx, n):
    """Block counts off the wave / workgroup / unroll multiples (the tails)."""
    rng = np.random.default_rng(n)
    src = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    pred = rng.integers(0, 256, (n, 16)).astype(np.uint8)
    lv, rc = zwebp.transform_quant_blocks(src, pred, 24, 30, 0, 0, ctx=ctx)
    co = O.blocks("or_fdct_c", src.astype(np.int32) - pred.astype(np.int32))
    olv, odq = O.quant_blocks(co, 0, 3, 0, False, 0, 24, 30, 0)
    orc = np.clip(pred.astype(np.int32) + O.blocks("or_idct_c", odq).reshape(n, 16), 0, 255)
    assert np.array_equal(lv.astype(np.int32), olv)
    assert np.array_equal(rc.astype(np.int32), orc)


def test_transform_quant_blocks_empty(ctx):
    lv, rc = zwebp.transform_quant_blocks(np.zeros((0, 16), np.uint8), np.zeros((0, 16), np.uint8), 24, 30, ctx=ctx)
    assert lv.shape == (0, 16)

