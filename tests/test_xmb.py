"""Streaming DCT+quant pass over per-MB records (zw_transform_quant_mbs,
k_xform_mb; SURVEY 8(a) a4-a7, a9-a11, a15 and the 8(d) roofline pass).

CPU: the oracle's streaming restatement (or_xform_mbs) fed with records built
from an oracle encode's own pass-2 modes, reconstruction and incoming
error-diffusion terms reproduces that encode's final transform bit for bit
(levels and reconstruction) at methods 0-3, where the reference runs
transform_luma_block without the trellis (encoder/vp8.rs:1293, :2674-2679).
GPU: k_xform_mb equals the oracle on the same records -- real ones, and
random ones with every luma / I4 / chroma mode, random edges, diffusion terms
at the clamp limits, all four segments and widths that are not a multiple of
the kernel's 8-MB groups.
"""
import numpy as np
import pytest

import oracle_lib as O
from zwebp.synth import synth_rgba
from zwebp.xmb import RECORD_BYTES, build_records, synthetic_derr


@pytest.fixture(scope="module")
def ctx():
    import zwebp
    return zwebp.Context(0)


def _oracle_case(w, h, q, m, seed=0x5EED0000):
    img = synth_rgba(w, h, seed + w)
    rc, _, d = O.encode(img, w, h, 3, q, m, debug=True)
    assert rc == 0
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    nmb = mbw * mbh
    p2 = d["p2_info"]
    modes = np.zeros((nmb, 20), np.uint8)
    for i in range(nmb):
        modes[i, :4] = (p2[i].luma_mode, p2[i].chroma_mode, p2[i].skip, p2[i].segment)
        modes[i, 4:20] = list(p2[i].bpred)
    recs = build_records(mbw, mbh, modes, d["recon_y"], d["recon_u"], d["recon_v"], d["derr_in"].reshape(nmb, 8))
    sq = np.array(d["seg_quant_index"], np.int32).reshape(1, 4)
    return d, mbw, mbh, modes, recs, sq


@pytest.mark.parametrize("w,h,q,m", [(96, 80, 75, 2), (200, 136, 60, 3), (256, 256, 90, 3), (64, 48, 20, 0),
                                     (330, 270, 75, 1), (17, 33, 100, 3)])
def test_streaming_oracle_equals_encoder_final_transform(w, h, q, m):
    d, mbw, mbh, modes, recs, sq = _oracle_case(w, h, q, m)
    lv, ry, ru, rv = O.xform_mbs(d["src_y"], d["src_u"], d["src_v"], recs, sq, 1, mbw, mbh)
    assert np.array_equal(ry, d["recon_y"]) and np.array_equal(ru, d["recon_u"]) and np.array_equal(rv, d["recon_v"])
    assert np.array_equal(lv.astype(np.int32), d["levels"].reshape(-1, 25, 16))


def test_records_layout():
    """Edge rules of create_border_luma / create_border_chroma (prediction.rs:15-130)."""
    mbw, mbh = 3, 2
    ry = np.arange(mbh * 16 * mbw * 16, dtype=np.uint32).astype(np.uint8)
    ru = (np.arange(mbh * 8 * mbw * 8) * 3).astype(np.uint8)
    rv = (np.arange(mbh * 8 * mbw * 8) * 5).astype(np.uint8)
    modes = np.zeros((mbw * mbh, 20), np.uint8)
    modes[:, 0] = 4
    modes[:, 4:20] = np.arange(16) % 10
    r = build_records(mbw, mbh, modes, ry, ru, rv)
    Y = ry.reshape(32, 48)
    assert r.shape == (6, RECORD_BYTES)
    assert (r[0, 24:44] == 127).all() and (r[0, 44:60] == 129).all() and r[0, 20] == 127 and r[0, 3] == 0
    assert (r[1, 44:60] == Y[0:16, 15]).all() and r[1, 20] == 127 and r[1, 3] == 2
    assert (r[3, 24:40] == Y[15, 0:16]).all() and (r[3, 40:44] == Y[15, 16:20]).all() and r[3, 20] == 129
    assert (r[5, 40:44] == Y[15, 47]).all() and r[5, 20] == Y[15, 31] and r[5, 3] == 3
    U = ru.reshape(16, 24)
    assert (r[4, 64:72] == U[7, 8:16]).all() and (r[4, 72:80] == U[8:16, 7]).all() and r[4, 21] == U[7, 7]
    assert r[0, 4] == (0 | (1 << 4)) and r[0, 11] == (4 | (5 << 4))


def _random_case(rng, nframes, mbw, mbh, i4_frac=0.3):
    nmb = mbw * mbh
    y = rng.integers(0, 256, nframes * nmb * 256, dtype=np.uint8)
    u = rng.integers(0, 256, nframes * nmb * 64, dtype=np.uint8)
    v = rng.integers(0, 256, nframes * nmb * 64, dtype=np.uint8)
    # smooth half of the frames (small residuals, many zero levels) as well as noise
    for f in range(0, nframes, 2):
        y[f * nmb * 256:(f + 1) * nmb * 256] = 100 + (y[f * nmb * 256:(f + 1) * nmb * 256] & 15)
    recs = rng.integers(0, 256, (nframes * nmb, RECORD_BYTES), dtype=np.uint8)
    lm = rng.integers(0, 4, nframes * nmb)
    lm[rng.random(nframes * nmb) < i4_frac] = 4
    recs[:, 0] = lm
    recs[:, 1] = rng.integers(0, 4, nframes * nmb)
    recs[:, 2] = rng.integers(0, 4, nframes * nmb)
    recs[:, 3] = rng.integers(0, 4, nframes * nmb)
    bp = rng.integers(0, 10, (nframes * nmb, 16))
    recs[:, 4:12] = bp[:, 0::2] | (bp[:, 1::2] << 4)
    dr = rng.integers(-127, 128, (nframes * nmb, 8)).astype(np.int8)
    dr[::7] = 127
    dr[1::7] = -127
    recs[:, 12:20] = dr.view(np.uint8)
    recs[:, 23] = 0
    recs[:, 60:64] = 0
    sq = rng.integers(0, 128, (nframes, 4)).astype(np.int32)
    sq[0] = (0, 127, 26, 60)
    return y, u, v, recs, sq


@pytest.mark.gpu
@pytest.mark.parametrize("nframes,mbw,mbh,i4", [(2, 8, 3, 0.3), (1, 13, 5, 0.0), (3, 5, 4, 1.0), (2, 17, 2, 0.5),
                                                (1, 1, 1, 1.0), (1, 120, 68, 0.03)])
def test_gpu_xform_mbs_random(ctx, nframes, mbw, mbh, i4):
    import zwebp
    rng = np.random.default_rng(nframes * 1000 + mbw * 10 + mbh)
    y, u, v, recs, sq = _random_case(rng, nframes, mbw, mbh, i4)
    want = O.xform_mbs(y, u, v, recs, sq, nframes, mbw, mbh)
    got = zwebp.transform_quant_mbs(y, u, v, recs, sq, nframes, mbw, mbh, ctx=ctx)
    for name, a, b in zip(("levels", "ry", "ru", "rv"), got, want):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"{name}: {len(bad)} differences, first {bad[:4].tolist()}"


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,q,m", [(200, 136, 60, 3), (1920, 1080, 75, 4), (330, 270, 95, 6)])
def test_gpu_xform_mbs_encoder_records(ctx, w, h, q, m):
    """Records of a real encode (its modes, reconstruction and diffusion
    terms): the device pass equals the oracle; at m <= 3 both equal the
    encoder's own pass-2 levels and reconstruction."""
    import zwebp
    d, mbw, mbh, modes, recs, sq = _oracle_case(w, h, q, m)
    got = zwebp.transform_quant_mbs(d["src_y"], d["src_u"], d["src_v"], recs, sq, 1, mbw, mbh, ctx=ctx)
    want = O.xform_mbs(d["src_y"], d["src_u"], d["src_v"], recs, sq, 1, mbw, mbh)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    if m <= 3:
        assert np.array_equal(got[1], d["recon_y"]) and np.array_equal(got[2], d["recon_u"])
        assert np.array_equal(got[0].astype(np.int32), d["levels"].reshape(-1, 25, 16))


_DEVICE_FORM = r"""
import sys
import numpy as np
import torch                      # torch's HIP runtime first, then the library (as bench.py does)
dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
import zwebp
import oracle_lib as O
from test_xmb import _random_case
from zwebp.xmb import synthetic_derr
mbw, mbh, nf = 9, 3, 2
y, u, v, recs, sq = _random_case(np.random.default_rng(5), nf, mbw, mbh)
recs[:, 12:20] = synthetic_derr(nf * mbw * mbh, 7).view(np.uint8)
want = O.xform_mbs(y, u, v, recs, sq, nf, mbw, mbh)
t = {k: torch.from_numpy(np.ascontiguousarray(a)).to(dev) for k, a in
     (("y", y), ("u", u), ("v", v), ("r", recs.reshape(-1)), ("s", zwebp.xmb_seg_table(sq)))}
lv = torch.empty(nf * mbw * mbh * 400, dtype=torch.int16, device=dev)
ry, ru, rv = torch.empty_like(t["y"]), torch.empty_like(t["u"]), torch.empty_like(t["v"])
ctx = zwebp.Context(0)
args = [t["y"].data_ptr(), t["u"].data_ptr(), t["v"].data_ptr(), t["r"].data_ptr(), t["s"].data_ptr(),
        lv.data_ptr(), ry.data_ptr(), ru.data_ptr(), rv.data_ptr()]
zwebp.transform_quant_mbs_device(nf, mbw, mbh, *args, ctx=ctx)
torch.cuda.synchronize()
assert np.array_equal(lv.cpu().numpy().reshape(-1, 25, 16), want[0])
assert np.array_equal(ry.cpu().numpy(), want[1]) and np.array_equal(rv.cpu().numpy(), want[3])
# two launches in flight on two streams at once (each stream has its own I4
# queue): both equal the oracle
cases = []
for seed, (nf2, w2, h2) in ((11, (3, 40, 20)), (12, (2, 33, 25))):
    c = _random_case(np.random.default_rng(seed), nf2, w2, h2, 0.5)
    tt = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (c[0], c[1], c[2], c[3].reshape(-1))]
    tt.append(torch.from_numpy(zwebp.xmb_seg_table(c[4])).to(dev))
    outs = (torch.empty(nf2 * w2 * h2 * 400, dtype=torch.int16, device=dev), torch.empty_like(tt[0]),
            torch.empty_like(tt[1]), torch.empty_like(tt[2]))
    cases.append((nf2, w2, h2, c, tt, outs, torch.cuda.Stream(dev)))
torch.cuda.synchronize()
for rep in range(3):
    for nf2, w2, h2, c, tt, outs, st in cases:
        zwebp.transform_quant_mbs_device(nf2, w2, h2, *[x.data_ptr() for x in tt], *[o.data_ptr() for o in outs],
                                         stream=st.cuda_stream, ctx=ctx)
    torch.cuda.synchronize()
    for nf2, w2, h2, c, tt, outs, st in cases:
        want2 = O.xform_mbs(c[0], c[1], c[2], c[3], c[4], nf2, w2, h2)
        assert np.array_equal(outs[0].cpu().numpy().reshape(-1, 25, 16), want2[0]), "levels, two streams"
        assert np.array_equal(outs[1].cpu().numpy(), want2[1]), "ry, two streams"
# more launch streams than the context keeps I4 queues for (8): the least
# recently used stream's queue is handed over, every launch still exact
nf2, w2, h2, c, tt, outs, _ = cases[0]
want2 = O.xform_mbs(c[0], c[1], c[2], c[3], c[4], nf2, w2, h2)
streams = [torch.cuda.Stream(dev) for _ in range(11)]
for rep in range(2):
    for st in streams:
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        zwebp.transform_quant_mbs_device(nf2, w2, h2, *[x.data_ptr() for x in tt], *[o.data_ptr() for o in outs],
                                         stream=st.cuda_stream, ctx=ctx)
        st.synchronize()
        assert np.array_equal(outs[0].cpu().numpy().reshape(-1, 25, 16), want2[0]), "levels, stream rotation"
bad = list(args)
bad[3] += 4  # misaligned records
try:
    zwebp.transform_quant_mbs_device(nf, mbw, mbh, *bad, ctx=ctx)
    sys.exit("misaligned record pointer accepted")
except zwebp.ZwError:
    pass
print("device form ok")
"""


@pytest.mark.gpu
def test_gpu_xform_mbs_device_form():
    """Device pointers from torch tensors (the bench's form).  Own process:
    torch's HIP runtime must initialise before the library's in one process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(root, "image-webp_amd"),
                                                       os.path.join(root, "tests")]))
    r = subprocess.run([sys.executable, "-c", _DEVICE_FORM], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "device form ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_gpu_xform_mbs_errors(ctx):
    import zwebp
    mbw, mbh, nf = 9, 3, 2
    y, u, v, recs, sq = _random_case(np.random.default_rng(5), nf, mbw, mbh)
    with pytest.raises(zwebp.ZwError):
        zwebp.transform_quant_mbs(y, u, v, recs, np.full((nf, 4), 200, np.int32), nf, mbw, mbh, ctx=ctx)
    with pytest.raises(ValueError):
        zwebp.transform_quant_mbs(y, u, v, recs[:-1], sq, nf, mbw, mbh, ctx=ctx)


@pytest.mark.gpu
def test_gpu_xform_mbs_i4_drain_at_scale(ctx):
    """k_xform_mb_i4q over more I4 MBs than its grid takes in one pass (16
    frames of 120 x 68 MBs, every MB I4: 130 560 queue entries; the grid is
    sized for an I4 share of 1/16, 8 160 MBs a pass), then launches back to back on the same queue with
    other I4 shares: each launch appends to its own parity's count and the
    drain zeroes the other's, so every launch equals the oracle."""
    import zwebp
    for nf, mbw, mbh, i4, seed in ((16, 120, 68, 1.0, 1), (2, 120, 68, 0.0, 2), (3, 33, 17, 0.6, 3),
                                   (1, 120, 68, 1.0, 4)):
        y, u, v, recs, sq = _random_case(np.random.default_rng(seed), nf, mbw, mbh, i4)
        got = zwebp.transform_quant_mbs(y, u, v, recs, sq, nf, mbw, mbh, ctx=ctx)
        want = O.xform_mbs(y, u, v, recs, sq, nf, mbw, mbh)
        for name, a, b in zip(("levels", "ry", "ru", "rv"), got, want):
            bad = np.argwhere(a != b)
            assert bad.size == 0, f"case {seed} {name}: {len(bad)} differences, first {bad[:4].tolist()}"


@pytest.mark.gpu
def test_gpu_xform_mbs_queue_overflow_reported(monkeypatch):
    """An I4 queue whose count is stale (test hook: preset past the launch's
    MBs, as a shared queue would leave it) makes k_xform_mb flag the context's
    error word instead of writing past the queue, k_xform_mb_i4 read nothing
    through it, and the call -- and every later one on that context -- fail
    with DeviceError; other contexts are unaffected."""
    import zwebp
    mbw, mbh, nf = 9, 3, 2
    y, u, v, recs, sq = _random_case(np.random.default_rng(9), nf, mbw, mbh, 0.5)
    bad = zwebp.Context(0)
    try:
        monkeypatch.setenv("ZW_XMB_FORCE_OVERFLOW", "1")
        with pytest.raises(zwebp.ZwError) as e:
            zwebp.transform_quant_mbs(y, u, v, recs, sq, nf, mbw, mbh, ctx=bad)
        assert e.value.code == 4
        monkeypatch.delenv("ZW_XMB_FORCE_OVERFLOW")
        with pytest.raises(zwebp.ZwError):
            zwebp.transform_quant_mbs(y, u, v, recs, sq, nf, mbw, mbh, ctx=bad)
    finally:
        bad.close()
    good = zwebp.Context(0)
    try:
        got = zwebp.transform_quant_mbs(y, u, v, recs, sq, nf, mbw, mbh, ctx=good)
        want = O.xform_mbs(y, u, v, recs, sq, nf, mbw, mbh)
        assert all(np.array_equal(a, b) for a, b in zip(got, want))
    finally:
        good.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,bpp,nframes", [(1920, 1080, 4, 2), (97, 33, 4, 2), (200, 136, 3, 1), (15, 7, 4, 1),
                                             (64, 48, 3, 2), (130, 17, 3, 1), (257, 255, 4, 1)])
def test_gpu_xform_mbs_rgb(ctx, w, h, bpp, nframes):
    """The pass fused with convert_image_yuv (zw_transform_quant_mbs_rgb, BASELINE
    config 2 from RGB(A)): equals the oracle's rgb_to_yuv420 followed by the
    streaming restatement, at aligned widths (16-/8-byte pixel runs) and at
    ragged ones, odd heights and the MB padding rows (per-pixel edge path)."""
    import zwebp
    rng = np.random.default_rng(w * 7 + h + bpp)
    mbw, mbh = (w + 15) // 16, (h + 15) // 16
    _, _, _, recs, sq = _random_case(rng, nframes, mbw, mbh, 0.2)
    imgs = [synth_rgba(w, h, 0x5EED3000 + f, "natural" if f % 2 else "noise")[..., :bpp] for f in range(nframes)]
    planes = [O.rgb_to_yuv420(np.ascontiguousarray(im), w, h, bpp) for im in imgs]
    y, u, v = (np.concatenate([p[k] for p in planes]) for k in range(3))
    want = O.xform_mbs(y, u, v, recs, sq, nframes, mbw, mbh)
    got = zwebp.transform_quant_mbs_rgb(np.stack(imgs), w, h, bpp, recs, sq, nframes, ctx=ctx)
    for name, a, b in zip(("levels", "ry", "ru", "rv"), got, want):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f"{name}: {len(bad)} differences, first {bad[:4].tolist()}"
