"""Per-MB records of the streaming DCT+quant pass (zw_transform_quant_mbs).

build_records() makes, for every MB of a frame, the 96-byte record the pass
reads instead of the encoder's running state: the modes and segment an
encode chose, the borders create_border_luma / create_border_chroma
(common/prediction.rs:15-130) build from the reconstruction of the MBs above
and to the left, and the incoming error-diffusion terms
(apply_chroma_error_diffusion, encoder/vp8.rs:572-647).  Layout: include/zwebp.h.
"""
import numpy as np

RECORD_BYTES = 96


def build_records(mbw, mbh, modes, ry, ru, rv, derr=None):
    """modes: (nmb, >=20) uint8 rows of (luma, chroma, skip, segment, bpred[16])
    (Pipeline.mbinfo / the oracle's MbInfo); ry/ru/rv: the frame's MB-padded
    reconstruction; derr: (nmb, 8) int8 incoming diffusion terms (U top0, top1,
    left0, left1, then V), or None for zeros.  Returns (nmb, 96) uint8."""
    nmb = mbw * mbh
    modes = np.asarray(modes, np.uint8).reshape(nmb, -1)
    Y = np.asarray(ry, np.uint8).reshape(mbh * 16, mbw * 16)
    U = np.asarray(ru, np.uint8).reshape(mbh * 8, mbw * 8)
    V = np.asarray(rv, np.uint8).reshape(mbh * 8, mbw * 8)
    r = np.zeros((mbh, mbw, RECORD_BYTES), np.uint8)
    m = modes.reshape(mbh, mbw, -1)
    r[:, :, 0] = m[:, :, 0]
    r[:, :, 1] = m[:, :, 1]
    r[:, :, 2] = m[:, :, 3] & 3
    ys, xs = np.meshgrid(np.arange(mbh), np.arange(mbw), indexing="ij")
    r[:, :, 3] = (ys > 0).astype(np.uint8) | ((xs > 0).astype(np.uint8) << 1)
    bp = m[:, :, 4:20].astype(np.uint8)
    r[:, :, 4:12] = (bp[:, :, 0::2] & 15) | ((bp[:, :, 1::2] & 15) << 4)
    if derr is not None:
        r[:, :, 12:20] = np.asarray(derr, np.int8).reshape(mbh, mbw, 8).view(np.uint8)
    # luma: corner (20), top 16 + top-right 4 (24..43), left 16 (44..59)
    top = np.full((mbh, mbw, 20), 127, np.uint8)
    if mbh > 1:
        above = Y[15:-1:16, :]  # bottom row of each MB row above: (mbh-1, mbw*16)
        ext = np.concatenate([above, np.repeat(above[:, -1:], 4, axis=1)], axis=1)  # last MB: replicate
        idx = np.arange(mbw)[:, None] * 16 + np.arange(20)[None, :]
        top[1:] = ext[:, idx]
    r[:, :, 24:44] = top
    left = np.full((mbh, mbw, 16), 129, np.uint8)
    if mbw > 1:
        lc = Y[:, 15:-1:16]  # (mbh*16, mbw-1): right column of each MB to the left
        left[:, 1:] = lc.reshape(mbh, 16, mbw - 1).transpose(0, 2, 1)
    r[:, :, 44:60] = left
    corner = np.full((mbh, mbw), 127, np.uint8)
    corner[1:, 0] = 129
    if mbh > 1 and mbw > 1:
        corner[1:, 1:] = Y[15:-1:16, 15:-1:16]
    r[:, :, 20] = corner
    # chroma: corners (21, 22), top 8 / left 8 per plane (64.., 80..)
    for k, P in enumerate((U, V)):
        t = np.full((mbh, mbw, 8), 127, np.uint8)
        if mbh > 1:
            t[1:] = P[7:-1:8, :].reshape(mbh - 1, mbw, 8)
        lft = np.full((mbh, mbw, 8), 129, np.uint8)
        if mbw > 1:
            lft[:, 1:] = P[:, 7:-1:8].reshape(mbh, 8, mbw - 1).transpose(0, 2, 1)
        c = np.full((mbh, mbw), 127, np.uint8)
        c[1:, 0] = 129
        if mbh > 1 and mbw > 1:
            c[1:, 1:] = P[7:-1:8, 7:-1:8]
        r[:, :, 64 + 16 * k:72 + 16 * k] = t
        r[:, :, 72 + 16 * k:80 + 16 * k] = lft
        r[:, :, 21 + k] = c
    return r.reshape(nmb, RECORD_BYTES)


def synthetic_derr(nmb, seed):
    """Deterministic incoming diffusion terms in [-24, 24] (a bench workload where
    no encode state is at hand)."""
    i = np.arange(nmb * 8, dtype=np.uint64)
    s = np.uint64(((seed & 0xFFFFFFFF) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
    x = (i + s) * np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(31)
    x *= np.uint64(0x94D049BB133111EB)
    x ^= x >> np.uint64(29)
    return ((x % np.uint64(49)).astype(np.int16) - 24).astype(np.int8).reshape(nmb, 8)
