"""Deterministic synthetic frames for tests and benchmarks.

synth_rgba(w, h, seed): per-channel gradient + 8x8 checker (amplitude 32) +
approximately Gaussian noise (sigma ~6, Irwin-Hall of 4 hashed uniforms),
alpha = 255.  kind="alpha": the same colours with a real alpha plane, a
cut-out: transparent background, an opaque disc with a soft 32-pixel edge
carrying noise (sigma ~6), and a smooth ramp across the top eighth -- the
content encode_alpha_lossless codes for a product shot or a sticker.  Counter-based hashing (PCG-style output permutation of the
pixel index mixed with the seed) so any frame can be generated independently,
vectorised with numpy.  Seed convention from BASELINE.md: 0x5EED0000 + index.
"""
import numpy as np

_M = np.uint64(0xFFFFFFFF)


def _hash32(x):
    # PCG output function (RXS-M-XS 32) on a 64-bit LCG step of x.
    x = (x * np.uint64(6364136223846793005) + np.uint64(1442695040888963407)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    s = (x >> np.uint64(32)) & _M
    w = ((s >> ((s >> np.uint64(28)) + np.uint64(4))) ^ s) * np.uint64(277803737) & _M
    return ((w >> np.uint64(22)) ^ w) & _M


def synth_rgba(w, h, seed=0x5EED0000, kind="natural"):
    """Return a (h, w, 4) uint8 RGBA array."""
    if kind == "flat":
        out = np.full((h, w, 4), 128, np.uint8)
        out[..., 3] = 255
        return out
    yy, xx = np.mgrid[0:h, 0:w]
    idx = (yy.astype(np.uint64) * np.uint64(w) + xx.astype(np.uint64)) * np.uint64(4)
    base = np.uint64(seed) << np.uint64(32)
    if kind == "noise":
        out = np.empty((h, w, 4), np.uint8)
        for c in range(3):
            out[..., c] = (_hash32(base + idx + np.uint64(c)) & np.uint64(0xFF)).astype(np.uint8)
        out[..., 3] = 255
        return out
    checker = (((yy >> 3) + (xx >> 3)) & 1) * 32 - 16
    grads = [
        (xx * 200) // max(w - 1, 1) + 20,
        (yy * 200) // max(h - 1, 1) + 20,
        ((xx + yy) * 160) // max(w + h - 2, 1) + 40,
    ]
    out = np.empty((h, w, 4), np.uint8)
    for c in range(3):
        acc = np.zeros((h, w), np.int64)
        for k in range(4):
            acc += (_hash32(base + idx + np.uint64(c) + np.uint64(k << 20)) & np.uint64(0xFFFF)).astype(np.int64)
        # sum of 4 U(0,65535): mean 131070, sd ~37837 -> scale to sigma 6
        noise = ((acc - 131070) * 6) // 37837
        out[..., c] = np.clip(grads[c] + checker + noise, 0, 255).astype(np.uint8)
    out[..., 3] = 255 if kind != "alpha" else _alpha_plane(w, h, base, yy, xx, idx)
    return out


def _alpha_plane(w, h, base, yy, xx, idx):
    # a cut-out: transparent background, an opaque disc whose 32-pixel soft edge
    # carries noise (sigma ~6), and a smooth horizontal ramp across the top eighth
    cy, cx, r = h / 2.0, w / 2.0, 0.35 * min(w, h)
    d = np.sqrt((yy - cy) ** 2 + (xx - cx) ** 2)
    a = np.clip((r + 16 - d) * (255.0 / 32.0), 0, 255).astype(np.int64)
    acc = np.zeros((h, w), np.int64)
    for k in range(4):
        acc += (_hash32(base + idx + np.uint64(3) + np.uint64((k + 8) << 20)) & np.uint64(0xFFFF)).astype(np.int64)
    noise = ((acc - 131070) * 6) // 37837
    a = np.where((a > 0) & (a < 255), a + noise, a)
    top = yy * 8 < h
    a = np.where(top, (xx * 255) // max(w - 1, 1), a)
    return np.clip(a, 0, 255).astype(np.uint8)
