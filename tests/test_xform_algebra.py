"""CPU check of the arithmetic reformulation k_fdct_quant uses
(image-webp_amd/csrc/zw_xform_kernels.hip, xform_block): packed-i16 butterflies,
v_dot2 rotations with the rounding folded in, and the branch-free quantizer.
Compared against the oracle's fdct (oracle/or_core.c, transform.rs:176) and
quantize_coeff (cost.rs:457) on random and extreme residuals; also asserts the
i16 headroom every packed intermediate relies on."""
import numpy as np

import oracle_lib as O


def _fdct_packed(r):
    r = r.astype(np.int64)
    o = np.zeros_like(r)
    for i in range(4):
        ax, ay = r[:, 4 * i] + r[:, 4 * i + 3], r[:, 4 * i + 1] + r[:, 4 * i + 2]
        dx, dy = r[:, 4 * i] - r[:, 4 * i + 3], r[:, 4 * i + 1] - r[:, 4 * i + 2]
        for v in (ax, ay, dx, dy):
            assert np.abs(v).max() < 32768
        o[:, 4 * i] = ax * 8 + ay * 8
        o[:, 4 * i + 2] = ax * 8 - ay * 8
        o[:, 4 * i + 1] = (dx * 10704 + dy * 4434 + 3625) >> 10
        o[:, 4 * i + 3] = (dx * 4434 - dy * 10704 + 1875) >> 10
    assert np.abs(o).max() < 32768
    c = np.zeros_like(r)
    for i in range(4):
        ax, ay = o[:, i] + o[:, 12 + i], o[:, 4 + i] + o[:, 8 + i]
        dx, dy = o[:, i] - o[:, 12 + i], o[:, 4 + i] - o[:, 8 + i]
        for v in (ax, ay, dx, dy):
            assert np.abs(v).max() < 32768
        c[:, i] = (ax + ay + 7) >> 4
        c[:, 8 + i] = (ax - ay + 7) >> 4
        c[:, 4 + i] = ((dx * 5352 + dy * 2217 + 12000) >> 16) + (dx != 0)
        c[:, 12 + i] = (dx * 2217 - dy * 5352 + 51000) >> 16
    return c


def test_fdct_packed_matches_oracle():
    rng = np.random.default_rng(7)
    n = 60000
    r = rng.integers(-255, 256, (n, 16))
    r[: n // 3] = rng.choice([-255, 255], (n // 3, 16))
    r[n // 3: n // 2] = rng.choice([-255, 0, 255], (n // 2 - n // 3, 16))
    ref = O.blocks("or_fdct_c", r.astype(np.int32))
    assert np.array_equal(_fdct_packed(r), ref.astype(np.int64).reshape(n, 16))


def test_quant_branch_free_identity():
    c = np.arange(-4096, 4097, dtype=np.int64)
    for q in (4, 5, 8, 13, 24, 30, 46, 157, 284):
        iq = (1 << 17) // q
        for b in (0, 1, 96, 110, 115):
            bias = ((b << 17) + 128) >> 8
            ref = np.sign(c) * ((np.abs(c) * iq + bias) >> 17)
            got = (c * iq + np.where(c < 0, (1 << 17) - 1 - bias, bias)) >> 17
            assert np.array_equal(ref, got), (q, b)
