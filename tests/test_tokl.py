"""The device token parse's state machine, checked on the CPU (no GPU needed).

The device parse (zw_dec_tokens.hip) runs zw_tokl.h in two stages: k_dec_tok1,
one frame per lane, the boolean decoder (bit_reader.rs:254-640 / RFC 6386 s7)
with a bit-granular 64-bit window and one table-driven state per decision (the
token tree, position and row context folded into one transition table), which
stores a snapshot at each MB start; and k_dec_tok2, one MB per lane, which
replays each MB from its snapshot with the full bookkeeping (read_coefficients,
decoder/vp8.rs:872-1058) and writes the packed records.  zw_dbg_tokl_frame steps
the SAME functions over one frame on the host (stage 1, then stage 2's count,
offsets and records) and compares the packed MB records with the host parser's
(parse_mbs, the product's host path, which test_gpu_parity pins to the oracle
and the reference goldens).  Here: every golden stream, oracle streams over the
quality range and odd sizes, and truncated / byte-flipped streams, whose failure
must be reported exactly where parse_mbs fails (the eof rule: a frame fails when
a decision starts with all bytes consumed past 8 len - 7 bits)."""
import glob
import os

import numpy as np
import pytest

import oracle_lib as O
import zwebp
from zwebp.synth import synth_rgba

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _goldens():
    return sorted(glob.glob(os.path.join(GOLD, "*.vp8")))


@pytest.mark.parametrize("path", _goldens(), ids=lambda p: os.path.basename(p))
def test_tokl_goldens(path):
    vp8 = open(path, "rb").read()
    rc, match = zwebp.dbg_tokl_frame(vp8)
    one_column = ((vp8[6] | vp8[7] << 8) & 0x3FFF) <= 16  # (parsed on the host only)
    assert rc == 0 and match == (-1 if one_column else 1)


@pytest.mark.parametrize("q", [0, 5, 20, 50, 75, 90, 100])
def test_tokl_oracle_streams(q):
    """Oracle encodes (flat, noise, natural content; sizes with partial MBs),
    including Q100 streams whose levels need the large categories."""
    for (w, h, kind) in ((96, 64, "natural"), (37, 21, "noise"), (130, 18, "flat"), (64, 64, "noise"),
                         (16, 72, "noise"), (24, 40, "natural"), (8, 8, "noise")):  # (one and two MB columns)
        img = synth_rgba(w, h, 77 + q + w, kind)
        rc, s, _ = O.encode(img, w, h, 3, q, 4)
        assert rc == 0
        rc, match = zwebp.dbg_tokl_frame(s)
        assert rc == 0 and match == (1 if w > 16 else -1), (w, h, kind, q)  # (one MB column: host only)


def test_tokl_partitions_stay_on_host():
    img = synth_rgba(64, 48, 5, "natural")
    rc, s, _ = O.encode(img, 64, 48, 3, 75, 4, nparts=4)
    assert rc == 0
    assert zwebp.dbg_tokl_frame(s) == (0, -1)


@pytest.mark.parametrize("name", ["libwebp_natural_64x48_q75.vp8", "gallery1_1.vp8", "gallery2_2_a.vp8",
                                  "libwebp_noise_256x256_q90.vp8"])
def test_tokl_damaged_streams(name):
    """Every truncation point of the token partition's tail and random byte
    flips: the state machine fails exactly where parse_mbs fails (the same
    DecodingError), and otherwise gives the same records."""
    vp8 = open(os.path.join(GOLD, name), "rb").read()
    rng = np.random.default_rng(len(vp8))
    cases = [vp8[:n] for n in range(10, len(vp8), max(1, len(vp8) // 64))]
    cases += [vp8[:n] for n in range(max(10, len(vp8) - 40), len(vp8))]  # the last bytes one by one
    for _ in range(64):
        b = bytearray(vp8)
        for k in rng.integers(10, len(vp8), int(rng.integers(1, 4))):
            b[k] ^= int(rng.integers(1, 256))
        cases.append(bytes(b))
    taken = failed = 0
    for s in cases:
        rc, match = zwebp.dbg_tokl_frame(s)
        if match == -1:
            continue
        assert match == 1, (len(s), rc)
        taken += 1
        failed += rc != 0
    assert taken > len(cases) // 3 and failed > 0, (taken, failed)
