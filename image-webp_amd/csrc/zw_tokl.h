// zw_tokl.h -- the VP8 token partition of one frame as a per-lane state machine
// (read_coefficients, decoder/vp8.rs:872-1058, over the boolean decoder of
// bit_reader.rs:254-640 / RFC 6386 section 7).
//
// One lane decodes one frame.  On the device a wave runs 64 frames side by side
// (k_dec_tokl, zw_dec_tokens.hip); on the host the same functions step one frame
// (zw_dbg_tokl_frame, the CPU check against the host parser).  The memory
// interface M supplies the tables, the stream bits, the per-MB modes and the
// record stores; the output is the packed MB records of zw_common.h ZW_DREC_*,
// byte-identical to zw_dec_host.cpp parse_mbs.
//
// step() is one binary decision and everything it implies, written branch-free
// (selects, and stores with a condition that the device turns into an
// out-of-range offset): in SIMT every branch a lane takes costs the whole wave,
// and at 64 lanes some lane ends a token or a block at almost every decision.
// The rare work -- the end and start of an MB -- waits for the MB phase.
//
// * Bool decoder: a 64-bit window V whose top byte is compared with the split,
//   rm1 = range - 1 in [127, 254], vb valid bits.  Top-ups append the next
//   64 - vb stream bits (bit-granular), so any schedule that keeps vb >= 8 at a
//   decision gives the same decisions; a decision consumes at most 7 bits, so
//   a top-up every 8 decisions suffices.  The reference loads 7 bytes, then
//   single bytes, then one zero byte and sets eof: a frame fails
//   (read_levels_into -> -1) iff some decision starts with S >= 8 len - 7, S =
//   the bits shifted out so far (bp - vb); checked at each block's end on its
//   last decision (S only grows).
// * Token tree: 38 states (tree nodes 0..10 with the row's probabilities, the
//   sign, 26 extra-bit states with fixed probabilities) and a transition table
//   TT[state][bit] (te() below); the events EOB / ZERO / TOKEN end a token.
// * Blocks: per MB class (I16 with Y2, or I4) a descriptor per block k (order
//   Y2, Y 0..15, U 0..3, V 0..3): context bit positions in TL (top bits 0..8,
//   left bits 16..24), the probability row base, the first position.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TKL_HD __host__ __device__ __forceinline__

namespace tokl {

enum : uint32_t { S_SIGN = 11, NST = 38, EV_EOB = 40, EV_ZERO = 41, EV_TOKEN = 42 };
enum : uint32_t { PH_DECIDE = 0, PH_MB = 1, PH_DONE = 2 };
constexpr int PROBS = 1056;  // bytes of probabilities per frame, [type 4][band 8][ctx 3][node 11]
constexpr int NDESC = 27;    // descriptors per MB class (k = 0..24; 25, 26 dummies)

// TT entry for (state, bit): next state (or event) | probability of a
// fixed-probability next state << 6 | multiplier of acc << 14 | addend << 15 |
// next state is a tree node (probability from the row) << 26.  acc becomes
// acc * mul + add: set on entering the sign or a category, accumulated over the
// extra bits (weight of each bit = 2^(bits left)).
constexpr uint32_t te(uint32_t ns, uint32_t pc, uint32_t mul, uint32_t av, uint32_t tree)
{
    return ns | (pc << 6) | (mul << 14) | (av << 15) | (tree << 26);
}
constexpr uint32_t tr(uint32_t n) { return te(n, 0, 0, 0, 1); }
constexpr uint32_t sg(uint32_t v) { return te(S_SIGN, 128, 0, v, 0); }
// an extra bit of weight w going to state ns (probability pc); bit 0 / bit 1
constexpr uint32_t x0(uint32_t ns, uint32_t pc) { return te(ns, pc, 1, 0, 0); }
constexpr uint32_t x1(uint32_t ns, uint32_t pc, uint32_t w) { return te(ns, pc, 1, w, 0); }

// PROB_DCT_CAT (vp8.rs) enter the category states: cat1 {159}, cat2 {165, 145},
// cat3 {173, 148, 140}, cat4 {176, 155, 140, 135}, cat5 {180, 157, 141, 134,
// 130}, cat6 {254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129}; bases 5,
// 7, 11, 19, 35, 67 (3 + (8 << cat) for cat3..6).
#define ZW_TOKL_TT_INIT                                                                              \
    {                                                                                                \
        /* N0 */ tokl::te(tokl::EV_EOB, 0, 0, 0, 0), tokl::tr(1),                                   \
        /* N1 */ tokl::te(tokl::EV_ZERO, 0, 0, 0, 0), tokl::tr(2),                                  \
        /* N2 */ tokl::sg(1), tokl::tr(3),                                                           \
        /* N3 */ tokl::tr(4), tokl::tr(6),                                                           \
        /* N4 */ tokl::sg(2), tokl::tr(5),                                                           \
        /* N5 */ tokl::sg(3), tokl::sg(4),                                                           \
        /* N6 */ tokl::tr(7), tokl::tr(8),                                                           \
        /* N7 */ tokl::te(12, 159, 0, 5, 0), tokl::te(13, 165, 0, 7, 0),                             \
        /* N8 */ tokl::tr(9), tokl::tr(10),                                                          \
        /* N9 */ tokl::te(15, 173, 0, 11, 0), tokl::te(18, 176, 0, 19, 0),                           \
        /* N10 */ tokl::te(22, 180, 0, 35, 0), tokl::te(27, 254, 0, 67, 0),                          \
        /* sign (the bit is the sign) */ tokl::te(tokl::EV_TOKEN, 0, 1, 0, 0),                      \
        tokl::te(tokl::EV_TOKEN, 0, 1, 0, 0),                                                        \
        /* 12 cat1 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                       \
        /* 13 cat2 */ tokl::x0(14, 145), tokl::x1(14, 145, 2),                                       \
        /* 14 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                            \
        /* 15 cat3 */ tokl::x0(16, 148), tokl::x1(16, 148, 4),                                       \
        /* 16 */ tokl::x0(17, 140), tokl::x1(17, 140, 2),                                            \
        /* 17 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                            \
        /* 18 cat4 */ tokl::x0(19, 155), tokl::x1(19, 155, 8),                                       \
        /* 19 */ tokl::x0(20, 140), tokl::x1(20, 140, 4),                                            \
        /* 20 */ tokl::x0(21, 135), tokl::x1(21, 135, 2),                                            \
        /* 21 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                            \
        /* 22 cat5 */ tokl::x0(23, 157), tokl::x1(23, 157, 16),                                      \
        /* 23 */ tokl::x0(24, 141), tokl::x1(24, 141, 8),                                            \
        /* 24 */ tokl::x0(25, 134), tokl::x1(25, 134, 4),                                            \
        /* 25 */ tokl::x0(26, 130), tokl::x1(26, 130, 2),                                            \
        /* 26 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                            \
        /* 27 cat6 */ tokl::x0(28, 254), tokl::x1(28, 254, 1024),                                    \
        /* 28 */ tokl::x0(29, 243), tokl::x1(29, 243, 512),                                          \
        /* 29 */ tokl::x0(30, 230), tokl::x1(30, 230, 256),                                          \
        /* 30 */ tokl::x0(31, 196), tokl::x1(31, 196, 128),                                          \
        /* 31 */ tokl::x0(32, 177), tokl::x1(32, 177, 64),                                           \
        /* 32 */ tokl::x0(33, 153), tokl::x1(33, 153, 32),                                           \
        /* 33 */ tokl::x0(34, 140), tokl::x1(34, 140, 16),                                           \
        /* 34 */ tokl::x0(35, 133), tokl::x1(35, 133, 8),                                            \
        /* 35 */ tokl::x0(36, 130), tokl::x1(36, 130, 4),                                            \
        /* 36 */ tokl::x0(37, 129), tokl::x1(37, 129, 2),                                            \
        /* 37 */ tokl::x0(11, 128), tokl::x1(11, 128, 1),                                            \
    }

// 24-bit multiply (v_mul_u32_u24 on the device; operands < 2^24)
TKL_HD uint32_t mul24(uint32_t a, uint32_t b)
{
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t d;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
#else
    return a * b;
#endif
}

// COEFF_BANDS (vp8.rs) as nibbles: positions 0..7 in the low word, 8..15 in the high one
TKL_HD uint32_t band(uint32_t n)
{
    const uint32_t w = n < 8u ? 0x65463210u : 0x76666666u;
    return (w >> (4u * (n & 7u))) & 15u;
}

// Block descriptor of block k in MB class c (0: I16 + Y2, 1: I4), four words:
//   x = the block's context bits in TL (top bit tb, left bit 16 + lb)
//   y = tb | (16 + lb) << 4 | first << 9
//   z = the row base of its first position: type * 264 + band(first) * 33
//   w = its type's base: type * 264
// Blocks: k = 0 Y2 (type 1), 1..16 Y (type 0 after Y2, else 3; first 1 after
// Y2), 17..20 U, 21..24 V (type 2); the context bits follow parse_mbs (top:
// 0 Y2, 1..4 Y columns, 5..6 U, 7..8 V; left the same with rows).
TKL_HD void desc(uint32_t c, uint32_t k, uint32_t* d)
{
    d[0] = d[1] = d[2] = d[3] = 0;
    if (k > 24 || (k == 0 && c == 1)) return;
    uint32_t tb, lb, t, first = 0;
    if (k == 0) {
        tb = lb = 0;
        t = 1;
    } else if (k <= 16) {
        tb = ((k - 1) & 3) + 1;
        lb = ((k - 1) >> 2) + 1;
        t = c == 0 ? 0 : 3;
        first = c == 0 ? 1 : 0;
    } else {
        const uint32_t q = k - 17, pl = q >> 2;
        tb = (q & 1) + 5 + 2 * pl;
        lb = ((q >> 1) & 1) + 5 + 2 * pl;
        t = 2;
    }
    d[0] = (1u << tb) | (1u << (16 + lb));
    d[1] = tb | ((16 + lb) << 4) | (first << 9);
    d[2] = t * 264 + band(first) * 33;
    d[3] = t * 264;
}

// Probability rows are addressed in the memory interface's units: entry i of
// the lane's table is at M::U * i + m.lane0 (the device's LDS table is
// [entry][lane] bytes, U = 64; the host's is the frame's own table, U = 1).
struct Lane {
    uint64_t V;    // window: stream bits MSB first, the top byte compared with the split
    uint32_t vb;   // valid bits in V
    uint32_t bp;   // stream bits appended to V so far
    uint32_t rm1;  // range - 1
    int32_t thr;   // 8 len - 7
    uint32_t st, p, t0, t1, acc;  // state, its probability and TT entries (bit 0 / 1)
    uint32_t n, eob, first, rbl, tbl;  // position; row address; type base address (+ lane0)
    uint32_t k, dsb, TL, nzm2, nlv;    // dsb = c * NDESC; nzm2: block k's non-zero flag at bit k (bit 0 = Y2)
    uint32_t dx, dy, dnx, dny, dnz, dnw;  // this block's descriptor (x, y) and the next one's
    uint32_t hb, lvb;                     // record bytes: the MB's header, its next level (hb + 80 + 2 nlv)
    uint32_t mbi, mbx;
    uint32_t w0, w2, w3;  // the MB's mode words (header bytes 0..3, 8..15)
    uint32_t phase, bad;
};

TKL_HD void init(Lane& L, uint32_t len, bool active)
{
    L.V = 0;
    L.vb = 0;
    L.bp = 0;
    L.rm1 = 254;
    L.thr = 8 * (int32_t)len - 7;
    L.st = L.p = L.t0 = L.t1 = L.acc = 0;
    L.n = L.eob = L.first = L.rbl = L.tbl = 0;
    L.k = L.dsb = L.TL = L.nzm2 = L.nlv = 0;
    L.dx = L.dy = L.dnx = L.dny = L.dnz = L.dnw = 0;
    L.hb = 0;
    L.lvb = 80;
    L.mbi = L.mbx = 0;
    L.w0 = L.w2 = L.w3 = 0;
    L.phase = active ? PH_MB : PH_DONE;
    L.bad = 0;
}

// Append stream bits up to a full window.
template <class M>
TKL_HD void topup(Lane& L, M& m)
{
    if (L.vb < 64u) {
        const uint64_t s = m.bits64(L.bp);
        L.V |= s >> L.vb;
        L.bp += 64u - L.vb;
        L.vb = 64u;
    }
}

// One binary decision with probability L.p in state L.st, and what it ends:
// a token (store its level, next position and probability row), a block
// (contexts, non-zero mask, the next block's descriptor, row and start), an MB
// (the lane goes to PH_MB).  The next decision's probability and TT entries
// are read as soon as its row and state are known, before the bookkeeping, so
// the reads land meanwhile.  Positions a ZERO token stores past the block's
// last nonzero level are overwritten by the next block or lie in the record's
// zero pad.
template <class M>
TKL_HD void step(Lane& L, M& m)
{
    constexpr uint32_t U = M::U;
    // the decision (RFC 6386 7.3 in the range - 1 form)
    const uint32_t vb0 = L.vb;
    const uint32_t split = (mul24(L.rm1, L.p) >> 8) + 1u;  // 1 + ((range - 1) * prob >> 8)
    const uint32_t big = split << 24;
    uint32_t vh = (uint32_t)(L.V >> 32);
    const bool bit = vh >= big;
    const uint32_t r = bit ? L.rm1 + 1u - split : split;
    vh = bit ? vh - big : vh;
    const uint32_t sh = (uint32_t)__builtin_clz(r) - 24u;
    L.rm1 = (r << sh) - 1u;
    L.V = ((((uint64_t)vh) << 32) | (uint32_t)L.V) << sh;
    L.vb = vb0 - sh;
    // the token tree
    const uint32_t e = bit ? L.t1 : L.t0;
    const uint32_t ns = e & 63u;
    const uint32_t acc = L.acc * ((e >> 14) & 1u) + ((e >> 15) & 2047u);
    L.acc = acc;
    const bool ev = ns >= EV_EOB, zero = ns == EV_ZERO, tok = ns == EV_TOKEN, wr = ns >= EV_ZERO;
    const uint32_t n0 = L.n;
    const uint32_t n1 = n0 + (wr ? 1u : 0u);
    const uint32_t eob1 = tok ? n1 : L.eob;
    const bool be = ns == EV_EOB || n1 == 16u;
    // the next row within the block (ctx 0 after a ZERO, 1 after a one, else
    // 2; tree node 1 after a ZERO: no EOB check), or the next block's first
    const uint32_t ctx = zero ? 0u : (acc > 1u ? 2u : 1u);
    const uint32_t rblt = L.tbl + mul24(band(n1), 33u * U) + mul24(ctx, 11u * U);
    const bool nz = n1 > L.first;
    const uint32_t TLn = nz ? (L.TL | L.dx) : (L.TL & ~L.dx);
    const uint32_t TL = be ? TLn : L.TL;
    const uint32_t dy = be ? L.dny : L.dy;
    const uint32_t bctx = ((TL >> (dy & 15u)) & 1u) + ((TL >> ((dy >> 4) & 31u)) & 1u);
    const uint32_t rblb = mul24(L.dnz, U) + m.lane0 + mul24(bctx, 11u * U);
    const uint32_t st = be ? 0u : (ev ? (zero ? 1u : 0u) : ns);
    const uint32_t rbl = be ? rblb : (ev ? rblt : L.rbl);
    L.st = st;
    L.rbl = rbl;
    const uint32_t pt = m.prob_at(rbl + st * U);  // (every lane reads: no branch)
    m.tt(st, L.t0, L.t1);
    // bookkeeping (while the reads are in flight)
    const int lvl = tok ? (bit ? -(int)acc : (int)acc) : 0;
    m.st16c(wr, L.lvb + 2u * n0, (uint32_t)lvl);
    const bool eof = (int32_t)(L.bp - vb0) >= L.thr;
    L.bad = (be && eof) ? 1u : L.bad;
    L.TL = TL;
    L.nzm2 |= (be && nz) ? (1u << L.k) : 0u;
    const uint32_t nlv = L.nlv + (be ? eob1 : 0u);
    L.nlv = nlv;
    const uint32_t lvb = L.lvb + (be ? 2u * eob1 : 0u);
    L.lvb = lvb;
    const uint32_t k = L.k + (be ? 1u : 0u);
    L.k = k;
    const uint32_t first = (dy >> 9) & 1u;
    const uint32_t tbln = mul24(L.dnw, U) + m.lane0;
    L.tbl = be ? tbln : L.tbl;
    L.dx = be ? L.dnx : L.dx;
    L.dy = dy;
    uint32_t dn[4];
    m.desc(L.dsb + k + 1u, dn);
    L.dnx = dn[0];
    L.dny = dn[1];
    L.dnz = dn[2];
    L.dnw = dn[3];
    L.first = be ? first : L.first;
    L.n = be ? first : n1;
    L.eob = be ? 0u : eob1;
    m.st16c(be, L.hb + 14u + 2u * k, nlv);               // start[k - 1] (k = 25: start[24], the total)
    m.st16c(be && first != 0u && k < 25u, lvb, 0u);      // position 0 of a luma block after Y2
    L.phase = (be && eof) ? PH_DONE : ((be && k == 25u) ? PH_MB : L.phase);
    L.p = (be || ev || ((e >> 26) & 1u)) ? pt : ((e >> 6) & 255u);
}

template <class M>
TKL_HD void next_mb(Lane& L, M& m)
{
    L.mbi++;
    if (++L.mbx == m.mbw) L.mbx = 0;
}

// The MB phase: finish the MB whose last block ended (its header and the zero
// pad after its levels), then start the next MB or finish the frame.  A skipped
// MB (mb_no_coeff_skip) is a header-only record; it returns with the lane still
// at PH_MB.
template <class M>
TKL_HD void mb_phase(Lane& L, M& m)
{
    constexpr uint32_t U = M::U;
    if (L.k == 25u) {
        m.st128(L.hb, L.w0, L.nzm2 >> 1, L.w2, L.w3);
        m.st128(L.hb + 64u, L.nlv, 0u, 0u, 0u);
        m.st128(L.lvb, 0u, 0u, 0u, 0u);  // (2-byte aligned)
        L.hb = (L.lvb + 15u) & ~15u;
        m.set_tcx(L.mbx, L.TL & 511u);
        next_mb(L, m);
        L.k = 0;
    }
    if (L.mbi == m.nmb) {
        m.moff(m.nmb, L.hb);
        L.phase = PH_DONE;
        return;
    }
    m.moff(L.mbi, L.hb);
    uint32_t mr[4];
    m.mode(L.mbi, mr);
    L.w0 = mr[0];
    L.w2 = mr[2];
    L.w3 = mr[3];
    const uint32_t lm = mr[0] & 7u, skip = (mr[0] >> 5) & 1u;
    L.TL = (L.mbx == 0 ? 0u : (L.TL & 0x01FF0000u)) | m.tcx(L.mbx);
    if (skip) {
        // parse_mbs: every context but Y2's (kept for I4 MBs) becomes 0
        L.TL &= lm != 4u ? 0u : 0x00010001u;
        m.st128(L.hb, mr[0], 0u, mr[2], mr[3]);
        m.st128(L.hb + 16u, 0u, 0u, 0u, 0u);
        m.st128(L.hb + 32u, 0u, 0u, 0u, 0u);
        m.st128(L.hb + 48u, 0u, 0u, 0u, 0u);
        m.st128(L.hb + 64u, 0u, 0u, 0u, 0u);
        L.hb += 80u;
        m.set_tcx(L.mbx, L.TL & 511u);
        next_mb(L, m);
        return;
    }
    const uint32_t c = lm == 4u ? 1u : 0u;
    L.dsb = c * NDESC;
    L.k = c;
    L.nzm2 = L.nlv = 0;
    L.lvb = L.hb + 80u;
    uint32_t d[4];
    m.desc(L.dsb + L.k, d);
    L.dx = d[0];
    L.dy = d[1];
    m.desc(L.dsb + L.k + 1u, d);
    L.dnx = d[0];
    L.dny = d[1];
    L.dnz = d[2];
    L.dnw = d[3];
    m.desc(L.dsb + L.k, d);
    const uint32_t ctx = ((L.TL >> (L.dy & 15u)) & 1u) + ((L.TL >> ((L.dy >> 4) & 31u)) & 1u);
    L.first = (L.dy >> 9) & 1u;
    L.n = L.first;
    L.eob = 0;
    L.tbl = d[3] * U + m.lane0;
    L.rbl = (d[2] + ctx * 11u) * U + m.lane0;
    if (c) m.st16c(true, L.hb + 16u, 0u);  // start[0] of an I4 MB
    if (L.first) m.st16c(true, L.lvb, 0u);
    L.st = 0;
    L.p = m.prob_at(L.rbl);
    m.tt(0, L.t0, L.t1);
    L.phase = PH_DECIDE;
}

}  // namespace tokl
