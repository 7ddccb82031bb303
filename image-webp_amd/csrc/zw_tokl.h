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
TKL_HD constexpr uint32_t band(uint32_t n)
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
TKL_HD constexpr void desc(uint32_t c, uint32_t k, uint32_t* d)
{
    d[0] = d[1] = d[2] = d[3] = 0;
    if (k > 24 || (k == 0 && c == 1)) return;
    uint32_t tb = 0, lb = 0, t = 0, first = 0;
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

// Stage 2's MB boundaries (one MB per lane, started from stage 1's snapshot).
// mb_begin: the record starts at L.hb; mr = the MB's ZW_TOK_MODE bytes (as
// words), TL = its block contexts at its start (top bits 0..8 from the MB
// above, left bits 16..24 from the MB to the left).  Not for skipped MBs (a
// header-only record, written by the caller).
template <class M>
TKL_HD void mb_begin(Lane& L, M& m, const uint32_t* mr, uint32_t TL)
{
    constexpr uint32_t U = M::U;
    L.w0 = mr[0];
    L.w2 = mr[2];
    L.w3 = mr[3];
    const uint32_t lm = mr[0] & 7u;
    L.TL = TL;
    const uint32_t c = lm == 4u ? 1u : 0u;
    L.dsb = c * NDESC;
    L.k = c;
    L.nzm2 = L.nlv = 0;
    L.lvb = L.hb + 80u;
    uint32_t d[4];
    m.desc(L.dsb + L.k + 1u, d);
    L.dnx = d[0];
    L.dny = d[1];
    L.dnz = d[2];
    L.dnw = d[3];
    m.desc(L.dsb + L.k, d);
    L.dx = d[0];
    L.dy = d[1];
    const uint32_t ctx = ((L.TL >> (L.dy & 15u)) & 1u) + ((L.TL >> ((L.dy >> 4) & 31u)) & 1u);
    L.first = (L.dy >> 9) & 1u;
    L.n = L.first;
    L.eob = 0;
    L.tbl = d[3] * U + m.lane0;
    L.rbl = (d[2] + ctx * 11u) * U + m.lane0;
    if (c) m.st16c(true, L.hb + 16u, 0u);  // start[0] of an I4 MB
    if (L.first) m.st16c(true, L.lvb, 0u);
    L.st = 0;
    L.acc = 0;
    L.p = m.prob_at(L.rbl);
    m.tt(0, L.t0, L.t1);
    L.phase = PH_DECIDE;
}

// mb_end: the MB's last block ended (k == 25): its header, the total level
// count and the zero pad after its levels; L.hb = the end of the record.
// (step()'s stores can fall past the record's end -- a ZERO run's zeros after
// the last nonzero level, position 0 of an empty luma block -- so a memory
// interface whose MBs are written in parallel drops stores past the MB's end.)
template <class M>
TKL_HD void mb_end(Lane& L, M& m)
{
    m.st128(L.hb, L.w0, L.nzm2 >> 1, L.w2, L.w3);
    m.st128(L.hb + 64u, L.nlv, 0u, 0u, 0u);
    const uint32_t end = (L.lvb + 15u) & ~15u;
    for (uint32_t a = L.lvb; a < end; a += 2u) m.st16c(true, a, 0u);  // the zero pad (not past the record)
    L.hb = end;
}

// A header-only record (a skipped MB, mb_no_coeff_skip): every start 0.
template <class M>
TKL_HD void mb_skip(M& m, uint32_t hb, const uint32_t* mr)
{
    m.st128(hb, mr[0], 0u, mr[2], mr[3]);
    m.st128(hb + 16u, 0u, 0u, 0u, 0u);
    m.st128(hb + 32u, 0u, 0u, 0u, 0u);
    m.st128(hb + 48u, 0u, 0u, 0u, 0u);
    m.st128(hb + 64u, 0u, 0u, 0u, 0u);
}

// Stage 2's lane from stage 1's MB snapshot: s0 = bits shifted out at the MB's
// start, s1 = the window's top byte | rm1 << 8 | min(vb, 8) << 16 (the top
// min(vb, 8) bits of that byte are valid, the rest not yet loaded), len = the
// partition's bytes.  The window is refilled from the stream at s0 + that
// count, so the MB's decisions are the ones stage 1 made.
template <class M>
TKL_HD void from_snapshot(Lane& L, M& m, uint32_t s0, uint32_t s1, uint32_t len)
{
    init(L, len, true);
    const uint32_t vbs = (s1 >> 16) & 15u;
    const uint64_t top = (uint64_t)(s1 & 255u) << 56;
    L.V = vbs ? (top | (m.bits64(s0 + vbs) >> vbs)) : m.bits64(s0);
    L.vb = 64u;
    L.bp = s0 + 64u;
    L.rm1 = (s1 >> 8) & 255u;
}

}  // namespace tokl

// ===========================================================================
// Stage 1: the serial decision chain alone (the device's k_dec_tok1).
//
// A frame's decisions cannot be split (each one's range and value depend on the
// one before), so the chain's length per decision is what a batch waits for.
// Stage 1 carries only what the next decision needs: the bool decoder, one
// state index S and the block contexts.  S folds the tree node, the position n
// and the row context into one transition table T1[S][bit] (982 states per
// block type; the same for every frame), whose entry also holds the next
// state's probability source (a row entry of the frame's table, or a fixed
// probability), so a decision is the arithmetic, one table select and two LDS
// reads (probability, T1 entry) for the next.  Levels, starts and records are
// not built here: at each MB start the lane stores a 16-byte snapshot (stream
// position, the window's top byte, range, block contexts), and stage 2
// (k_dec_tok2, one MB per lane, thousands of MBs in parallel) replays each MB
// from its snapshot with step() above and writes the packed records.
//
// States (n = position 0..15, c = row context 0..2):
//   TN(n, c, node)  tree node 0..10 of the token at n, row (band(n), c)
//   FR(first, c)    node 0 of a block's first token (EOB here: the block is empty)
//   SG(n, c')       the sign of the token at n; c' = the next row context (1 after a ONE, else 2)
//   XS(n, j)        extra bit j of a category token at n (tokl states 12 + j), fixed probabilities
// Entry (state, bit): next state * 8 (its T1 row's byte offset, bits 0..12) |
// its probability source << 13 (a row entry e as e * U, or the fixed
// probability) | fixed << 29 | the block's non-zero flag << 30 | block end << 31.
// A block-end entry's next state is the next block's FR(first, ctx), which the
// lane computes from the contexts (popcount of its two context bits).
// ===========================================================================
namespace tok1 {
using namespace tokl;

// SINK (982): the state of a lane that makes no decision (waiting for the MB
// phase, or done): both entries lead back to it and leave everything but the
// decoder unchanged, so the wave steps every lane without a branch.
constexpr uint32_t FR0 = 528, SG0 = 534, XS0 = 566, SINK = 982, NS = 983;
constexpr uint32_t E_BE = 1u << 31, E_NZ = 1u << 30, E_FX = 1u << 29, E_S = 0x1FFFu, E_PV = 13;
constexpr uint32_t E_SINK = SINK * 8u | (128u << E_PV) | E_FX;
constexpr uint32_t NDESC1 = 27;
// the lane's k: 0..24 a block of the MB (decisions), 25 the MB phase is due, 26 done
constexpr uint32_t K_MB = 25, K_DONE = 26;

TKL_HD constexpr uint32_t tn(uint32_t n, uint32_t c, uint32_t node) { return n * 33u + c * 11u + node; }
TKL_HD constexpr uint32_t fr(uint32_t first, uint32_t c) { return FR0 + first * 3u + c; }
TKL_HD constexpr uint32_t sg(uint32_t n, uint32_t c1) { return SG0 + n * 2u + (c1 - 1u); }
TKL_HD constexpr uint32_t xs(uint32_t n, uint32_t j) { return XS0 + n * 26u + j; }

// tokl states 12..37 (the categories' extra bits): probability and successor (11 = the sign)
TKL_HD constexpr uint32_t cat_prob(uint32_t s)
{
    constexpr uint8_t P[26] = {159, 165, 145, 173, 148, 140, 176, 155, 140, 135, 180, 157, 141,
                               134, 130, 254, 254, 243, 230, 196, 177, 153, 140, 133, 130, 129};
    return P[s - 12u];
}
TKL_HD constexpr uint32_t cat_next(uint32_t s)
{
    return (s == 12u || s == 14u || s == 17u || s == 21u || s == 26u || s == 37u) ? 11u : s + 1u;
}

template <uint32_t U>
struct Table {
    uint32_t e[2 * NS];
    // an entry going to state s (its probability source with it)
    static constexpr uint32_t to(uint32_t s)
    {
        if (s < FR0) {
            const uint32_t n = s / 33u, c = (s % 33u) / 11u, node = s % 11u;
            return s * 8u | ((band(n) * 33u + c * 11u + node) * U) << E_PV;
        }
        if (s < XS0) return s * 8u | (128u << E_PV) | E_FX;  // a sign (FR states are never a direct target)
        const uint32_t j = (s - XS0) % 26u;
        return s * 8u | (cat_prob(12u + j) << E_PV) | E_FX;
    }
    // the token at n ended (a ZERO goes on at node 1 with context 0, a token at node 0)
    static constexpr uint32_t next_pos(uint32_t n, uint32_t c1, uint32_t node)
    {
        return n + 1u == 16u ? (E_BE | E_NZ) : to(tn(n + 1u, c1, node));
    }
    constexpr Table() : e()
    {
        for (uint32_t n = 0; n < 16; n++)
            for (uint32_t c = 0; c < 3; c++) {
                uint32_t* t = e + 2 * tn(n, c, 0);
                t[0] = E_BE | E_NZ;                       // node 0: EOB
                t[1] = to(tn(n, c, 1));
                t[2] = next_pos(n, 0, 1);                 // node 1: ZERO
                t[3] = to(tn(n, c, 2));
                t[4] = to(sg(n, 1));                      // node 2: ONE
                t[5] = to(tn(n, c, 3));
                t[6] = to(tn(n, c, 4));                   // node 3
                t[7] = to(tn(n, c, 6));
                t[8] = to(sg(n, 2));                      // node 4: TWO
                t[9] = to(tn(n, c, 5));
                t[10] = t[11] = to(sg(n, 2));             // node 5: THREE / FOUR
                t[12] = to(tn(n, c, 7));                  // node 6
                t[13] = to(tn(n, c, 8));
                t[14] = to(xs(n, 0));                     // node 7: cat1 / cat2
                t[15] = to(xs(n, 1));
                t[16] = to(tn(n, c, 9));                  // node 8
                t[17] = to(tn(n, c, 10));
                t[18] = to(xs(n, 3));                     // node 9: cat3 / cat4
                t[19] = to(xs(n, 6));
                t[20] = to(xs(n, 10));                    // node 10: cat5 / cat6
                t[21] = to(xs(n, 15));
            }
        for (uint32_t first = 0; first < 2; first++)
            for (uint32_t c = 0; c < 3; c++) {
                e[2 * fr(first, c)] = E_BE;  // EOB first: an empty block
                e[2 * fr(first, c) + 1] = to(tn(first, c, 1));
            }
        e[2 * SINK] = e[2 * SINK + 1] = E_SINK;
        for (uint32_t n = 0; n < 16; n++) {
            for (uint32_t c1 = 1; c1 < 3; c1++) e[2 * sg(n, c1)] = e[2 * sg(n, c1) + 1] = next_pos(n, c1, 0);
            for (uint32_t j = 0; j < 26; j++) {
                const uint32_t ns = cat_next(12u + j);
                e[2 * xs(n, j)] = e[2 * xs(n, j) + 1] = ns == 11u ? to(sg(n, 2)) : to(xs(n, ns - 12u));
            }
        }
    }
};

// Descriptor of block k in MB class c (tokl::desc's blocks): its two context
// bits in TL, its type's row base (type * 264 * U), FR(first, 0) * 8, and the
// probability source of FR(first, 0) (band(first) * 33 * U); k = 25, 26 and
// (c = 1, k = 0) lead to SINK (no context bits, FR = SINK).
template <uint32_t U>
TKL_HD constexpr void desc1(uint32_t c, uint32_t k, uint32_t* d)
{
    uint32_t q[4] = {0, 0, 0, 0};
    tokl::desc(c, k, q);
    d[0] = q[0];
    d[1] = q[3] * U;
    const uint32_t first = (q[1] >> 9) & 1u;
    d[2] = q[0] ? fr(first, 0) * 8u : SINK * 8u;
    d[3] = band(first) * 33u * U;
}

struct Lane1 {
    uint64_t V;
    uint32_t vb, bp, rm1;
    uint32_t pr, pv, pf;       // this decision's probability: pf ? pv : pr (pr read from the frame's table)
    uint32_t t0, t1;           // its T1 entries
    uint32_t tbl, TL, dx, k, dsb;
    uint32_t dnx, dnt, dnf, dnp;  // the next block's descriptor
    uint32_t mbi, mbx, sk;        // sk: the MB phase continues a run of skipped MBs
    uint32_t tcn;                 // the top contexts of the next MB's column (read ahead)
};

TKL_HD void init1(Lane1& L, bool active)
{
    L.V = 0;
    L.vb = L.bp = 0;
    L.rm1 = 254;
    L.pr = L.pv = L.pf = 0;
    L.t0 = L.t1 = E_SINK;
    L.tbl = L.TL = L.dx = L.dsb = 0;
    L.k = active ? K_MB : K_DONE;
    L.dnx = L.dnt = L.dnf = L.dnp = 0;
    L.mbi = L.mbx = 0;
    L.sk = 1;  // (nothing to finish before MB 0)
    L.tcn = 0;
}

template <class M>
TKL_HD void topup1(Lane1& L, M& m)
{
    if (L.vb < 64u) {
        const uint64_t s = m.bits64(L.bp);
        L.V |= s >> L.vb;
        L.bp += 64u - L.vb;
        L.vb = 64u;
    }
}

TKL_HD uint32_t popc(uint32_t x)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_popcount(x);
#else
    return (uint32_t)__builtin_popcount(x);
#endif
}

// bfi(m, a, b) = (a & m) | (b & ~m): a per-lane select by a mask (v_bfi_b32),
// which the compiler keeps as one instruction instead of an exec-mask branch
TKL_HD uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

// One decision (tokl::step's arithmetic), the transition and, at a block's end,
// the next block's first state from its contexts.  A lane in SINK (k >= 25)
// keeps its decoder state; the rest of its state stays by SINK's entries.
template <class M>
TKL_HD void step1(Lane1& L, M& m)
{
    constexpr uint32_t U = M::U;
    const bool fz = L.k >= K_MB;
    const uint32_t p = bfi(L.pf, L.pv, L.pr);  // (pf: all ones for a fixed probability)
    const uint32_t sm1 = mul24(L.rm1, p) >> 8;  // split - 1
    const uint32_t big = (sm1 << 24) + (1u << 24);
    uint32_t vh = (uint32_t)(L.V >> 32);
    const bool bit = vh >= big;
    // the next decision's state first: its probability and T1 reads go out
    // before the rest of the step, which runs while they are in flight
    const uint32_t e = bit ? L.t1 : L.t0;
    const uint32_t bm = (uint32_t)((int32_t)e >> 31);                       // all ones at a block end
    const uint32_t nzm = (uint32_t)((int32_t)(e << 1) >> 31) & L.dx;        // the ended block's bits if non-zero
    const uint32_t TL = bfi(bm, (L.TL & ~L.dx) | nzm, L.TL);
    const uint32_t bctx = popc(TL & L.dnx);
    const uint32_t S8 = bfi(bm, L.dnf + bctx * 8u, e & E_S);
    const uint32_t pv = bfi(bm, L.dnp + mul24(bctx, 11u * U), (e >> E_PV) & 0xFFFFu);
    const uint32_t tbl = bfi(bm, L.dnt, L.tbl);
    L.pr = m.prob_at(tbl + pv);
    m.tt1(S8, L.t0, L.t1);
#ifdef __HIP_DEVICE_COMPILE__
    __builtin_amdgcn_sched_barrier(0);
#endif
    L.TL = TL;
    L.tbl = tbl;
    L.pv = pv;
    L.pf = (uint32_t)((int32_t)(e << 2) >> 31);  // E_FX as a mask (block-end entries have it clear)
    // the block bookkeeping (the next descriptor's read goes out next)
    L.dx = bfi(bm, L.dnx, L.dx);
    const uint32_t k = L.k - bm;
    L.k = k;
    uint32_t dn[4];
    m.desc1(L.dsb + k + 1u, dn);
#ifdef __HIP_DEVICE_COMPILE__
    __builtin_amdgcn_sched_barrier(0);
#endif
    // the decoder's update
    const uint32_t r = bit ? L.rm1 - sm1 : sm1 + 1u;
    vh -= bit ? big : 0u;
    const uint32_t sh = (uint32_t)__builtin_clz(r) - 24u;
    L.rm1 = fz ? L.rm1 : (r << sh) - 1u;
    {
        const uint64_t Vn = ((((uint64_t)vh) << 32) | (uint32_t)L.V) << sh;  // (halves selected: no exec branch)
        const uint32_t lo = fz ? (uint32_t)L.V : (uint32_t)Vn, hi = fz ? (uint32_t)(L.V >> 32) : (uint32_t)(Vn >> 32);
        L.V = ((uint64_t)hi << 32) | lo;
    }
    L.vb = fz ? L.vb : L.vb - sh;
    L.dnx = dn[0];
    L.dnt = dn[1];
    L.dnf = dn[2];
    L.dnp = dn[3];
#ifdef __HIP_DEVICE_COMPILE__
    __builtin_amdgcn_sched_barrier(0);
#endif
}

// The MB phase (lanes with k = 25): finish the MB whose last block ended (its
// top contexts), then start the next MB (a skipped one is context bookkeeping
// only: the lane stays at k = 25) or finish the frame (k = 26).  m.cls(i): bit 0 = MB i is I4, bit 1 = skipped.
// m.snap(c, i, s0, s1, TL): if c, MB i's snapshot (from_snapshot above).  The
// next column's top contexts are read when an MB starts (the row above wrote
// them long before), so the MB phase waits for no context read.  (Frames of one
// MB column, whose next MB's top contexts are the MB's own, parse on the host.)
// m.set_tcx(mbw, v) writes a dummy column.
template <class M>
TKL_HD void mb1(Lane1& L, M& m)
{
    constexpr uint32_t U = M::U;
    // (written branch-free: at 64 lanes some lane is at an MB boundary in most
    // MB phases, and every branch costs the whole wave)
    const bool fin = L.sk == 0u;  // the MB's last block ended: its column's top contexts, then the next MB
    m.set_tcx(fin ? L.mbx : m.mbw, L.TL & 511u);  // (column mbw: a dummy)
    const uint32_t mbi = L.mbi + (fin ? 1u : 0u);
    const uint32_t mbx = fin ? (L.mbx + 1u == m.mbw ? 0u : L.mbx + 1u) : L.mbx;
    const bool done = mbi == m.nmb;
    const uint32_t cs = m.cls(done ? mbi - 1u : mbi);
    const bool skip = (cs & 2u) != 0u, i4 = (cs & 1u) != 0u;
    const uint32_t TL = (mbx == 0 ? 0u : (L.TL & 0x01FF0000u)) | L.tcn;
    const uint32_t mbxn = mbx + 1u == m.mbw ? 0u : mbx + 1u;
    const uint32_t tcn = m.tcx(mbxn);  // (the row above wrote it; with mbw = 2 and fin, the write above)
    // a skipped MB: parse_mbs's contexts (every one but Y2's, kept for I4 MBs, becomes 0)
    const uint32_t TLs = i4 ? (TL & 0x00010001u) : 0u;
    m.set_tcx(skip && !done ? mbx : m.mbw, TLs & 511u);
    // an MB with tokens: its snapshot and first block
    const bool start = !done && !skip;
    const uint32_t vbs = L.vb < 8u ? L.vb : 8u;
    m.snap(start, mbi, L.bp - L.vb, (uint32_t)(L.V >> 56) | (L.rm1 << 8) | (vbs << 16), TL);
    // the class's first two blocks (constants: I16 starts at Y2, I4 at Y 0)
    uint32_t a0[4] = {0, 0, 0, 0}, a1[4] = {0, 0, 0, 0}, b0[4] = {0, 0, 0, 0}, b1[4] = {0, 0, 0, 0};
    desc1<U>(0, 0, a0);
    desc1<U>(0, 1, a1);
    desc1<U>(1, 1, b0);
    desc1<U>(1, 2, b1);
    const uint32_t dx = i4 ? b0[0] : a0[0], tbl = i4 ? b0[1] : a0[1];
    const uint32_t bctx = popc(TL & dx);
    const uint32_t S8 = start ? (i4 ? b0[2] : a0[2]) + bctx * 8u : SINK * 8u;
    const uint32_t pv = (i4 ? b0[3] : a0[3]) + mul24(bctx, 11u * U);
    L.pv = pv;
    L.pf = 0;
    L.pr = m.prob_at(tbl + pv);
    m.tt1(S8, L.t0, L.t1);
    L.dx = dx;
    L.tbl = tbl;
    L.dsb = i4 ? NDESC1 : 0u;
    L.dnx = i4 ? b1[0] : a1[0];
    L.dnt = i4 ? b1[1] : a1[1];
    L.dnf = i4 ? b1[2] : a1[2];
    L.dnp = i4 ? b1[3] : a1[3];
    L.k = done ? K_DONE : (skip ? K_MB : (i4 ? 1u : 0u));
    L.sk = skip ? 1u : 0u;
    L.TL = skip ? TLs : TL;
    L.tcn = tcn;
    L.mbi = skip ? mbi + 1u : mbi;
    L.mbx = skip ? mbxn : mbx;
}

}  // namespace tok1
