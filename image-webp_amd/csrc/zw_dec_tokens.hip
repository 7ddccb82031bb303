// zw_dec_tokens.hip -- the VP8 token partition parsed on the device (gfx950),
// in two stages.
//
// read_coefficients (decoder/vp8.rs:872-1058) over the boolean decoder of
// bit_reader.rs:254-640.  A frame's token partition is one serial chain of
// binary decisions (each one's range and value depend on the one before), so a
// frame cannot be split, and a batch's launch takes as long as one frame's
// chain.  The host keeps the frame header and the first partition's per-MB
// modes (ZW_TOK_MODE bytes per MB, a short chain); the records written here
// are byte-identical to the host parser's (zw_dec_host.cpp parse_mbs), and
// k_dec_recon reads them unchanged.
//
//   k_dec_tok1      stage 1, one frame per LANE: the decision chain alone
//                   (zw_tokl.h tok1: one table-driven state per decision) and a
//                   16-byte snapshot per MB start.
//   k_dec_tok2<0>   stage 2, one MB per lane over every frame: each MB replayed
//                   from its snapshot (zw_tokl.h step(), the full bookkeeping),
//                   counting its record's bytes (and the eof rule's failures).
//   k_dec_tok_scan  per frame: MB record offsets (exclusive scan) and the error word.
//   k_dec_tok_fbase frame bases (256-B aligned) and the batch's record bytes.
//   k_dec_tok2<1>   the same replay, writing the records (after the host has
//                   sized the record buffer from that total).
// Stage 1 is the serial part; stage 2 is thousands of short independent chains.
#include "zw_dev.h"
#include "zw_tokl.h"

namespace {

__constant__ uint32_t d_TOKL_TT[2 * tokl::NST] = ZW_TOKL_TT_INIT;
__constant__ tok1::Table<64> d_T1 = tok1::Table<64>();

// stage-1 LDS (dwords): T1 (static), then dynamic: probabilities [264][64] (entry i of lane l at byte i * 64 + l),
// stream ring [16][64] (64 bytes per lane), class ring [4][64] (16 MBs a word), sync
// words, stage-1 descriptors, then the top contexts [mbw + 1][64] u16 (column mbw: a dummy)
constexpr int TK1_P = 264 * 64, TK1_SR = 16 * 64, TK1_CR = 4 * 64, TK1_SY = 4 * 64 + 4, TK1_T = 2 * tok1::NS,
              TK1_D = 2 * 4 * tok1::NDESC1;
constexpr int TK1_FIXED = TK1_P + TK1_SR + TK1_CR + TK1_SY + TK1_D + 32;  // dynamic (+ the dummy column); T1 is static
constexpr uint32_t TKL_SPIN = 1u << 22;

typedef __attribute__((address_space(3))) uint32_t lds_u32;  // (a generic volatile pointer would become a flat access)

struct Tok1Dev {
    static constexpr uint32_t U = 64;
    const uint8_t* P8;
    const uint32_t* T1;
    const uint32_t* D1;
    const uint32_t* SR;
    uint16_t* TCX;
    const uint32_t* CR;
    volatile lds_u32* sfill;
    volatile lds_u32* scons;
    volatile lds_u32* cfill;
    volatile lds_u32* ccons;
    uint32_t cw, cq;  // the class word of MBs [16 cq, 16 cq + 16): 2 bits per MB (bit 0 I4, bit 1 skipped)
    __amdgpu_buffer_rsrc_t sr;  // the wave's snapshots
    uint32_t sbase;
    uint32_t lane, nmb, mbw, tmo;

    DI uint32_t prob_at(uint32_t a) const { return P8[a + lane]; }
    DI void tt1(uint32_t s8, uint32_t& t0, uint32_t& t1) const
    {
        const uint2 v = *(const uint2*)((const uint8_t*)T1 + s8);
        t0 = v.x;
        t1 = v.y;
    }
    DI void desc1(uint32_t i, uint32_t* d) const
    {
        const uint4 v = *(const uint4*)(D1 + 4 * i);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    // 64 stream bits from bit bp on, MSB first (dwords hold 4 stream bytes, the
    // first in the low byte)
    // The fill counter and the three words are read back to back (one LDS round
    // trip): LDS operations of a wave execute in order, and the feeder releases
    // a chunk (its words, then the counter) before the counter can show it.  The
    // wait-and-reread path is for a ring that has fallen behind (rare).
    DI uint64_t bits64(uint32_t bp)
    {
        const uint32_t dw = bp >> 5, need = ((4u * dw + 11u) >> 4) + 1u;
        const volatile lds_u32* R = (const volatile lds_u32*)SR;
        const uint32_t sf = sfill[lane];
        uint32_t d0 = R[((dw) & 15u) * 64u + lane], d1 = R[((dw + 1u) & 15u) * 64u + lane],
                 d2 = R[((dw + 2u) & 15u) * 64u + lane];
        if (sf < need) {
            for (uint32_t i = 0; sfill[lane] < need; i++) {
                if (i > TKL_SPIN) {
                    tmo = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // (the feeder is another wave)
            d0 = R[((dw) & 15u) * 64u + lane];
            d1 = R[((dw + 1u) & 15u) * 64u + lane];
            d2 = R[((dw + 2u) & 15u) * 64u + lane];
        }
        scons[lane] = 4u * dw;  // (issued after the reads: the feeder may now refill older chunks)
        const uint32_t b0 = __builtin_bswap32(d0), b1 = __builtin_bswap32(d1), b2 = __builtin_bswap32(d2);
        const uint32_t o = bp & 31u;
        return ((((uint64_t)b0) << 32 | b1) << o) | (uint32_t)((((uint64_t)b2) << o) >> 32);
    }
    // MB classes from the feeder's ring (the decoder wave issues no global loads:
    // a wait for one would also wait for its snapshot stores)
    DI uint32_t cls(uint32_t mbi)
    {
        const uint32_t q = mbi >> 4;
        if (q != cq) {
            for (uint32_t i = 0; cfill[lane] <= q; i++) {
                if (i > TKL_SPIN) {
                    tmo = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            cw = CR[(q & 3u) * 64u + lane];
            cq = q;
            ccons[lane] = q;
        }
        return (cw >> (2u * (mbi & 15u))) & 3u;
    }
    DI uint32_t tcx(uint32_t mbx) const { return TCX[mbx * 64u + lane]; }
    DI void set_tcx(uint32_t mbx, uint32_t v) { TCX[mbx * 64u + lane] = (uint16_t)v; }
    DI void snap(bool c, uint32_t mbi, uint32_t s0, uint32_t s1, uint32_t tl)
    {
        const zu4 v = {s0, s1, tl, 0u};
        bst128(v, sr, c ? sbase + mbi * 16u : ZW_OOB);
    }
};

}  // namespace

#ifndef ZW_TOK1_MK
#define ZW_TOK1_MK 16  // steps between MB phases (a lane at an MB's end idles until the next one; a power of 2: 8 / 16 / 32 measured 433 / 390 / 399 cycles a decision)
#endif
#ifndef ZW_TOK1_MBRUN
#define ZW_TOK1_MBRUN 8  // MBs one MB phase may start (skipped MBs need no decisions)
#endif
#ifndef ZW_TOKL_FSLEEP
#define ZW_TOKL_FSLEEP 32  // feeder pause between ring refills (64 cycles each)
#endif

// Stage 1.  One workgroup = a decoder wave (64 frames, lane l = frame
// blockIdx.x * 64 + l) and a feeder wave that streams each lane's partition
// bytes into an LDS ring.  probs: tokl::PROBS bytes per frame ([type][band]
// [ctx][node]); cls: ncw = (nmb + 15) / 16 dwords per frame; snaps: nmb
// uint4 per frame (written for the MBs that are not skipped); err1[f] = 2 when
// a bounded wait gave up, else 0.
extern "C" __global__ __launch_bounds__(128) void k_dec_tok1(const uint8_t* __restrict__ blob,
                                                            const ZwTokFrame* __restrict__ tf,
                                                            const uint8_t* __restrict__ probs,
                                                            const uint32_t* __restrict__ cls, uint8_t* snaps,
                                                            int* err1, int mbw, int mbh, int nframes)
{
    extern __shared__ uint32_t sm[];
    __shared__ uint32_t T1[TK1_T];  // (static: its reads fold the base into the offset)
    uint32_t* P = sm;
    uint32_t* SR = P + TK1_P;
    uint32_t* CR = SR + TK1_SR;
    uint32_t* SY = CR + TK1_CR;
    uint32_t* D1 = SY + TK1_SY;
    uint16_t* TCX = (uint16_t*)(D1 + TK1_D);
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int f = (int)blockIdx.x * 64 + lane;
    const bool act = f < nframes;
    const uint32_t nmb = (uint32_t)mbw * (uint32_t)mbh, ncw = (nmb + 15u) >> 4;
    for (int i = tid; i < TK1_T; i += 128) T1[i] = d_T1.e[i];
    for (int i = tid; i < 2 * (int)tok1::NDESC1; i += 128)
        tok1::desc1<64>((uint32_t)(i / (int)tok1::NDESC1), (uint32_t)(i % (int)tok1::NDESC1), D1 + 4 * i);
    for (int i = tid; i < TK1_SY; i += 128) SY[i] = 0u;
    for (int i = tid; i < (mbw + 1) * 32; i += 128) ((uint32_t*)TCX)[i] = 0u;
    {
        const uint4* pr = (const uint4*)(probs + (size_t)(act ? f : 0) * tokl::PROBS);
        uint8_t* P8 = (uint8_t*)P;  // entry i of lane l at byte i * 64 + l
#pragma unroll 11
        for (int q = wv; q < tokl::PROBS / 16; q += 2) {
            const uint4 v = act ? pr[q] : make_uint4(0, 0, 0, 0);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 16; j++) P8[(16 * q + j) * 64 + lane] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
        }
    }
    __syncthreads();
    volatile lds_u32* sfill = (volatile lds_u32*)SY;
    volatile lds_u32* scons = sfill + 64;
    volatile lds_u32* cfill = sfill + 128;
    volatile lds_u32* ccons = sfill + 192;
    volatile lds_u32* done = sfill + 256;
    if (wv == 1) {
        // feeder: lane l keeps frame l's stream ring (4 chunks of 16 bytes) and
        // class ring (4 words) full; stream bytes past the partition are 0
        const uint8_t* src = act ? blob + tf[f].off : blob;
        const uint32_t len = act ? tf[f].len : 0u, nch = (len + 15u) >> 4;
        const uint32_t* cl = cls + (size_t)(act ? f : 0) * ncw;
        uint32_t sf = 0, cf = 0;
        while (!*done) {
            const uint32_t sc = scons[lane], cc = ccons[lane];
            {
                const uint32_t c = cf < ncw ? cf : ncw - 1u;
                const uint32_t v = cl[c];  // (unconditional, clamped)
                if (act && cf < ncw && cf < cc + 4u) {
                    CR[(cf & 3u) * 64 + lane] = v;
                    cf++;
                }
            }
            uint4 s[2];
            uint32_t ns = 0;
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t c = sf + (uint32_t)u;
                const bool ok = act && c < (sc >> 4) + 4u;
                const uint4 v = ((const uint4*)src)[c < nch ? c : 0u];  // (unconditional, clamped: both in flight)
                s[u] = c < nch ? v : make_uint4(0, 0, 0, 0);
                ns += ok ? 1u : 0u;
            }
#pragma unroll
            for (int u = 0; u < 2; u++)
                if ((uint32_t)u < ns) {
                    const uint32_t b = ((sf + (uint32_t)u) & 3u) * 4u;
                    SR[(b + 0) * 64 + lane] = s[u].x;
                    SR[(b + 1) * 64 + lane] = s[u].y;
                    SR[(b + 2) * 64 + lane] = s[u].z;
                    SR[(b + 3) * 64 + lane] = s[u].w;
                }
            sf += ns;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // ring data before the fill counters
            sfill[lane] = sf;
            cfill[lane] = cf;
            __builtin_amdgcn_s_sleep(ZW_TOKL_FSLEEP);
        }
        return;
    }
    // decoder
    Tok1Dev m;
    m.P8 = (const uint8_t*)P;
    m.T1 = T1;
    m.D1 = D1;
    m.SR = SR;
    m.TCX = TCX;
    m.CR = CR;
    m.sfill = sfill;
    m.scons = scons;
    m.cfill = cfill;
    m.ccons = ccons;
    m.cq = 0xFFFFFFFFu;
    m.cw = 0;
    {
        const int f0 = (int)blockIdx.x * 64, nw = nframes - f0 < 64 ? nframes - f0 : 64;
        m.sr = brsrc(snaps + (size_t)f0 * nmb * 16u, (uint32_t)((size_t)nw * nmb * 16u));
        m.sbase = (uint32_t)lane * nmb * 16u;
    }
    m.lane = (uint32_t)lane;
    m.nmb = nmb;
    m.mbw = (uint32_t)mbw;
    m.tmo = 0;
    tok1::Lane1 L;
    tok1::init1(L, act);
#ifdef ZW_TOK_PROF
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    uint32_t ndec = 0, nstep = 0, n_mb = 0;
#endif
    // rounds of 8 steps: a top-up first (every live lane, whatever its phase:
    // then no lane makes more than 8 decisions between two top-ups), an MB phase
    // every ZW_TOK1_MK steps, the exit test once a round
    for (uint32_t rnd = 0;; rnd++) {
        if (L.k != tok1::K_DONE) tok1::topup1(L, m);
#pragma unroll
        for (int j = 0; j < 8; j++) {
#ifdef ZW_TOK_PROF
            ndec += L.k < tok1::K_MB;
#endif
            tok1::step1(L, m);  // (every lane: SINK keeps the waiting ones)
            if ((ZW_TOK1_MK <= 8 && j % ZW_TOK1_MK == ZW_TOK1_MK - 1) ||
                (ZW_TOK1_MK > 8 && j == 7 && (rnd % (ZW_TOK1_MK / 8)) == ZW_TOK1_MK / 8 - 1)) {
#ifdef ZW_TOK_PROF
                n_mb += __builtin_amdgcn_ballot_w64(L.k == tok1::K_MB) != 0;
#endif
#pragma unroll 1
                for (int r = 0; r < ZW_TOK1_MBRUN && L.k == tok1::K_MB; r++) tok1::mb1(L, m);
            }
        }
        if (m.tmo) L.k = tok1::K_DONE;
#ifdef ZW_TOK_PROF
        nstep += 8;
#endif
        if (__builtin_amdgcn_ballot_w64(L.k != tok1::K_DONE) == 0) break;
    }
    if (lane == 0) *done = 1u;
    if (act) err1[f] = m.tmo ? 2 : 0;
#ifdef ZW_TOK_PROF
    if (f == 0 || f == nframes - 1)
        printf("[k_dec_tok1] frame %d: %u decisions in %u steps, %llu cycles (%.1f per step), MB phases in %u steps\n",
               f, ndec, nstep, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start),
               (double)(__builtin_amdgcn_s_memtime() - t_start) / (double)nstep, n_mb);
#endif
}

namespace {

// Stage 2's memory: the frame's probabilities, TT and descriptors in LDS, the
// stream straight from HBM, the records through a buffer over the frame's
// record bytes (W = false: no stores, the replay only counts).
template <bool W>
struct Tok2Dev {
    static constexpr uint32_t U = 1;
    static constexpr uint32_t lane0 = 0;
    const uint8_t* P8;
    const uint32_t* TT;
    const uint32_t* DS;
    const uint32_t* src;  // the partition's dwords (16-aligned; zero-padded to 16 bytes)
    uint32_t ndw;         // its dwords up to the 16-byte padding
    __amdgpu_buffer_rsrc_t rr;

    DI void tt(uint32_t st, uint32_t& t0, uint32_t& t1) const
    {
        t0 = TT[2 * st];
        t1 = TT[2 * st + 1];
    }
    DI void desc(uint32_t i, uint32_t* d) const
    {
        const uint4 v = *(const uint4*)(DS + 4 * i);
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
    DI uint32_t prob_at(uint32_t a) const { return P8[a]; }
    DI uint64_t bits64(uint32_t bp) const
    {
        const uint32_t dw = bp >> 5;
        const uint32_t d0 = dw < ndw ? src[dw] : 0u, d1 = dw + 1u < ndw ? src[dw + 1u] : 0u,
                       d2 = dw + 2u < ndw ? src[dw + 2u] : 0u;
        const uint32_t b0 = __builtin_bswap32(d0), b1 = __builtin_bswap32(d1), b2 = __builtin_bswap32(d2);
        const uint32_t o = bp & 31u;
        return ((((uint64_t)b0) << 32 | b1) << o) | (uint32_t)((((uint64_t)b2) << o) >> 32);
    }
    uint32_t lim;  // the MB's record end: stores past it belong to the next MB (mb_end's note)
    DI void st16c(bool c, uint32_t off, uint32_t v)
    {
        if (W) __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rr, (int)(c && off < lim ? off : ZW_OOB), 0, 0);
    }
    DI void st128(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
    {
        if (W) {
            const zu4 v = {a, b, c, d};
            bst128(v, rr, off);
        }
    }
};

}  // namespace

// Stage 2: grid (ceil(nmb / 256), frames), lane = MB.  W = 0: sizes[f][i] = MB
// i's record bytes, err2[f] = 1 if the eof rule fails the frame (a decision
// starting past 8 len - 7 bits).  W = 1: the records at recs + fbase[f] +
// moff[f][i].  Frames whose stage 1 gave up (err1) get header-only zero records.
template <bool W>
__global__ __launch_bounds__(256) void k_dec_tok2(const uint8_t* __restrict__ blob, const ZwTokFrame* __restrict__ tf,
                                                  const uint8_t* __restrict__ probs, const uint8_t* __restrict__ modes,
                                                  const uint4* __restrict__ snaps, const int* __restrict__ err1,
                                                  uint32_t* sizes, int* err2, const uint32_t* __restrict__ moff,
                                                  const uint64_t* __restrict__ fbase, uint8_t* recs, int nmb)
{
    __shared__ uint32_t P[tokl::PROBS / 4], TT[2 * tokl::NST], DS[2 * 4 * tokl::NDESC];
    const int tid = (int)threadIdx.x, f = (int)blockIdx.y;
    for (int i = tid; i < tokl::PROBS / 4; i += 256) P[i] = ((const uint32_t*)(probs + (size_t)f * tokl::PROBS))[i];
    for (int i = tid; i < 2 * (int)tokl::NST; i += 256) TT[i] = d_TOKL_TT[i];
    for (int i = tid; i < 2 * tokl::NDESC; i += 256)
        tokl::desc((uint32_t)(i / tokl::NDESC), (uint32_t)(i % tokl::NDESC), DS + 4 * i);
    __syncthreads();
    const int i = (int)blockIdx.x * 256 + tid;
    if (i >= nmb) return;
    const size_t fi = (size_t)f * nmb + i;
    const uint4 mv = *(const uint4*)(modes + fi * ZW_TOK_MODE);
    const uint32_t mr[4] = {mv.x, mv.y, mv.z, mv.w};
    const bool skip = (mv.x >> 5) & 1u, e1 = err1[f] != 0;
    Tok2Dev<W> m;
    m.P8 = (const uint8_t*)P;
    m.TT = TT;
    m.DS = DS;
    const ZwTokFrame t = tf[f];
    m.src = (const uint32_t*)(blob + t.off);
    m.ndw = ((t.len + 15u) & ~15u) >> 2;
    uint32_t hb = 0;
    if (W) {
        const uint32_t* mo = moff + (size_t)f * (nmb + 1);
        m.rr = brsrc(recs + fbase[f], mo[nmb]);
        hb = mo[i];
        m.lim = mo[i + 1];
    }
    uint32_t size = ZW_DREC_HDR;
    if (e1 || skip) {
        const uint32_t z[4] = {0u, 0u, 0u, 0u};
        tokl::mb_skip(m, hb, e1 ? z : mr);
    } else {
        const uint4 s = snaps[fi];
        tokl::Lane L;
        tokl::from_snapshot(L, m, s.x, s.y, t.len);
        L.hb = hb;
        tokl::mb_begin(L, m, mr, s.z);
#pragma unroll 1
        for (uint32_t it = 0; L.phase == tokl::PH_DECIDE; it++) {
            if ((it & 7u) == 0) tokl::topup(L, m);
            tokl::step(L, m);
        }
        tokl::mb_end(L, m);
        size = L.hb - hb;
        if (!W && L.bad) err2[f] = 1;
    }
    if (!W) sizes[fi] = size;
}

// Per frame (one workgroup): moff[f][i] = exclusive prefix of sizes[f][.],
// moff[f][nmb] = the frame's record bytes; terr[f] = 2 (stage 1 gave up),
// 1 (ZW_EBITSTREAM) or 0.
extern "C" __global__ __launch_bounds__(1024) void k_dec_tok_scan(const uint32_t* __restrict__ sizes, uint32_t* moff,
                                                                 const int* __restrict__ err1,
                                                                 const int* __restrict__ err2, int* terr, int nmb)
{
    __shared__ uint32_t s[1024];
    const int tid = (int)threadIdx.x, f = (int)blockIdx.x;
    const int per = (nmb + 1023) / 1024, j0 = tid * per, j1 = j0 + per < nmb ? j0 + per : nmb;
    const uint32_t* sz = sizes + (size_t)f * nmb;
    uint32_t* mo = moff + (size_t)f * (nmb + 1);
    uint32_t sum = 0;
    for (int j = j0; j < j1; j++) sum += sz[j];
    s[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
        const uint32_t v = tid >= o ? s[tid - o] : 0u;
        __syncthreads();
        s[tid] += v;
        __syncthreads();
    }
    uint32_t run = s[tid] - sum;
    for (int j = j0; j < j1; j++) {
        mo[j] = run;
        run += sz[j];
    }
    if (tid == 1023) {
        mo[nmb] = s[1023];
        terr[f] = err1[f] ? 2 : (err2[f] ? 1 : 0);
    }
}

// One workgroup: fbase[f] = 256-B aligned exclusive prefix of the frames'
// record bytes, *total = the batch's span.
extern "C" __global__ __launch_bounds__(1024) void k_dec_tok_fbase(const uint32_t* __restrict__ moff, uint64_t* fbase,
                                                                  uint64_t* total, int nmb, int nframes)
{
    __shared__ uint64_t s[1024];
    const int tid = (int)threadIdx.x;
    const int per = (nframes + 1023) / 1024, j0 = tid * per, j1 = j0 + per < nframes ? j0 + per : nframes;
    auto span = [&](int j) -> uint64_t { return ((uint64_t)moff[(size_t)j * (nmb + 1) + nmb] + 255u) & ~(uint64_t)255; };
    uint64_t sum = 0;
    for (int j = j0; j < j1; j++) sum += span(j);
    s[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint64_t v = tid >= o ? s[tid - o] : 0u;
        __syncthreads();
        s[tid] += v;
        __syncthreads();
    }
    uint64_t run = s[tid] - sum;
    for (int j = j0; j < j1; j++) {
        fbase[j] = run;
        run += span(j);
    }
    if (tid == 1023) *total = s[1023];
}

extern "C" size_t zw_tok1_lds_bytes(int mbw) { return (size_t)(TK1_FIXED + TK1_T + mbw * 32) * 4; }  // (static + dynamic)

// Stage 1, then stage 2's count, the scans, and the total's copy to host_total
// (pinned), all on stream s.  Buffers as the kernels above describe them.
extern "C" hipError_t zwk_dec_tok_count(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                                        const uint8_t* modes, const uint32_t* cls, uint8_t* snaps, int* err1,
                                        uint32_t* sizes, int* err2, uint32_t* moff, uint64_t* fbase, int* terr,
                                        uint64_t* d_total, uint64_t* host_total, int mbw, int mbh, int n,
                                        hipEvent_t stage1_done)
{
    const size_t lds = zw_tok1_lds_bytes(mbw) - (size_t)TK1_T * 4;  // (the dynamic part)
    if (lds + (size_t)TK1_T * 4 > 160 * 1024) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_dec_tok1, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024 - TK1_T * 4);
        if (e != hipSuccess) return e;
        attr = true;
    }
    const int nmb = mbw * mbh;
    hipError_t e = hipMemsetAsync(err2, 0, (size_t)n * sizeof(int), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dec_tok1, dim3((n + 63) / 64), dim3(128), lds, s, blob, tf, probs, cls, snaps, err1, mbw, mbh,
                       n);
    if (stage1_done && (e = hipEventRecord(stage1_done, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_dec_tok2<false>, dim3((nmb + 255) / 256, n), dim3(256), 0, s, blob, tf, probs, modes,
                       (const uint4*)snaps, (const int*)err1, sizes, err2, (const uint32_t*)nullptr,
                       (const uint64_t*)nullptr, (uint8_t*)nullptr, nmb);
    hipLaunchKernelGGL(k_dec_tok_scan, dim3(n), dim3(1024), 0, s, (const uint32_t*)sizes, moff, (const int*)err1,
                       (const int*)err2, terr, nmb);
    hipLaunchKernelGGL(k_dec_tok_fbase, dim3(1), dim3(1024), 0, s, (const uint32_t*)moff, fbase, d_total, nmb, n);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(host_total, d_total, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
}

// Stage 2's record pass into recs (at least the total zwk_dec_tok_count reported).
extern "C" hipError_t zwk_dec_tok_write(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                                        const uint8_t* modes, const uint8_t* snaps, const int* err1,
                                        const uint32_t* moff, const uint64_t* fbase, uint8_t* recs, int nmb, int n)
{
    hipLaunchKernelGGL(k_dec_tok2<true>, dim3((nmb + 255) / 256, n), dim3(256), 0, s, blob, tf, probs, modes,
                       (const uint4*)snaps, err1, (uint32_t*)nullptr, (int*)nullptr, moff, fbase, recs, nmb);
    return hipGetLastError();
}
