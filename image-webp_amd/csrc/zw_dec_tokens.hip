// zw_dec_tokens.hip -- the VP8 token partition parsed on the device (gfx950),
// one frame per LANE (k_dec_tokl).
//
// read_coefficients (decoder/vp8.rs:872-1058) over the boolean decoder of
// bit_reader.rs:254-640.  A frame's token partition is one serial chain of
// binary decisions (each one's range and value depend on the one before), so a
// frame cannot be split; a batch parses its frames side by side.  The host
// keeps the frame header and the first partition's per-MB modes (ZW_TOK_MODE
// bytes per MB, a short chain); the records written here are byte-identical to
// the host parser's (zw_dec_host.cpp parse_mbs), and k_dec_recon reads them
// unchanged.
#include "zw_dev.h"

// ---------------------------------------------------------------------------
// Lane-parallel form (k_dec_tokl): one frame per LANE, 64 frames per wave.
//
// Every lane runs zw_tokl.h's state machine for its own frame: one decision per
// step, written branch-free (a branch any lane takes costs the whole wave, and
// some lane ends a token or a block at almost every step), the MB bookkeeping
// in an MB phase.  Round 4's form, one frame per wave on the scalar unit, ran
// ≈517 cycles per decision and held a wave per frame.  The decoder wave issues
// no global loads (its stores never have to be waited for); a second wave of the
// workgroup, the feeder, copies each lane's stream bytes and per-MB mode records
// from HBM into LDS rings ahead of use and publishes fill counters that the
// decoder lanes read (LDS operations of a CU complete in issue order; every
// spin is bounded and a lane that gives up reports a device error).
//
// LDS per workgroup (dwords): probabilities [264][64] (lane l's dword j at
// j * 64 + l: a lane-varying row index never makes two lanes of a group hit one
// bank), stream ring [16][64] (64 bytes per lane), mode ring [32 slots][4][64],
// sync words, the transition and descriptor tables, and the top contexts
// [mbw][64] u16.  ≈122 KB at 1080p: one workgroup per CU.  Record stores are
// raw buffer stores over the wave's 64 frame slots, with an out-of-range offset
// for a lane that stores nothing (no branch).
// ---------------------------------------------------------------------------
#include "zw_tokl.h"

namespace {

__constant__ uint32_t d_TOKL_TT[2 * tokl::NST] = ZW_TOKL_TT_INIT;

constexpr int TKL_P = 264 * 64, TKL_SR = 16 * 64, TKL_MRS = 32, TKL_MR = TKL_MRS * 4 * 64, TKL_SY = 4 * 64 + 4,
              TKL_TT = 2 * tokl::NST, TKL_DS = 2 * 4 * tokl::NDESC;
constexpr int TKL_FIXED = TKL_P + TKL_SR + TKL_MR + TKL_SY + TKL_TT + TKL_DS;  // dwords before the top contexts
constexpr uint32_t TKL_SPIN = 1u << 22;

typedef __attribute__((address_space(3))) uint32_t lds_u32;  // (a generic volatile pointer would become a flat access)

struct TokDev {
    static constexpr uint32_t U = 64;  // probability table [entry][lane] bytes
    uint32_t* P;
    const uint32_t* TT;
    const uint32_t* DS;
    const uint32_t* SR;
    const uint32_t* MR;
    uint16_t* TCX;
    volatile lds_u32* sfill;
    volatile lds_u32* mfill;
    volatile lds_u32* scons;
    volatile lds_u32* mcons;
    __amdgpu_buffer_rsrc_t rr;  // the wave's 64 record slots
    uint32_t rbase;             // this lane's slot in rr
    uint32_t* mo;
    uint32_t lane, lane0, nmb, mbw, tmo;

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
    DI uint32_t prob_at(uint32_t a) const { return ((const uint8_t*)P)[a]; }
    // 64 stream bits from bit bp on, MSB first (dwords hold 4 stream bytes, the
    // first in the low byte)
    DI uint64_t bits64(uint32_t bp)
    {
        const uint32_t dw = bp >> 5, need = ((4u * dw + 11u) >> 4) + 1u;
        for (uint32_t i = 0; sfill[lane] < need; i++) {
            if (i > TKL_SPIN) {
                tmo = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t d0 = SR[((dw) & 15u) * 64u + lane], d1 = SR[((dw + 1u) & 15u) * 64u + lane],
                       d2 = SR[((dw + 2u) & 15u) * 64u + lane];
        scons[lane] = 4u * dw;  // (issued after the reads: the feeder may now refill older chunks)
        const uint32_t b0 = __builtin_bswap32(d0), b1 = __builtin_bswap32(d1), b2 = __builtin_bswap32(d2);
        const uint32_t o = bp & 31u;
        return ((((uint64_t)b0) << 32 | b1) << o) | (uint32_t)((((uint64_t)b2) << o) >> 32);
    }
    DI void mode(uint32_t mbi, uint32_t* r)
    {
        for (uint32_t i = 0; mfill[lane] <= mbi; i++) {
            if (i > TKL_SPIN) {
                tmo = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t s = (mbi & (TKL_MRS - 1)) * 4u;
#pragma unroll
        for (int j = 0; j < 4; j++) r[j] = MR[(s + j) * 64u + lane];
        mcons[lane] = mbi + 1u;
    }
    DI uint32_t tcx(uint32_t mbx) const { return TCX[mbx * 64u + lane]; }
    DI void set_tcx(uint32_t mbx, uint32_t v) { TCX[mbx * 64u + lane] = (uint16_t)v; }
    DI void st16c(bool c, uint32_t off, uint32_t v)
    {
#ifndef ZW_TOKL_EXP_NOSTORE  // (timing experiment: no level / start stores, wrong records)
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rr, (int)(c ? rbase + off : ZW_OOB), 0, 0);
#endif
    }
    DI void st128(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
    {
        const zu4 v = {a, b, c, d};
        bst128(v, rr, rbase + off);
    }
    DI void st128u(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d) { st128(off, a, b, c, d); }
    DI void moff(uint32_t i, uint32_t v) { mo[i] = v; }
};

}  // namespace

#ifndef ZW_TOKL_TK
#define ZW_TOKL_TK 8  // steps between top-ups (one decision per step: <= 8 keeps >= 8 valid bits)
#endif
#ifndef ZW_TOKL_MK
#define ZW_TOKL_MK 1  // steps between MB phases
#endif
#ifndef ZW_TOKL_FSLEEP
#define ZW_TOKL_FSLEEP 32  // feeder pause between ring refills (64 cycles each; 2: +1.4 % launch time, the feeder
                           // wave's loads and VALU beside the decoder)
#endif
#ifndef ZW_TOKL_MBRUN
#define ZW_TOKL_MBRUN 8  // MBs one MB phase may start (skipped MBs need no decisions)
#endif

// One workgroup = a decoder wave (64 frames, lane l = frame blockIdx.x * 64 + l)
// and a feeder wave.  probs: tokl::PROBS bytes per frame in [type][band][ctx][node] order.  err[f]:
// 1 = the partition ran out (ZW_EBITSTREAM), 2 = a bounded wait gave up.
extern "C" __global__ __launch_bounds__(128) void k_dec_tokl(const uint8_t* __restrict__ blob,
                                                            const ZwTokFrame* __restrict__ tf,
                                                            const uint8_t* __restrict__ probs,
                                                            const uint8_t* __restrict__ modes, uint8_t* recs,
                                                            uint64_t slot, uint32_t* moff, int* err, int mbw, int mbh,
                                                            int nframes)
{
    extern __shared__ uint32_t sm[];
    uint32_t* P = sm;
    uint32_t* SR = P + TKL_P;
    uint32_t* MR = SR + TKL_SR;
    uint32_t* SY = MR + TKL_MR;
    uint32_t* TT = SY + TKL_SY;
    uint32_t* DS = TT + TKL_TT;
    uint16_t* TCX = (uint16_t*)(DS + TKL_DS);
    const int tid = (int)threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int f = (int)blockIdx.x * 64 + lane;
    const bool act = f < nframes;
    const uint32_t nmb = (uint32_t)mbw * (uint32_t)mbh;
    // tables, zeroed state, the lanes' probabilities (both waves)
    for (int i = tid; i < TKL_TT; i += 128) TT[i] = d_TOKL_TT[i];
    for (int i = tid; i < 2 * tokl::NDESC; i += 128) tokl::desc((uint32_t)(i / tokl::NDESC), (uint32_t)(i % tokl::NDESC), DS + 4 * i);
    for (int i = tid; i < TKL_SY; i += 128) SY[i] = 0u;
    for (int i = tid; i < mbw * 32; i += 128) ((uint32_t*)TCX)[i] = 0u;
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
    volatile lds_u32* mfill = sfill + 64;
    volatile lds_u32* scons = sfill + 128;
    volatile lds_u32* mcons = sfill + 192;
    volatile lds_u32* done = sfill + 256;
    if (wv == 1) {
        // feeder: lane l keeps frame l's stream ring (4 chunks of 16 bytes) and
        // mode ring (TKL_MRS MBs) full; stream bytes past the partition are 0
        const uint8_t* src = act ? blob + tf[f].off : blob;
        const uint32_t len = act ? tf[f].len : 0u, nch = (len + 15u) >> 4;
        const uint4* mrec = (const uint4*)(modes + (size_t)(act ? f : 0) * nmb * ZW_TOK_MODE);
        uint32_t sf = 0, mf = 0;
        while (!*done) {
            const uint32_t sc = scons[lane], mc = mcons[lane];
            uint4 s[2], m[8];
            uint32_t ns = 0, nm = 0;
            // every load unconditional at a clamped (valid) address, so the ten are in
            // flight together; the lanes keep what is theirs
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t c = sf + (uint32_t)u;
                const bool ok = act && c < (sc >> 4) + 4u;
                const uint4 v = ((const uint4*)src)[c < nch ? c : 0u];
                s[u] = c < nch ? v : make_uint4(0, 0, 0, 0);
                ns += ok ? 1u : 0u;
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t k = mf + (uint32_t)u;
                const bool ok = act && k < nmb && k < mc + (uint32_t)TKL_MRS;
                m[u] = mrec[k < nmb ? k : 0u];
                nm += ok ? 1u : 0u;
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
#pragma unroll
            for (int u = 0; u < 8; u++)
                if ((uint32_t)u < nm) {
                    const uint32_t b = ((mf + (uint32_t)u) & (TKL_MRS - 1)) * 4u;
                    MR[(b + 0) * 64 + lane] = m[u].x;
                    MR[(b + 1) * 64 + lane] = m[u].y;
                    MR[(b + 2) * 64 + lane] = m[u].z;
                    MR[(b + 3) * 64 + lane] = m[u].w;
                }
            sf += ns;
            mf += nm;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // ring data before the fill counters
            sfill[lane] = sf;
            mfill[lane] = mf;
            __builtin_amdgcn_s_sleep(ZW_TOKL_FSLEEP);
        }
        return;
    }
    // decoder
    TokDev m;
    m.P = P;
    m.TT = TT;
    m.DS = DS;
    m.SR = SR;
    m.MR = MR;
    m.TCX = TCX;
    m.sfill = sfill;
    m.mfill = mfill;
    m.scons = scons;
    m.mcons = mcons;
    {
        const int f0 = (int)blockIdx.x * 64, nw = nframes - f0 < 64 ? nframes - f0 : 64;
        m.rr = brsrc(recs + (size_t)f0 * slot, (uint32_t)(nw * slot));
        m.rbase = (uint32_t)(lane * slot);
    }
    m.mo = moff + (size_t)(act ? f : 0) * (nmb + 1);
    m.lane = m.lane0 = (uint32_t)lane;
    m.nmb = nmb;
    m.mbw = (uint32_t)mbw;
    m.tmo = 0;
    tokl::Lane L;
    tokl::init(L, act ? tf[f].len : 0u, act);
#ifdef ZW_TOK_PROF
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    uint32_t ndec = 0, nstep = 0;
#endif
#ifdef ZW_TOK_PROF
    uint64_t c_top = 0, c_step = 0, c_mb = 0, t_a, t_b;
    uint32_t n_mb = 0;
#define TKL_STAMP(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define TKL_STAMP(v)
#endif
    for (uint32_t step = 0;; step++) {
        // every live lane, whatever its phase: then no lane makes more than
        // ZW_TOKL_TK decisions between two top-ups (step 0 fills the windows)
        TKL_STAMP(t_a);
        if (step % ZW_TOKL_TK == 0 && L.phase != tokl::PH_DONE) tokl::topup(L, m);
        TKL_STAMP(t_b);
#ifdef ZW_TOK_PROF
        c_top += t_b - t_a;
#endif
        if (L.phase == tokl::PH_DECIDE) {
#ifdef ZW_TOK_PROF
            ndec++;
#endif
            tokl::step(L, m);
        }
        TKL_STAMP(t_a);
#ifdef ZW_TOK_PROF
        c_step += t_a - t_b;
#endif
        if (step % ZW_TOKL_MK == 0) {
#ifdef ZW_TOK_PROF
            n_mb += __builtin_amdgcn_ballot_w64(L.phase == tokl::PH_MB) != 0;
#endif
#pragma unroll 1
            for (int r = 0; r < ZW_TOKL_MBRUN && L.phase == tokl::PH_MB; r++) tokl::mb_phase(L, m);
        }
        TKL_STAMP(t_b);
#ifdef ZW_TOK_PROF
        c_mb += t_b - t_a;
#endif
        if (m.tmo) L.phase = tokl::PH_DONE;
#ifdef ZW_TOK_PROF
        nstep++;
#endif
        if (__builtin_amdgcn_ballot_w64(L.phase != tokl::PH_DONE) == 0) break;
    }
    if (lane == 0) *done = 1u;
    if (act) {
        if (L.bad || m.tmo) {
            // the frame stopped early: its MB and the rest get empty records at the
            // bytes used, so the reconstruction that still runs before the host
            // reads err stays inside the frame's records
            m.st128(L.hb, 0u, 0u, 0u, 0u);
            m.st128(L.hb + 16u, 0u, 0u, 0u, 0u);
            m.st128(L.hb + 32u, 0u, 0u, 0u, 0u);
            m.st128(L.hb + 48u, 0u, 0u, 0u, 0u);
            m.st128(L.hb + 64u, 0u, 0u, 0u, 0u);
            for (uint32_t j = L.mbi; j <= nmb; j++) m.mo[j] = L.hb;
        }
        err[f] = m.tmo ? 2 : (L.bad ? 1 : 0);
    }
#ifdef ZW_TOK_PROF
    if (f == 0 || f == nframes - 1)
        printf("[k_dec_tokl] frame %d: %u decisions in %u steps, %llu cycles (%.1f per step: top-up %.1f, step %.1f, "
               "MB phase %.1f in %u steps)\n",
               f, ndec, nstep, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start),
               (double)(__builtin_amdgcn_s_memtime() - t_start) / (double)nstep, (double)c_top / nstep,
               (double)c_step / nstep, (double)c_mb / nstep, n_mb);
#endif
}

extern "C" size_t zw_tokl_lds_bytes(int mbw) { return (size_t)(TKL_FIXED + mbw * 32) * 4; }

extern "C" hipError_t zwk_dec_tokl(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                                   const uint8_t* modes, uint8_t* recs, uint64_t slot, uint32_t* moff, int* err, int mbw,
                                   int mbh, int n)
{
    const size_t lds = zw_tokl_lds_bytes(mbw);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        const hipError_t e = hipFuncSetAttribute((const void*)k_dec_tokl, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 160 * 1024);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(k_dec_tokl, dim3((n + 63) / 64), dim3(128), lds, s, blob, tf, probs, modes, recs, slot, moff, err,
                       mbw, mbh, n);
    return hipGetLastError();
}
