// zw_stats_kernels.hip -- the pass-1 token statistics on the device (SURVEY.md
// 8(f) row 1: "stats pre-aggregation"), exact.
//
// The reference replays record_residual_stats (encoder/vp8.rs:1027) /
// record_coeffs (encoder/cost.rs:1297) over the pass-1 levels in raster order;
// every binary decision of every token updates one ProbaStats counter
// (cost.rs:1173-1255):  if s >= 0xfffe0000: s = ((s + 1) >> 1) & 0x7fff7fff;
// s += 0x10000 + bit   (upper half: decisions, lower half: ones).
//
// The halving makes a counter order-dependent only once it has seen 65 535
// decisions.  Three kernels per chunk of frames:
//   k_stats_flags  one thread per MB: the all-zero (skip) flag and the non-zero
//                  flags of its 25 blocks (eob > first), which alone fix every
//                  block's token context;
//   k_stats_hist   one workgroup per stripe of ZS_STRIPE MBs: every block's
//                  decisions in parallel into ZS_COPIES lane-private LDS copies
//                  of the counters (lane % ZS_COPIES), reduced to per-stripe
//                  (decisions, ones);
//   k_stats_final  one workgroup per frame: counters with <= 65 534 decisions are
//                  final, s = (n << 16) | ones; every other ("heavy") counter is
//                  replayed exactly, one wave per counter, in raster order:
//                  whole stripes are added while no halving can fall inside
//                  them, a stripe that can reach the threshold is walked 64 MBs
//                  at a time, then MB by MB, and the MB where a halving falls is
//                  walked decision by decision.
// Output per frame: s[4][8][3][11] as the host's zwh::Stats, plus the number of
// MBs that were not all-zero (the skip probability).
#include "zw_dev.h"

#define ZS_WG 1024
// Stripe of MBs per k_stats_hist workgroup and lane-private LDS copies of the
// counters: measured per 256 1080p frames (hist + final), 512 / 16 copies:
// 1.37 + 0.78 ms; 128 / 4: 1.06 + 0.29 ms (small stripes bound the MB walk of
// a heavy counter's exact replay to 128 MBs; few copies leave LDS for four
// workgroups per CU).
#ifndef ZS_STRIPE
#define ZS_STRIPE 128
#endif
#ifndef ZS_COPIES
#define ZS_COPIES 4
#endif
static_assert((ZS_STRIPE * 25 + ZS_COPIES - 1) / ZS_COPIES * 9 < 65536, "a packed 16:16 copy must not carry");
#ifndef ZS_HWG
#define ZS_HWG 512  // k_stats_hist workgroup size
#endif
#define ZS_NCTR (4 * 8 * 3 * 11)

typedef ZwStatsOut StatsOut;

__device__ __forceinline__ int zs_band(int n) { return n >= 16 ? 0 : (int)((0x7666666665463210ull >> (4 * n)) & 15); }

// eob (last nonzero zigzag position + 1) of a block's 16 zigzag levels
__device__ __forceinline__ int zs_eob(const int16_t* lv)
{
    const uint32_t* w = (const uint32_t*)lv;
    int e = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        const uint32_t v = w[q];
        if (v & 0xffffu) e = 2 * q + 1;
        if (v >> 16) e = 2 * q + 2;
    }
    return e;
}

// The decisions record_coeffs makes for one block, in order: fn(counter, bit).
// Counter index = ((type * 8 + band) * 3 + ctx) * 11 + node.  Quirk: skip_eob
// is never cleared once a zero token was seen (cost.rs:1325-1342).
template <class F>
__device__ __forceinline__ void zs_walk(const int16_t* lv, int eob, int t, int first, int ctx, F&& fn)
{
    auto C = [&](int band, int c, int node) { return ((t * 8 + band) * 3 + c) * 11 + node; };
    if (eob <= first) {
        fn(C(zs_band(first), ctx, 0), 0);
        return;
    }
    int skip_eob = 0;
    int n = first;
    for (; n < eob; n++) {
        const int band = zs_band(n);
        const int c = lv[n];
        int v = c < 0 ? -c : c;
        if (!skip_eob) fn(C(band, ctx, 0), 1);
        if (v == 0) {
            fn(C(band, ctx, 1), 0);
            skip_eob = 1;
            ctx = 0;
            continue;
        }
        fn(C(band, ctx, 1), 1);
        if (v == 1) {
            fn(C(band, ctx, 2), 0);
            ctx = 1;
        } else {
            fn(C(band, ctx, 2), 1);
            if (v > 67) v = 67;
            if (v <= 4) {
                fn(C(band, ctx, 3), 0);
                if (v == 2) {
                    fn(C(band, ctx, 4), 0);
                } else {
                    fn(C(band, ctx, 4), 1);
                    fn(C(band, ctx, 5), v == 4);
                }
            } else if (v <= 10) {
                fn(C(band, ctx, 3), 1);
                fn(C(band, ctx, 6), 0);
                fn(C(band, ctx, 7), v > 6);
            } else {
                fn(C(band, ctx, 3), 1);
                fn(C(band, ctx, 6), 1);
                if (v < 35) {
                    fn(C(band, ctx, 8), 0);
                    fn(C(band, ctx, 9), v >= 19);
                } else {
                    fn(C(band, ctx, 8), 1);
                    fn(C(band, ctx, 10), v >= 67);
                }
            }
            ctx = 2;
        }
    }
    if (n < 16) fn(C(zs_band(n), ctx, 0), 0);
}

// Per-MB flags in LDS: bits 0..15 Y non-zero, 16 Y2 non-zero, 17..24 U/V
// non-zero, 25 I4, 26 all-zero (skipped: no decisions, contexts cleared).
#define ZS_I4 (1u << 25)
#define ZS_SKIP (1u << 26)

// Token context of block b of MB mb (raster), from the neighbours' flags
// (record_residual_stats' left/top contexts; skipped MBs read as zero, and
// the Y2 context skips over I4 MBs, which neither set nor clear it).
template <class FL>
__device__ __forceinline__ int zs_ctx_f(FL&& flag, int mb, int mbx, int mby, int mbw, int b)
{
    auto nz = [&](int m, int bb) -> int { return (int)((flag(m) >> bb) & 1u); };
    int l = 0, t = 0;
    if (b < 16) {
        const int bx = b & 3, by = b >> 2;
        l = bx > 0 ? nz(mb, b - 1) : (mbx > 0 ? nz(mb - 1, b + 3) : 0);
        t = by > 0 ? nz(mb, b - 4) : (mby > 0 ? nz(mb - mbw, b + 12) : 0);
    } else if (b == 16) {
        for (int x = mbx - 1; x >= 0; x--)
            if (!(flag(mb - (mbx - x)) & ZS_I4)) {
                l = nz(mb - (mbx - x), 16);
                break;
            }
        for (int y = mby - 1; y >= 0; y--)
            if (!(flag(mb - (mby - y) * mbw) & ZS_I4)) {
                t = nz(mb - (mby - y) * mbw, 16);
                break;
            }
    } else {
        const int bb = (b - 17) & 3, bx = bb & 1, by = bb >> 1;
        l = bx > 0 ? nz(mb, b - 1) : (mbx > 0 ? nz(mb - 1, b + 1) : 0);
        t = by > 0 ? nz(mb, b - 2) : (mby > 0 ? nz(mb - mbw, b + 2) : 0);
    }
    return min(l + t, 2);
}
__device__ __forceinline__ int zs_ctx(const uint32_t* fl, int mb, int mbx, int mby, int mbw, int b)
{
    return zs_ctx_f([&](int m) { return fl[m]; }, mb, mbx, mby, mbw, b);
}

// Walk the decisions of MB mb's blocks of token type t (a counter's type), in
// record_residual_stats' order (Y2, Y 0..15, U 0..3, V 0..3).
template <class F>
__device__ __forceinline__ void zs_walk_mb(const ZwMbOut* M, const uint32_t* fl, int mb, int mbw, int t, F&& fn)
{
    const uint32_t f = fl[mb];
    if (f & ZS_SKIP) return;
    const int mbx = mb % mbw, mby = mb / mbw;
    const bool i4 = (f & ZS_I4) != 0;
    if (t == 1 && !i4) zs_walk(M->levels[16], zs_eob(M->levels[16]), 1, 0, zs_ctx(fl, mb, mbx, mby, mbw, 16), fn);
    if (t == (i4 ? 3 : 0))
        for (int b = 0; b < 16; b++)
            zs_walk(M->levels[b], zs_eob(M->levels[b]), t, i4 ? 0 : 1, zs_ctx(fl, mb, mbx, mby, mbw, b), fn);
    if (t == 2)
        for (int b = 17; b < 25; b++)
            zs_walk(M->levels[b], zs_eob(M->levels[b]), 2, 0, zs_ctx(fl, mb, mbx, mby, mbw, b), fn);
}

__device__ __forceinline__ void zs_rec(uint32_t& s, int bit)
{
    if (s >= 0xfffe0000u) s = ((s + 1) >> 1) & 0x7fff7fffu;
    s += 0x00010000u + (bit ? 1u : 0u);
}

// Per-MB flags (bits 0..24 non-zero blocks, ZS_I4, ZS_SKIP): 32 lanes per MB,
// lane b < 25 reads block b's 16 levels (the MB's record is read as one
// contiguous run across the lanes) and the half-wave ballot forms the mask.
extern "C" __global__ __launch_bounds__(256) void k_stats_flags(const ZwMbOut* __restrict__ mbs, int nmb,
                                                              uint32_t* __restrict__ fl)
{
    const int b = threadIdx.x & 31, f = blockIdx.y;
    const int mb = blockIdx.x * 8 + (threadIdx.x >> 5);
    const bool in = mb < nmb;
    const ZwMbOut& M = mbs[(size_t)f * nmb + (in ? mb : 0)];
    const bool i4 = M.luma_mode == 4;
    int nzb = 0;
    if (in && b < 25) {
        const int e = zs_eob(M.levels[b]);
        nzb = b < 16 ? e > (i4 ? 0 : 1) : (b == 16 ? (!i4 && e > 0) : e > 0);
    }
    const unsigned long long bal = __ballot(nzb);
    uint32_t m = (uint32_t)(bal >> (threadIdx.x & 32));
    // check_all_coeffs_zero on the pass-1 levels (mb_all_zero_p1)
    if (m == 0) m = ZS_SKIP;
    if (in && b == 0) fl[(size_t)f * nmb + mb] = m | (i4 ? ZS_I4 : 0u);
}

// Per-stripe (decisions, ones) of every counter.  Copy j of the counters takes
// the items it = j (mod ZS_COPIES) of the stripe: <= ceil(ZS_STRIPE * 25 / ZS_COPIES) blocks,
// each adding <= 9 decisions to one counter (band 6 spans 9 positions), so the
// packed 16:16 copy cannot carry (14 400 < 65 536 even at 8 copies).
// The stripe's flags and the MB row above it are staged in LDS first, so a
// block's context costs no dependent global load, and each block's levels are
// loaded one item ahead of its walk.
#define ZS_FL_MAX (ZS_STRIPE + 1024)  // staged flags: the stripe + up to 1024 MBs of the row above
extern "C" __global__ __launch_bounds__(ZS_HWG) void k_stats_hist(const ZwMbOut* __restrict__ mbs,
                                                                const uint32_t* __restrict__ flags, int mbw, int mbh,
                                                                uint2* __restrict__ part)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cp = (uint32_t*)smem;  // [ZS_COPIES][ZS_NCTR] (decisions << 16) | ones
    uint32_t* sfl = cp + ZS_COPIES * ZS_NCTR;  // [ZS_FL_MAX] flags of MBs lo .. mb1 - 1
    const int st = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, nst = gridDim.x;
    const int nmb = mbw * mbh;
    const ZwMbOut* F = mbs + (size_t)f * nmb;
    const uint32_t* fl = flags + (size_t)f * nmb;
    const int mb0 = st * ZS_STRIPE, mb1 = min(nmb, mb0 + ZS_STRIPE);
    const int lo = max(0, mb0 - min(mbw, 1024));
    for (int i = tid; i < ZS_COPIES * ZS_NCTR; i += ZS_HWG) cp[i] = 0;
    for (int m = lo + tid; m < mb1; m += ZS_HWG) sfl[m - lo] = fl[m];
    __syncthreads();
    auto flag = [&](int m) -> uint32_t { return m >= lo ? sfl[m - lo] : fl[m]; };
    uint32_t* my = cp + (tid & (ZS_COPIES - 1)) * ZS_NCTR;
    const int nit = (mb1 - mb0) * 25;
    // (ZwMbOut records are 4-byte aligned: the levels are read as words)
    struct Lv {
        uint32_t w[8];
    };
    auto lv_of = [&](int it) {
        Lv r;
        const uint32_t* p = (const uint32_t*)F[mb0 + it / 25].levels[it % 25];
#pragma unroll
        for (int k = 0; k < 8; k++) r.w[k] = p[k];
        return r;
    };
    Lv nx;
    if (tid < nit) nx = lv_of(tid);
    for (int it = tid; it < nit; it += ZS_HWG) {
        const Lv cur = nx;
        if (it + ZS_HWG < nit) nx = lv_of(it + ZS_HWG);
        const int mb = mb0 + it / 25, b = it % 25;
        const uint32_t fm = sfl[mb - lo];
        if (fm & ZS_SKIP) continue;
        const bool i4 = (fm & ZS_I4) != 0;
        if (b == 16 && i4) continue;
        const int t = b < 16 ? (i4 ? 3 : 0) : (b == 16 ? 1 : 2);
        const int first = b < 16 && !i4 ? 1 : 0;
        const int ctx = zs_ctx_f(flag, mb, mb % mbw, mb / mbw, mbw, b);
        int16_t lv[16];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            lv[2 * k] = (int16_t)(cur.w[k] & 0xffffu);
            lv[2 * k + 1] = (int16_t)(cur.w[k] >> 16);
        }
        zs_walk(lv, zs_eob(lv), t, first, ctx, [&](int c, int bit) { atomicAdd(&my[c], 0x10000u + (bit ? 1u : 0u)); });
    }
    __syncthreads();
    for (int c = tid; c < ZS_NCTR; c += ZS_HWG) {
        uint32_t n = 0, o = 0;
#pragma unroll 8
        for (int j = 0; j < ZS_COPIES; j++) {
            const uint32_t v = cp[j * ZS_NCTR + c];
            n += v >> 16;
            o += v & 0xffffu;
        }
        part[((size_t)f * nst + st) * ZS_NCTR + c] = make_uint2(n, o);
    }
}

extern "C" __global__ __launch_bounds__(ZS_WG) void k_stats_final(const ZwMbOut* __restrict__ mbs,
                                                                 const uint32_t* __restrict__ flags, int mbw, int mbh,
                                                                 const uint2* __restrict__ part, int nst, int fl_lds,
                                                                 StatsOut* __restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int* heavy = (int*)smem;        // [ZS_NCTR] list of heavy counters
    int* nheavy = heavy + ZS_NCTR;  // [2]: heavy count, non-zero MBs
    uint32_t* fll = (uint32_t*)(nheavy + 2);  // [nmb] flags copy when fl_lds
    const int f = blockIdx.x, tid = threadIdx.x;
    const int nmb = mbw * mbh;
    const ZwMbOut* F = mbs + (size_t)f * nmb;
    const uint2* P = part + (size_t)f * nst * ZS_NCTR;
    if (tid < 2) nheavy[tid] = 0;
    __syncthreads();
    int nz = 0;
    for (int mb = tid; mb < nmb; mb += ZS_WG) {
        const uint32_t m = flags[(size_t)f * nmb + mb];
        if (fl_lds) fll[mb] = m;
        nz += (m & ZS_SKIP) ? 0 : 1;
    }
    if (nz) atomicAdd(&nheavy[1], nz);
    const uint32_t* fl = fl_lds ? fll : flags + (size_t)f * nmb;
    // light counters are final; heavy ones are listed
    for (int c = tid; c < ZS_NCTR; c += ZS_WG) {
        uint32_t n = 0, o = 0;
        for (int st = 0; st < nst; st++) {
            const uint2 v = P[st * ZS_NCTR + c];
            n += v.x;
            o += v.y;
        }
        if (n <= 0xfffeu) {
            out[f].s[c] = (n << 16) | o;
        } else {
            const int k = atomicAdd(&nheavy[0], 1);
            heavy[k] = c;
        }
    }
    __syncthreads();
    // exact replay of the heavy counters, one wave each
    const int wv = tid >> 6, lane = tid & 63, nh = nheavy[0];
    for (int k = wv; k < nh; k += ZS_WG / 64) {
        const int c = heavy[k], ct = c / (8 * 3 * 11);
        uint32_t s = 0;  // the counter, exactly as ProbaStats holds it
        for (int st = 0; st < nst; st++) {
            const uint2 v = P[st * ZS_NCTR + c];
            if ((s >> 16) + v.x <= 0xfffeu) {  // no decision of this stripe can see s >= 0xfffe0000
                s += (v.x << 16) + v.y;
                continue;
            }
            const int mb1 = min(nmb, (st + 1) * ZS_STRIPE);
            for (int base = st * ZS_STRIPE; base < mb1; base += 64) {
                const int mb = base + lane;
                uint32_t t = 0, o = 0;
                if (mb < mb1)
                    zs_walk_mb(F + mb, fl, mb, mbw, ct, [&](int cc, int bit) {
                        if (cc == c) {
                            t++;
                            o += bit ? 1u : 0u;
                        }
                    });
                uint32_t tsum = t;
#pragma unroll
                for (int o2 = 32; o2 >= 1; o2 >>= 1) tsum += __shfl_xor(tsum, o2);
                if ((s >> 16) + tsum <= 0xfffeu) {
                    uint32_t osum = o;
#pragma unroll
                    for (int o2 = 32; o2 >= 1; o2 >>= 1) osum += __shfl_xor(osum, o2);
                    s += (tsum << 16) + osum;
                } else {
                    for (int i = 0; i < 64 && base + i < mb1; i++) {  // MB by MB (uniform loop)
                        const uint32_t ti = (uint32_t)__shfl((int)t, i), oi = (uint32_t)__shfl((int)o, i);
                        if ((s >> 16) + ti <= 0xfffeu) {
                            s += (ti << 16) + oi;
                        } else {  // a halving falls inside this MB: decision by decision
                            uint32_t sl = s;
                            if (lane == 0)
                                zs_walk_mb(F + base + i, fl, base + i, mbw, ct, [&](int cc, int bit) {
                                    if (cc == c) zs_rec(sl, bit);
                                });
                            s = (uint32_t)__shfl((int)sl, 0);
                        }
                    }
                }
            }
        }
        if (lane == 0) out[f].s[c] = s;
    }
    if (tid == 0) {
        out[f].nonzero_mbs = (uint32_t)nheavy[1];
        out[f].total_mbs = (uint32_t)nmb;
    }
}

static int zs_stripes(int nmb) { return (nmb + ZS_STRIPE - 1) / ZS_STRIPE; }

// Device scratch for zwk_stats: flags [nframes][nmb] + stripe partials.  Linear
// in nframes (the caller carves per-chunk regions at scratch_bytes(nmb, f0)).
static size_t zs_flag_bytes(int nmb) { return ((size_t)nmb * 4 + 7) & ~(size_t)7; }
extern "C" size_t zw_stats_scratch_bytes(int nmb, int nframes)
{
    return (size_t)nframes * (zs_flag_bytes(nmb) + (size_t)zs_stripes(nmb) * ZS_NCTR * sizeof(uint2));
}

extern "C" hipError_t zwk_stats(hipStream_t s, const ZwMbOut* mbs, int mbw, int mbh, void* scratch, void* out,
                                int nframes)
{
    static const bool attr = []() {
        (void)hipFuncSetAttribute((const void*)k_stats_hist, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_stats_final, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        return true;
    }();
    (void)attr;
    const int nmb = mbw * mbh, nst = zs_stripes(nmb);
    if (nmb <= 0 || nframes <= 0) return hipErrorInvalidValue;
    uint32_t* fl = (uint32_t*)scratch;
    uint2* part = (uint2*)((uint8_t*)scratch + (size_t)nframes * zs_flag_bytes(nmb));
    hipLaunchKernelGGL(k_stats_flags, dim3((nmb + 7) / 8, nframes), dim3(256), 0, s, mbs, nmb, fl);
    hipLaunchKernelGGL(k_stats_hist, dim3(nst, nframes), dim3(ZS_HWG), (size_t)(ZS_COPIES * ZS_NCTR + ZS_FL_MAX) * 4, s,
                       mbs, fl, mbw, mbh, part);
    const size_t lds0 = ZS_NCTR * 4 + 8;
    const int fl_lds = lds0 + (size_t)nmb * 4 <= 160 * 1024;
    hipLaunchKernelGGL(k_stats_final, dim3(nframes), dim3(ZS_WG), lds0 + (fl_lds ? (size_t)nmb * 4 : 0), s, mbs, fl,
                       mbw, mbh, part, nst, fl_lds, (StatsOut*)out);
    return hipGetLastError();
}
