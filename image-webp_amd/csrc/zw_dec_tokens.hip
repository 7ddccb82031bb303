// zw_dec_tokens.hip -- the VP8 token partition parsed on the device (gfx950).
//
// read_coefficients (decoder/vp8.rs:872-1058) over the boolean decoder of
// bit_reader.rs:254-640.  A frame's token partition is one serial chain of
// binary decisions (each one's range and value depend on the one before), so a
// frame cannot be split; a batch parses its frames side by side, one wave per
// frame.  All control state is wave-uniform, so it lives in scalar registers
// and branches on the scalar unit; the lanes hold the current block's levels
// (lane n = zigzag position n) and copy each MB's packed
// record (zw_common.h ZW_DREC_*) out in one pass.  The records are
// byte-identical to the host parser's (zw_dec_host.cpp parse_mbs), and
// k_dec_recon reads them unchanged.  The host keeps the frame header and the
// first partition's per-MB modes (ZW_TOK_MODE bytes per MB, a short chain).
#include "zw_dev.h"

namespace {

DI uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// BitReader (bit_reader.rs; zw_dec_host.cpp BitReader) with the same loads:
// 7 bytes while at least 7 remain, then one byte at a time, then one zero byte
// and eof.  The 16 bytes holding the next 7-byte load are fetched into LDS by
// an LDS-DMA load as soon as the previous load is consumed (no register
// destination, so nothing on the decision chain waits for it until the next
// load; two slots alternate so a read never meets the DMA writing).
struct TokBD {
#ifdef ZW_TOK_PROF
    uint32_t ndec, nload;  // profiling build: decisions and 7-byte loads
#endif
    const uint8_t* p;
    uint64_t value;
    uint32_t range, pos, len, slot;
    int bits;
    bool eof;
};

DI void tok_fetch(TokBD& b, uint8_t* sbuf)
{
    if ((threadIdx.x & 63) == 0)
        __builtin_amdgcn_global_load_lds((const void*)(b.p + (b.pos & ~3u)), (void*)(sbuf + 16 * b.slot), 16, 0, 0);
}

DI void tok_load(TokBD& b, uint8_t* sbuf)
{
    const uint32_t rem = b.len - b.pos;
    if (rem >= 7) {
#ifdef ZW_TOK_PROF
        b.nload++;
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA fetch has landed
        const uint4 w = *(const uint4*)(sbuf + 16 * b.slot);
        const uint32_t o = b.pos & 3u;
        const uint64_t lo = ((uint64_t)rfl(w.y) << 32) | rfl(w.x);
        const uint64_t hi = ((uint64_t)rfl(w.w) << 32) | rfl(w.z);
        const uint64_t x = o ? (lo >> (8 * o)) | (hi << (64 - 8 * o)) : lo;  // bytes pos..pos+7, first in the low byte
        b.value = (__builtin_bswap64(x) >> 8) | (b.value << 56);
        b.bits += 56;
        b.pos += 7;
        b.slot ^= 1u;
        tok_fetch(b, sbuf);
    } else if (rem > 0) {
        const uint32_t w = rfl(*(const uint32_t*)(b.p + (b.pos & ~3u)));
        b.value = (uint64_t)((w >> (8 * (b.pos & 3u))) & 255u) | (b.value << 8);
        b.bits += 8;
        b.pos++;
    } else {
        // past the end: the reference shifts in one zero byte and sets eof, and
        // read_coefficients then fails the frame (vp8.rs; parse_mbs returns
        // ZW_EBITSTREAM) -- the device flags the frame the same way
        b.eof = true;
        b.value <<= 8;
        b.bits += 8;
    }
}

DI void tok_init(TokBD& b, const uint8_t* p, uint32_t len, uint8_t* sbuf)
{
    b.p = p;  // (the blob has 16 readable bytes past every partition)
    b.len = len;
    b.pos = 0;
    b.value = 0;
    b.range = 254;
    b.bits = -8;
    b.eof = false;
    b.slot = 0;
#ifdef ZW_TOK_PROF
    b.ndec = b.nload = 0;
#endif
    tok_fetch(b, sbuf);
    tok_load(b, sbuf);
}

// read_bool: split = range * prob >> 8 on range - 1 (bit_reader.rs), the
// update by selects (no branch on the decoded bit)
DI int tok_bit(TokBD& b, uint32_t prob, uint8_t* sbuf)
{
    if (b.bits < 0) tok_load(b, sbuf);
#ifdef ZW_TOK_PROF
    b.ndec++;
#endif
    const uint32_t split = (b.range * prob) >> 8;
    const uint32_t v = (uint32_t)(b.value >> b.bits);
    const bool bit = v > split;
    const uint32_t nr = bit ? b.range - split : split + 1;
    b.value = bit ? b.value - ((uint64_t)(split + 1) << b.bits) : b.value;
    const int shift = __builtin_clz(nr) - 24;
    b.bits -= shift;
    b.range = (nr << shift) - 1;
    return bit ? 1 : 0;
}

// The frame's coefficient probabilities live in registers: per block type t,
// VGPR A holds the rows of bands 0..6 (row (band, ctx) = dwords 0..2 at lanes
// (3 band + ctx) * 3 ..), VGPR B the rows of band 7 (lanes 3 ctx ..); a row is
// read with three v_readlane (no memory access on the decision chain).
struct TokRow {
    uint32_t r0, r1, r2;
};
DI uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
#ifdef ZW_TOK_SMEM
// (experiment: the rows as scalar loads from the frame's table in memory, A = the type's first register index)
DI TokRow prow_m(const uint8_t* __restrict__ Pf, uint32_t A, int n, int ctx)
{
    const uint32_t k = A + (n == 15 ? 1u : 0u);
    const int l = n < 15 ? (band_of(n) * 3 + ctx) * 3 : ctx * 3;
    const uint4 w = *(const uint4*)(Pf + (64 * k + l) * 4);
    TokRow r;
    r.r0 = w.x;
    r.r1 = w.y;
    r.r2 = w.z;
    return r;
}
#define prow(A, B, n, ctx) prow_m(Pf, A, n, ctx)
#else
DI TokRow prow(uint32_t A, uint32_t B, int n, int ctx)
{
    TokRow r;
    if (n < 15) {
        const int l = (band_of(n) * 3 + ctx) * 3;
        r.r0 = rdl(A, l);
        r.r1 = rdl(A, l + 1);
        r.r2 = rdl(A, l + 2);
    } else {
        const int l = ctx * 3;
        r.r0 = rdl(B, l);
        r.r1 = rdl(B, l + 1);
        r.r2 = rdl(B, l + 2);
    }
    return r;
}
#endif
// Byte k of a probability row (k constant at every call site).
DI uint32_t pb(const TokRow& r, int k)
{
    const uint32_t w = k < 4 ? r.r0 : (k < 8 ? r.r1 : r.r2);
    return (w >> (8 * (k & 3))) & 255u;
}

// One block's tokens (read_coefficients vp8.rs:872-1058; zw_dec_host.cpp
// read_levels_into): lane n of lvv gets the level at zigzag position n
// (positions < first and the zeros stay 0); eob = last nonzero position + 1.
// Returns the block's non-zero flag (n > first at the end of block; a zero run
// to position 16 counts as non-zero, as in the reference).
DI int tok_block(TokBD& b, uint8_t* sbuf, uint32_t A, uint32_t B, int first, int ctx, int& lvv, int& eob
#ifdef ZW_TOK_SMEM
                 , const uint8_t* __restrict__ Pf
#endif
)
{
    int n = first;
    eob = 0;
    lvv = 0;
    TokRow row = prow(A, B, n, ctx);
    for (;;) {
        if (!tok_bit(b, pb(row, 0), sbuf)) break;  // end of block
        while (!tok_bit(b, pb(row, 1), sbuf)) {    // DCT_0
            if (++n == 16) return 1;
            row = prow(A, B, n, 0);
        }
        int v, nctx = 2;
        if (!tok_bit(b, pb(row, 2), sbuf)) {
            v = 1;
            nctx = 1;
        } else if (!tok_bit(b, pb(row, 3), sbuf)) {
            if (!tok_bit(b, pb(row, 4), sbuf)) v = 2;
            else v = 3 + tok_bit(b, pb(row, 5), sbuf);
        } else if (!tok_bit(b, pb(row, 6), sbuf)) {
            if (!tok_bit(b, pb(row, 7), sbuf)) {
                v = 5 + tok_bit(b, 159, sbuf);
            } else {
                v = 7 + 2 * tok_bit(b, 165, sbuf);
                v += tok_bit(b, 145, sbuf);
            }
        } else {
            const int b1 = tok_bit(b, pb(row, 8), sbuf);
            const int b0 = tok_bit(b, b1 ? pb(row, 10) : pb(row, 9), sbuf);
            const int cat = 2 * b1 + b0;  // DCT_CAT3..6: 3, 4, 5, 11 extra bits
            // PROB_DCT_CAT[2 + cat] as byte immediates (no memory load on the chain)
            const uint64_t lo = cat == 0 ? 0x8c94adull : (cat == 1 ? 0x878c9bb0ull : (cat == 2 ? 0x82868d9db4ull : 0x8c99b1c4e6f3fefeull));
            const int nb = cat == 3 ? 11 : 3 + cat;
            int extra = 0;
            for (int k = 0; k < nb; k++) {
                const uint32_t p = k < 8 ? (uint32_t)(lo >> (8 * k)) & 255u : (0x818285u >> (8 * (k - 8))) & 255u;
                extra = extra + extra + tok_bit(b, p, sbuf);
            }
            v = 3 + (8 << cat) + extra;
        }
        const int s = tok_bit(b, 128, sbuf);
        lvv = (int)(threadIdx.x & 63) == n ? (s ? -v : v) : lvv;
        eob = ++n;
        if (n == 16) break;
        row = prow(A, B, n, nctx);
    }
    return n > first;
}

}  // namespace

// One wave per frame.  tf[f]: the frame's token partition in blob; probs:
// ZW_TOK_PROBS bytes per frame; modes: ZW_TOK_MODE bytes per MB per frame.
// Out: frame f's records at recs + f * slot, their offsets at moff + f * (nmb
// + 1) (moff[nmb] = the used bytes), err[f] = 1 when the partition ran out
// (the host then fails the call with ZW_EBITSTREAM, as parse_mbs does).
#ifndef ZW_TOK_WAVES
#define ZW_TOK_WAVES 1  // frames (waves) per workgroup: more confine the launch to fewer CUs
#endif
extern "C" __global__ __launch_bounds__(64 * ZW_TOK_WAVES) void k_dec_tokens(const uint8_t* __restrict__ blob,
                                                              const ZwTokFrame* __restrict__ tf,
                                                              const uint8_t* __restrict__ probs,
                                                              const uint8_t* __restrict__ modes, uint8_t* recs,
                                                              uint64_t slot, uint32_t* moff, int* err, int mbw, int mbh,
                                                              int nframes)
{
    __shared__ uint16_t tcx_all[ZW_TOK_WAVES][(ZW_MAX_W + 15) / 16];  // 9-bit top contexts per MB column (Y2, Y 1-4, U 5-6, V 7-8)
    __shared__ __attribute__((aligned(16))) uint8_t rec_all[ZW_TOK_WAVES][ZW_DREC_MAX + 16];
    __shared__ __attribute__((aligned(16))) uint8_t sbuf_all[ZW_TOK_WAVES][32];  // the stream's two 16-byte fetch slots
    const int wv = (int)(threadIdx.x >> 6), f = blockIdx.x * ZW_TOK_WAVES + wv, lane = (int)(threadIdx.x & 63);
    if (f >= nframes) return;  // (no workgroup barrier below: every wave runs alone)
    uint16_t* tcx = tcx_all[wv];
    uint8_t* rec = rec_all[wv];
    uint8_t* sbuf = sbuf_all[wv];
    const size_t nmb = (size_t)mbw * mbh;
    for (int i = lane; i < mbw; i += 64) tcx[i] = 0;
    // the frame's probabilities: 8 VGPRs (type t: A = P[2 t], B = P[2 t + 1]; ZW_TOK_PROBS layout)
    uint32_t P[8];
#pragma unroll
    for (int k = 0; k < 8; k++) P[k] = ((const uint32_t*)(probs + (size_t)f * ZW_TOK_PROBS))[k * 64 + lane];
    TokBD b;
#ifdef ZW_TOK_PROF
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
    tok_init(b, blob + tf[f].off, tf[f].len, sbuf);
    const uint4* __restrict__ M = (const uint4*)(modes + (size_t)f * nmb * ZW_TOK_MODE);
    const __amdgpu_buffer_rsrc_t ro = brsrc(recs + (size_t)f * slot, (uint32_t)slot);
    const __amdgpu_buffer_rsrc_t rm = brsrc(moff + (size_t)f * (nmb + 1), (uint32_t)(nmb + 1) * 4u);
    int16_t* lv = (int16_t*)(rec + ZW_DREC_HDR);
    uint32_t used = 0;
    // read_levels_into fails a frame when a block read ends with eof set (an
    // empty partition is fine while every MB is skipped)
    bool bad = false;
    uint32_t mdone = 0;  // MBs whose offset is written
    wsync();
    for (int mby = 0; mby < mbh && !bad; mby++) {
        uint32_t L = 0;  // left contexts, the same 9 bits
        for (int mbx = 0; mbx < mbw; mbx++) {
            const size_t i = (size_t)mby * mbw + mbx;
            const uint4 mr = M[i];
            const int lm = (int)(mr.x & 7u), skip = (int)((mr.x >> 5) & 1u);
            uint32_t T = rfl(tcx[mbx]);
            bst32(used, rm, lane == 0 ? (uint32_t)i * 4u : ZW_OOB);
            mdone = (uint32_t)i + 1u;
            if (skip) {
                // header only: the modes, no levels (every start 0)
                if (lm != 4) {
                    T &= ~1u;
                    L &= ~1u;
                }
                T &= 1u;
                L &= 1u;
                const zu4 h = {mr.x, 0u, mr.z, mr.w}, z = {0u, 0u, 0u, 0u};
                bst128(lane == 0 ? h : z, ro, lane < 5 ? used + 16u * (uint32_t)lane : ZW_OOB);
                used += ZW_DREC_HDR;
            } else {
                uint32_t nzm = 0;
                int nlv = 0, stv = 0, y2v = 0, y2eob = 0, lvv, eob;
                const uint32_t YA = lm != 4 ? P[0] : P[6], YB = lm != 4 ? P[1] : P[7];  // type 0 (after Y2) or 3 (I4)
                auto put = [&](int blk) {  // the block's levels after the previous blocks'
                    stv = lane == blk ? nlv : stv;
                    if (lane < eob) lv[nlv + lane] = (int16_t)lvv;
                    nlv += eob;
                };
                // the MB's blocks in the reference's order, through one call site (one copy
                // of the token walk in the code): k = 0 Y2 (I16 MBs only), 1..16 Y, 17..20 U,
                // 21..24 V; tb / lb = the block's bit in the top / left context words
#pragma unroll 1
                for (int k = lm != 4 ? 0 : 1; k < 25; k++) {
                    const int q = k - 17, pl = q >> 2;
                    const int tb = k == 0 ? 0 : (k <= 16 ? ((k - 1) & 3) + 1 : (q & 1) + 5 + 2 * pl);
                    const int lb = k == 0 ? 0 : (k <= 16 ? ((k - 1) >> 2) + 1 : ((q >> 1) & 1) + 5 + 2 * pl);
#ifdef ZW_TOK_SMEM
                    const uint32_t A = k == 0 ? 2u : (k <= 16 ? (lm != 4 ? 0u : 6u) : 4u), B = 0;
#else
                    const uint32_t A = k == 0 ? P[2] : (k <= 16 ? YA : P[4]), B = k == 0 ? P[3] : (k <= 16 ? YB : P[5]);
#endif
                    const int first = k >= 1 && k <= 16 && lm != 4 ? 1 : 0;
                    const int ctx = (int)((T >> tb) & 1u) + (int)((L >> lb) & 1u);
                    const int nz = tok_block(b, sbuf, A, B, first, ctx, lvv, eob
#ifdef ZW_TOK_SMEM
                                             , probs + (size_t)f * ZW_TOK_PROBS
#endif
                    );
                    T = (T & ~(1u << tb)) | ((uint32_t)nz << tb);
                    L = (L & ~(1u << lb)) | ((uint32_t)nz << lb);
                    bad = bad || b.eof;
                    if (k == 0) {
                        y2v = lvv;
                        y2eob = eob;
                    } else {
                        put(k - 1);
                        nzm |= (uint32_t)nz << (k - 1);
                    }
                }
                lvv = y2v;  // Y2 (parsed first) goes last
                eob = y2eob;
                put(24);
                stv = lane == 25 ? nlv : stv;
                // header dwords: modes, nzm, I4 modes, the 26 level starts as halfword pairs, pad
                const int s0 = __shfl(stv, 2 * (lane - 4)), s1 = __shfl(stv, 2 * (lane - 4) + 1);
                uint32_t hd = (uint32_t)(s0 & 0xffff) | ((uint32_t)s1 << 16);
                hd = lane == 0 ? mr.x : (lane == 1 ? nzm : (lane == 2 ? mr.z : (lane == 3 ? mr.w : hd)));
                if (lane < ZW_DREC_HDR / 4) ((uint32_t*)rec)[lane] = lane < 17 ? hd : 0u;
                const uint32_t bytes = ZW_DREC_HDR + 2u * (uint32_t)nlv, padded = (bytes + 15u) & ~15u;
                if (lane < 8 && ZW_DREC_HDR + 2u * (uint32_t)(nlv + lane) < padded) lv[nlv + lane] = 0;
                wsync();
                const zu4 w = *(const zu4*)(rec + 16 * (lane < 55 ? lane : 0));
                bst128(w, ro, 16u * (uint32_t)lane < padded ? used + 16u * (uint32_t)lane : ZW_OOB);
                wsync();
                used += padded;
            }
            if (lane == 0) tcx[mbx] = (uint16_t)T;
        }
    }
    // a frame that failed stopped early: its remaining MBs get empty records at
    // the end (offsets = the bytes used), so the reconstruction that still runs
    // before the host sees the error reads inside the frame's records
    const uint32_t from = bad ? (uint32_t)rfl(mdone) : (uint32_t)nmb;
    for (uint32_t j = from + (uint32_t)lane; j <= (uint32_t)nmb; j += 64) bst32(used, rm, j * 4u);
    if (lane == 0) err[f] = bad ? 1 : 0;
#ifdef ZW_TOK_PROF
    if (lane == 0 && (f == 0 || f == (int)gridDim.x - 1))
        printf("[k_dec_tokens] frame %d: %u decisions, %u loads, %llu cycles (%.1f per decision)\n", f, b.ndec, b.nload,
               (unsigned long long)(__builtin_amdgcn_s_memtime() - t_start),
               (double)(__builtin_amdgcn_s_memtime() - t_start) / (double)b.ndec);
#endif
}

// n frames, one wave each.
extern "C" hipError_t zwk_dec_tokens(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                                     const uint8_t* modes, uint8_t* recs, uint64_t slot, uint32_t* moff, int* err,
                                     int mbw, int mbh, int n)
{
    hipLaunchKernelGGL(k_dec_tokens, dim3((n + ZW_TOK_WAVES - 1) / ZW_TOK_WAVES), dim3(64 * ZW_TOK_WAVES), 0, s, blob, tf,
                       probs, modes, recs, slot, moff, err, mbw, mbh, n);
    return hipGetLastError();
}
