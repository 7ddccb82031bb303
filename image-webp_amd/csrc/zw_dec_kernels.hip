// zw_dec_kernels.hip -- device half of the VP8 decoder (gfx950).
//
//   k_dec_recon    dequant + iWHT + iDCT (exact i16 SSE2 semantics) + intra
//                  prediction + residual add  (decoder/vp8.rs:736-870, :1060-1168)
//   k_loopfilter   in-loop deblocking filter   (decoder/vp8.rs:1172-1345,
//                  decoder/loop_filter.rs)
//
// Both kernels run one workgroup per frame; macroblock rows go round-robin to
// NWD waves and advance as an x+2y wavefront (MB x of row y starts once row
// y-1 has finished MB x+1).  Reconstruction keeps the prediction borders in LDS
// (they are the unfiltered pixels, vp8.rs:791-797).  The loop filter stages
// each MB's 20x20 luma / 12x12 chroma neighbourhood in LDS, filters it in the
// reference's edge order and writes it back; the wavefront order makes every
// overlapping access happen in raster order, as in the reference.
#include "zw_dev.h"

#ifndef ZW_NWD
#define ZW_NWD 16  // 16 rows of the x+2y wavefront in flight per frame
#endif
#define NWD ZW_NWD
#define WGD (NWD * 64)

struct ZwDecQuant {
    int32_t ydc, yac, y2dc, y2ac, uvdc, uvac;
};

struct DecLds {
    uint4 rec[52];  // the current MB's ZwDecMb record (832 B), prefetched one MB ahead
    uint8_t i4idx[10][16];
    uint8_t ws[17 * ZW_BPS];
    uint8_t cu[9 * ZW_BPS], cv[9 * ZW_BPS];
    uint8_t left_y[20], left_u[12], left_v[12];
    int V[40];
    int dc[16];
    int res[16];
    int misc[4];
    uint32_t twy[8], twu[2], twv[2];  // row-parallel kernel: the row above's bottom pixels around this MB
    ZwDecQuant q[4];                  // row-parallel kernel: the frame's segment quantisers
};

__device__ __forceinline__ void dec_wait(const int* progress, int w, int need)
{
    while (__hip_atomic_load(&progress[w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void dec_publish(int* progress, int w, int val)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(&progress[w], val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
}

// I4 value vector for sub-block (x0,y0) of ws (see zw_dev.h d_I4_IDX).
__device__ void dec_i4_values(DecLds* W, int lane, int x0, int y0)
{
    const uint8_t* ws = W->ws;
    auto E = [&](int k) -> int {
        if (k < 4) return ws[(y0 + 3 - k) * ZW_BPS + x0 - 1];
        if (k == 4) return ws[(y0 - 1) * ZW_BPS + x0 - 1];
        return ws[(y0 - 1) * ZW_BPS + x0 + (k - 5)];
    };
    if (lane < 13) W->V[lane] = E(lane);
    else if (lane < 24) { int k = lane - 13; W->V[lane] = (E(k) + 2 * E(k + 1) + E(k + 2) + 2) >> 2; }
    else if (lane < 36) { int k = lane - 24; W->V[lane] = (E(k) + E(k + 1) + 1) >> 1; }
    else if (lane == 36) W->V[36] = (E(11) + 3 * E(12) + 2) >> 2;
    else if (lane == 37) W->V[37] = (E(1) + 3 * E(0) + 2) >> 2;
    else if (lane == 38) {
        int v = 4;
        for (int k = 0; k < 4; k++) v += E(k) + E(5 + k);
        W->V[38] = v >> 3;
    }
    wsync();
}
__device__ __forceinline__ int dec_i4_px(const DecLds* W, int mode, int p)
{
    const int idx = W->i4idx[mode][p];
    if (idx == 255) return W->V[38];
    if (idx == 254) return clamp255(W->V[3 - (p >> 2)] + W->V[5 + (p & 3)] - W->V[4]);
    return W->V[idx];
}

// Residual of one 4x4 block: full iDCT when the block's token run was
// non-empty, DC-only iDCT when only the DC is set (vp8.rs:1110-1117).
__device__ __forceinline__ void dec_block_residual(int* c, int nz)
{
    if (nz) idct16_exact(c);
    else if (c[0] != 0) {
        const int d = (c[0] + 4) >> 3;
#pragma unroll
        for (int k = 0; k < 16; k++) c[k] = d;
    }
}

// ---------------------------------------------------------------------------
// Loop filter (decoder/loop_filter.rs) on LDS-staged neighbourhoods.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int c8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
__device__ __forceinline__ int u2s(int v) { return v - 128; }
__device__ __forceinline__ uint8_t s2u(int v) { return (uint8_t)(c8(v) + 128); }

// p points at q0; s = step across the edge.
__device__ __forceinline__ int lf_common(int outer, uint8_t* p, int s)
{
    const int p1 = u2s(p[-2 * s]), p0 = u2s(p[-s]), q0 = u2s(p[0]), q1 = u2s(p[s]);
    const int o = outer ? c8(p1 - q1) : 0;
    int a = c8(o + 3 * (q0 - p0));
    const int b = c8(a + 3) >> 3;
    a = c8(a + 4) >> 3;
    p[0] = s2u(q0 - a);
    p[-s] = s2u(p0 + b);
    return a;
}
__device__ __forceinline__ bool lf_simple_th(int lim, const uint8_t* p, int s)
{
    return iabs(p[-s] - p[0]) * 2 + iabs(p[-2 * s] - p[s]) / 2 <= lim;
}
__device__ __forceinline__ bool lf_should(int il, int el, const uint8_t* p, int s)
{
    return lf_simple_th(el, p, s) && iabs(p[-4 * s] - p[-3 * s]) <= il && iabs(p[-3 * s] - p[-2 * s]) <= il &&
           iabs(p[-2 * s] - p[-s]) <= il && iabs(p[3 * s] - p[2 * s]) <= il && iabs(p[2 * s] - p[s]) <= il &&
           iabs(p[s] - p[0]) <= il;
}
__device__ __forceinline__ bool lf_hev(int t, const uint8_t* p, int s) { return iabs(p[-2 * s] - p[-s]) > t || iabs(p[s] - p[0]) > t; }

__device__ void lf_simple(int el, uint8_t* p, int s)
{
    if (lf_simple_th(el, p, s)) lf_common(1, p, s);
}
__device__ void lf_inner(int ht, int il, int el, uint8_t* p, int s)
{
    if (lf_should(il, el, p, s)) {
        const bool hv = lf_hev(ht, p, s);
        const int a = (lf_common(hv, p, s) + 1) >> 1;
        if (!hv) {
            p[s] = s2u(u2s(p[s]) - a);
            p[-2 * s] = s2u(u2s(p[-2 * s]) + a);
        }
    }
}
__device__ void lf_mb(int ht, int il, int el, uint8_t* p, int s)
{
    if (lf_should(il, el, p, s)) {
        if (!lf_hev(ht, p, s)) {
            const int p2 = u2s(p[-3 * s]), p1 = u2s(p[-2 * s]), p0 = u2s(p[-s]);
            const int q0 = u2s(p[0]), q1 = u2s(p[s]), q2 = u2s(p[2 * s]);
            const int w = c8(c8(p1 - q1) + 3 * (q0 - p0));
            int a = c8((27 * w + 63) >> 7);
            p[0] = s2u(q0 - a);
            p[-s] = s2u(p0 + a);
            a = c8((18 * w + 63) >> 7);
            p[s] = s2u(q1 - a);
            p[-2 * s] = s2u(p1 + a);
            a = c8((9 * w + 63) >> 7);
            p[2 * s] = s2u(q2 - a);
            p[-3 * s] = s2u(p2 + a);
        } else {
            lf_common(1, p, s);
        }
    }
}

#define LFY 20   // luma staging: rows/cols -4..15 around the MB
#define LFC 12   // chroma staging: -4..7

struct LfLds {
    uint8_t y[LFY * LFY];
    uint8_t u[LFC * LFC], v[LFC * LFC];
};

// Filter one MB (filter_row_in_cache's per-MB edge order, decoder/vp8.rs:1172-1345)
// on its LDS tile and write the tile back.  The lane holds the MB's interior
// word cy (luma row lane>>2, word lane&3) and, for lanes < 32, cc (chroma plane
// lane>>4, row (lane>>1)&7, word lane&1).  The tile's left 4 columns (with the
// corner rows) are carried over in L from the previous MB of the row; the 4
// rows above come from global memory, so the caller has waited for the row
// above to finish MB mbx+1.  Lanes write back the whole tile (the interior
// even when the level is 0: the fused kernel has not stored it yet).
// XCU: the rows above were written by another workgroup (any CU, any XCD), so
// they are read with sc1 loads, and every store is an sc1 (write-through) store
// (MI355X_MICROARCH.md, inter-workgroup hand-off, first table row).
__device__ __forceinline__ uint32_t ld_sc1(const uint8_t* p)
{
    return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint8_t* p, uint32_t v)
{
    __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pub() runs once the rows the MB row below reads (luma 12..15, chroma 4..7 of
// this tile) are stored; the rest of the write-back follows it.
template <bool XCU, class PUB>
__device__ __forceinline__ void lf_tile(LfLds* L, int lane, const ZwFilterParams& F, uint8_t* Yf, uint8_t* Uf,
                                        uint8_t* Vf, int ys, int cs, int mbx, int mby, int i4, int seg, int skip,
                                        int nzd, uint32_t cy, uint32_t cc, bool write_interior_always, PUB&& pub)
{
    auto ld = [](const uint8_t* p) -> uint32_t { return XCU ? ld_sc1(p) : *(const uint32_t*)p; };
    auto st = [](uint8_t* p, uint32_t v) {
        if (XCU) st_sc1(p, v);
        else *(uint32_t*)p = v;
    };
    const bool chroma = !F.filter_type;
    const int iy_r = lane >> 2, iy_w = lane & 3;
    const int ic_p = (lane >> 4) & 1, ic_r = (lane >> 1) & 7, ic_w = lane & 1;
    const int lvl = F.level[seg][i4], il = F.ilimit[seg][i4], ht = F.hev[seg][i4];
    const int x0 = mbx * 16, y0 = mby * 16;
    // ---- assemble the tile ----
    if (mbx > 0) {  // left 4 columns (rows -4..15) from the previous tile's columns 12..15
        if (lane < LFY) {
            uint32_t* row = (uint32_t*)(L->y + lane * LFY);
            row[0] = row[4];
        }
        if (chroma && lane >= 32 && lane < 32 + 2 * LFC) {
            const int pl = (lane - 32) / LFC, r = (lane - 32) % LFC;
            uint32_t* row = (uint32_t*)((pl ? L->v : L->u) + r * LFC);
            row[0] = row[2];
        }
    }
    ((uint32_t*)(L->y + (4 + iy_r) * LFY + 4))[iy_w] = cy;
    if (chroma && lane < 32) ((uint32_t*)((ic_p ? L->v : L->u) + (4 + ic_r) * LFC + 4))[ic_w] = cc;
    if (mby > 0) {  // the 4 rows above: luma lanes 0..15 (row lane>>2), chroma lanes 32..47
        if (lane < 16) {
            const int r = lane >> 2, w = lane & 3;
            ((uint32_t*)(L->y + r * LFY + 4))[w] = ld(Yf + (size_t)(y0 - 4 + r) * ys + x0 + 4 * w);
        } else if (chroma && lane >= 32 && lane < 48) {
            const int t = lane - 32, pl = t >> 3, r = (t >> 1) & 3, w = t & 1;
            ((uint32_t*)((pl ? L->v : L->u) + r * LFC + 4))[w] =
                ld((pl ? Vf : Uf) + (size_t)(mby * 8 - 4 + r) * cs + mbx * 8 + 4 * w);
        }
    }
    wsync();
    if (lvl != 0) {
        const int mbe = (lvl + 2) * 2 + il, sube = lvl * 2 + il;
        const int inner = i4 || (!skip && nzd);
        // lane roles: 0..15 luma line, 16..23 U line, 24..31 V line
        const bool isy = lane < 16, isu = lane >= 16 && lane < 24, isv = lane >= 24 && lane < 32;
        const int li = isy ? lane : (lane - 16) & 7;
        uint8_t* buf = isy ? L->y : (isu ? L->u : L->v);
        const int W_ = isy ? LFY : LFC;
        const bool act = isy || (chroma && (isu || isv));
        // left MB edge (vertical edge, filter along rows)
        if (mbx > 0 && act) {
            uint8_t* p = buf + (li + 4) * W_ + 4;
            if (F.filter_type) lf_simple(mbe, p, 1);
            else lf_mb(ht, il, mbe, p, 1);
        }
        wsync();
        if (inner) {
            for (int x = 4; x < 16; x += 4) {
                if (isy) {
                    uint8_t* p = buf + (li + 4) * W_ + 4 + x;
                    if (F.filter_type) lf_simple(sube, p, 1);
                    else lf_inner(ht, il, sube, p, 1);
                } else if (act && x == 4) {
                    lf_inner(ht, il, sube, buf + (li + 4) * W_ + 4 + 4, 1);
                }
                wsync();
            }
        }
        if (mby > 0 && act) {
            uint8_t* p = buf + 4 * W_ + 4 + li;
            if (F.filter_type) lf_simple(mbe, p, W_);
            else lf_mb(ht, il, mbe, p, W_);
        }
        wsync();
        if (inner) {
            for (int y = 4; y < 16; y += 4) {
                if (isy) {
                    uint8_t* p = buf + (4 + y) * W_ + 4 + li;
                    if (F.filter_type) lf_simple(sube, p, W_);
                    else lf_inner(ht, il, sube, p, W_);
                } else if (act && y == 4) {
                    lf_inner(ht, il, sube, buf + (4 + 4) * W_ + 4 + li, W_);
                }
                wsync();
            }
        }
    }
    const bool wb = lvl != 0 || write_interior_always;
    // write back: luma 20 rows x 5 words, chroma 2 x 12 rows x 3 words (inside the frame);
    // part 0: the rows the MB row below reads, part 1: the others
    for (int part = 0; part < 2; part++) {
        if (wb) {
            for (int t = lane; t < LFY * 5; t += 64) {
                const int r = t / 5 - 4, w = t % 5 - 1;
                if ((r >= 12) == (part == 0) && y0 + r >= 0 && x0 + 4 * w >= 0)
                    st(Yf + (size_t)(y0 + r) * ys + x0 + 4 * w, ((const uint32_t*)(L->y + (r + 4) * LFY))[w + 1]);
            }
            if (chroma) {  // (the simple filter leaves chroma alone: the caller stores it)
                for (int t = lane; t < 2 * LFC * 3; t += 64) {
                    const int pl = t / (LFC * 3), rr = t % (LFC * 3), r = rr / 3 - 4, w = rr % 3 - 1;
                    if ((r >= 4) == (part == 0) && mby * 8 + r >= 0 && mbx * 8 + 4 * w >= 0)
                        st((pl ? Vf : Uf) + (size_t)(mby * 8 + r) * cs + mbx * 8 + 4 * w,
                           ((const uint32_t*)((pl ? L->v : L->u) + (r + 4) * LFC))[w + 1]);
                }
            }
        }
        if (part == 0) pub();
    }
    wsync();
}

// One MB row of the reconstruction (shared by the one-workgroup-per-frame
// kernel and the row-parallel one).  wait(n): block until the row above has
// finished n MBs; pub(n): this row has finished n MBs.  XCU: the row above may
// run on another CU / XCD, so its bottom pixels are exchanged through the
// global border rows gty/gtu/gtv with sc1 stores and loads; otherwise
// gty/gtu/gtv are the workgroup's LDS border rows.
template <bool FUSE, bool XCU, class WAIT, class PUB>
__device__ __forceinline__ void dec_recon_row(const uint4* recs, const ZwDecQuant* __restrict__ quant, uint8_t* Y,
                                              uint8_t* U, uint8_t* V, uint8_t* flags,
                                              const ZwFilterParams* __restrict__ fp, int f, int mbw, int mbh,
                                              size_t ysz, size_t csz, int mby, DecLds* W, LfLds* LF, uint8_t* gty,
                                              uint8_t* gtu, uint8_t* gtv, WAIT&& wait, PUB&& pub)
{
    const int lane = threadIdx.x & 63;
    const int ys = mbw * 16, cs = mbw * 8;
    const size_t nmb = (size_t)mbw * mbh;
    if (lane < 20) W->left_y[lane] = 129;
    if (lane < 12) W->left_u[lane] = W->left_v[lane] = 129;
    wsync();
    uint4 nxt = {0u, 0u, 0u, 0u};
    if (lane < 52) nxt = recs[((size_t)f * nmb + (size_t)mby * mbw) * 52 + lane];
    for (int mbx = 0; mbx < mbw; mbx++) {
        const uint4 cur = nxt;
        if (mbx + 1 < mbw && lane < 52) nxt = recs[((size_t)f * nmb + (size_t)mby * mbw + mbx + 1) * 52 + lane];
        if (mby > 0) wait(min(mbx + 2, mbw));
        if (XCU && mby > 0) {  // the row above's bottom pixels (written by another workgroup)
            if (lane < 8) W->twy[lane] = ld_sc1(gty + mbx * 16 + 4 * lane);
            else if (lane < 10) W->twu[lane - 8] = ld_sc1(gtu + mbx * 8 + 4 * (lane - 8));
            else if (lane < 12) W->twv[lane - 10] = ld_sc1(gtv + mbx * 8 + 4 * (lane - 10));
        }
        const uint8_t* top_y = XCU ? (const uint8_t*)W->twy - mbx * 16 : gty;
        const uint8_t* top_u = XCU ? (const uint8_t*)W->twu - mbx * 8 : gtu;
        const uint8_t* top_v = XCU ? (const uint8_t*)W->twv - mbx * 8 : gtv;
        if (lane < 52) W->rec[lane] = cur;
        wsync();
        const ZwDecMb& M = *(const ZwDecMb*)W->rec;
        const ZwDecQuant& Q = quant[(XCU ? 0 : (size_t)f * 4) + M.segment];  // XCU: quant is the frame's LDS copy
        const int lm = M.luma_mode;
        // --- luma border (create_border_luma) ---
        uint8_t* ws = W->ws;
        if (lane < 32) {
            int v;
            if (lane == 0) v = mby == 0 ? 127 : (mbx == 0 ? 129 : W->left_y[0]);
            else if (mby == 0) v = 127;
            else if (lane <= 16) v = top_y[mbx * 16 + lane - 1];
            else if (mbx == mbw - 1) v = top_y[mbx * 16 + 15];
            else v = top_y[mbx * 16 + lane - 1];
            ws[lane] = (uint8_t)v;
            if (lane >= 17 && lane < 21) ws[4 * ZW_BPS + lane] = ws[8 * ZW_BPS + lane] = ws[12 * ZW_BPS + lane] = (uint8_t)v;
        } else if (lane < 48) {
            ws[(lane - 31) * ZW_BPS] = mbx == 0 ? 129 : W->left_y[lane - 31];
        }
        wsync();
        int nzdct = 0;
        if (lm != 4) {
            // Y2 in group form: lane b holds block b's DC after the iWHT (zero when skipped)
            const int b = lane & 15, bx = b & 3, by = b >> 2;
            const int y2v = M.skip ? 0 : (int)M.y2[b] * (b ? Q.y2ac : Q.y2dc);
            const int dcb = iwht_g(y2v, b);
            // DC predictor sum: lanes 0..15 top row, 16..31 left column
            const int above = mby != 0, left = mbx != 0;
            int dcv;
            {
                const int top = lane < 16;
                const int v = (int)ws[csel(top, 1 + b, (b + 1) * ZW_BPS)] & -(int)(lane < 32 && (top ? above : left));
                const int sum = red16(v);
                const int su = __builtin_amdgcn_readlane(sum, 0) + __builtin_amdgcn_readlane(sum, 16);
                const int shf = 3 + above + left;
                dcv = (!above && !left) ? 128 : ((su + (1 << (shf - 1))) >> shf);
            }
            int blocknz = 0;
            if (lane < 16) {
                int c[16];
                c[0] = dcb;
#pragma unroll
                for (int k = 1; k < 16; k++) c[k] = (int)M.coeffs[b][k] * Q.yac;
                const int nz = (M.nz_mask >> b) & 1;
                blocknz = (c[0] != 0) || nz;
                dec_block_residual(c, nz);
                const int P0 = ws[0];
                int px[16];
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int y = by * 4 + (k >> 2), x = bx * 4 + (k & 3);
                    const int L = ws[(y + 1) * ZW_BPS], T = ws[1 + x];
                    const int p = lm == 0 ? dcv : (lm == 1 ? T : (lm == 2 ? L : clamp255(L + T - P0)));
                    px[k] = clamp255(p + c[k]);
                }
                wsync();
#pragma unroll
                for (int k = 0; k < 16; k++) ws[(by * 4 + (k >> 2) + 1) * ZW_BPS + 1 + bx * 4 + (k & 3)] = (uint8_t)px[k];
            } else {
                wsync();
            }
            nzdct |= __any(blocknz) ? 1 : 0;
            wsync();
        } else {
            // group form: lane k = coefficient k of the sub-block (all four groups alike)
            const int k = lane & 15;
            for (int i = 0; i < 16; i++) {
                const int sby = i >> 2, sbx = i & 3, x0 = sbx * 4 + 1, y0 = sby * 4 + 1;
                dec_i4_values(W, lane, x0, y0);
                const int c = (int)M.coeffs[i][k] * (k ? Q.yac : Q.ydc);
                const int nz = (M.nz_mask >> i) & 1;
                const int c0 = __builtin_amdgcn_readfirstlane(c);  // lane 0 holds the DC
                const int full = idct_g_exact(c, k);
                const int r = nz ? full : (c0 != 0 ? (c0 + 4) >> 3 : 0);
                nzdct |= nz || c0 != 0;
                const int v = clamp255(dec_i4_px(W, M.bpred[i], k) + r);
                if (lane < 16) ws[(y0 + (k >> 2)) * ZW_BPS + x0 + (k & 3)] = (uint8_t)v;
                wsync();
            }
        }
        // --- chroma ---
        if (lane < 34) {  // per plane: corner, 8 top, 8 left
            const int pl = lane >= 17;
            const int i = pl ? lane - 17 : lane;
            uint8_t* w = pl ? W->cv : W->cu;
            const uint8_t* top = pl ? top_v : top_u;
            const uint8_t* lft = pl ? W->left_v : W->left_u;
            if (i == 0) w[0] = mby == 0 ? 127 : (mbx == 0 ? 129 : lft[0]);
            else if (i <= 8) w[i] = mby == 0 ? 127 : top[mbx * 8 + i - 1];
            else w[(i - 8) * ZW_BPS] = mbx == 0 ? 129 : lft[i - 8];
        }
        wsync();
        {
            int blocknz = 0;
            int px[16];
            const int b = lane & 7, pl = b >= 4, bb = b & 3, bx = bb & 1, by = bb >> 1;
            uint8_t* w = pl ? W->cv : W->cu;
            if (lane < 8) {
                const int cm = M.chroma_mode;
                const int above = mby != 0, left = mbx != 0;
                int dcv = 128;
                {
                    uint32_t s = 0;
                    int shf = 2;
                    if (left) {
                        for (int y = 0; y < 8; y++) s += w[(y + 1) * ZW_BPS];
                        shf++;
                    }
                    if (above) {
                        for (int x = 1; x <= 8; x++) s += w[x];
                        shf++;
                    }
                    if (above || left) dcv = (int)((s + (1u << (shf - 1))) >> shf);
                }
                int c[16];
#pragma unroll
                for (int k = 0; k < 16; k++) c[k] = (int)M.coeffs[16 + b][k] * (k ? Q.uvac : Q.uvdc);
                const int nz = (M.nz_mask >> (16 + b)) & 1;
                blocknz = (c[0] != 0) || nz;
                dec_block_residual(c, nz);
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int y = by * 4 + (k >> 2), x = bx * 4 + (k & 3);
                    const int L = w[(y + 1) * ZW_BPS], T = w[1 + x];
                    const int p = cm == 0 ? dcv : (cm == 1 ? T : (cm == 2 ? L : clamp255(L + T - w[0])));
                    px[k] = clamp255(p + c[k]);
                }
            }
            wsync();
            if (lane < 8) {
#pragma unroll
                for (int k = 0; k < 16; k++) w[(by * 4 + (k >> 2) + 1) * ZW_BPS + 1 + bx * 4 + (k & 3)] = (uint8_t)px[k];
            }
            nzdct |= __any(blocknz) ? 1 : 0;
            wsync();
        }
        // --- borders, output ---
        if (lane < 17) W->left_y[lane] = ws[lane * ZW_BPS + 16];
        else if (!XCU && lane < 33) gty[mbx * 16 + lane - 17] = ws[16 * ZW_BPS + lane - 17 + 1];
        if (lane < 9) {
            W->left_u[lane] = W->cu[lane * ZW_BPS + 8];
            W->left_v[lane] = W->cv[lane * ZW_BPS + 8];
        } else if (!XCU && lane >= 40 && lane < 48) {
            gtu[mbx * 8 + lane - 40] = W->cu[8 * ZW_BPS + lane - 40 + 1];
            gtv[mbx * 8 + lane - 40] = W->cv[8 * ZW_BPS + lane - 40 + 1];
        }
        if (XCU && lane >= 48 && lane < 56) {  // bottom row for the row below: 4 + 2 + 2 words, sc1
            const int t = lane - 48;
            const uint8_t* src =
                t < 4 ? ws + 16 * ZW_BPS + 1 + 4 * t : (t < 6 ? W->cu : W->cv) + 8 * ZW_BPS + 1 + 4 * (t & 1);
            const uint32_t w =
                (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) | ((uint32_t)src[3] << 24);
            st_sc1(t < 4 ? gty + mbx * 16 + 4 * t : (t < 6 ? gtu : gtv) + mbx * 8 + 4 * (t & 1), w);
        }
        if (XCU) pub(mbx + 1);  // the row below needs only the border: publish before the plane stores
        uint8_t* uo = U + (size_t)f * csz + (size_t)mby * 8 * cs + mbx * 8;
        uint8_t* vo = V + (size_t)f * csz + (size_t)mby * 8 * cs + mbx * 8;
        if (FUSE) {
            const ZwFilterParams& F = fp[f];
            // interior words: luma row lane>>2 word lane&3; chroma plane lane>>4, row (lane>>1)&7, word lane&1
            const int iy_r = lane >> 2, iy_w = lane & 3;
            const uint8_t* py = ws + (iy_r + 1) * ZW_BPS + 1 + 4 * iy_w;
            const uint32_t cy = (uint32_t)py[0] | ((uint32_t)py[1] << 8) | ((uint32_t)py[2] << 16) | ((uint32_t)py[3] << 24);
            const uint8_t* pc = ((lane >> 4) & 1 ? W->cv : W->cu) + (((lane >> 1) & 7) + 1) * ZW_BPS + 1 + 4 * (lane & 1);
            const uint32_t cc = (uint32_t)pc[0] | ((uint32_t)pc[1] << 8) | ((uint32_t)pc[2] << 16) | ((uint32_t)pc[3] << 24);
            if (F.filter_type) {  // simple filter: chroma is final as reconstructed
                uo[(size_t)(lane >> 3) * cs + (lane & 7)] = W->cu[((lane >> 3) + 1) * ZW_BPS + 1 + (lane & 7)];
                vo[(size_t)(lane >> 3) * cs + (lane & 7)] = W->cv[((lane >> 3) + 1) * ZW_BPS + 1 + (lane & 7)];
            }
            lf_tile<false>(LF, lane, F, Y + (size_t)f * ysz, U + (size_t)f * csz, V + (size_t)f * csz, ys, cs, mbx, mby,
                    lm == 4, M.segment, M.skip, nzdct, cy, cc, true, [] {});
        } else {
            uint8_t* yo = Y + (size_t)f * ysz + (size_t)mby * 16 * ys + mbx * 16;
            for (int k = lane; k < 256; k += 64) yo[(size_t)(k >> 4) * ys + (k & 15)] = ws[((k >> 4) + 1) * ZW_BPS + 1 + (k & 15)];
            uo[(size_t)(lane >> 3) * cs + (lane & 7)] = W->cu[((lane >> 3) + 1) * ZW_BPS + 1 + (lane & 7)];
            vo[(size_t)(lane >> 3) * cs + (lane & 7)] = W->cv[((lane >> 3) + 1) * ZW_BPS + 1 + (lane & 7)];
            if (lane < 4) {
                const int v = lane == 0 ? lm : (lane == 1 ? M.segment : (lane == 2 ? M.skip : nzdct));
                flags[((size_t)f * nmb + (size_t)mby * mbw + mbx) * 4 + lane] = (uint8_t)v;
            }
            wsync();
        }
            if (!XCU) pub(mbx + 1);
        }
}

// FUSE: the loop filter runs in the same wavefront right after each MB's
// reconstruction (the prediction of later MBs reads the unfiltered borders kept
// in LDS, vp8.rs:791-797; the filter reads and writes the planes in the same
// raster-consistent order as k_loopfilter), so a frame pays one wavefront
// instead of two.
template <bool FUSE>
__global__ __launch_bounds__(WGD) __attribute__((amdgpu_waves_per_eu(NWD / 4, NWD / 4))) void k_dec_recon(const ZwDecMb* __restrict__ mbs,
                                                              const ZwDecQuant* __restrict__ quant, uint8_t* Y, uint8_t* U,
                                                              uint8_t* V, uint8_t* flags, int mbw, int mbh, size_t ysz,
                                                              size_t csz, const ZwFilterParams* __restrict__ fp)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int f = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    size_t off = 0;
    DecLds* Wall = (DecLds*)smem;
    off += ((sizeof(DecLds) + 15) & ~(size_t)15) * NWD;
    int* progress = (int*)(smem + off);
    off += 64;
    uint8_t* top_y = smem + off;
    off += ((size_t)mbw * 16 + 48 + 15) & ~(size_t)15;
    uint8_t* top_u = smem + off;
    off += ((size_t)mbw * 8 + 48 + 15) & ~(size_t)15;
    uint8_t* top_v = smem + off;
    off += ((size_t)mbw * 8 + 48 + 15) & ~(size_t)15;
    LfLds* LF = (LfLds*)(smem + off) + wv;  // FUSE only
    DecLds* W = (DecLds*)((uint8_t*)Wall + ((sizeof(DecLds) + 15) & ~(size_t)15) * wv);
    for (int i = lane; i < 160; i += 64) (&W->i4idx[0][0])[i] = (&d_I4_IDX[0][0])[i];
    for (int i = threadIdx.x; i < mbw * 16 + 48; i += WGD) top_y[i] = 127;
    for (int i = threadIdx.x; i < mbw * 8 + 48; i += WGD) top_u[i] = top_v[i] = 127;
    if (threadIdx.x < NWD) progress[threadIdx.x] = -1;
    __syncthreads();
    const uint4* recs = (const uint4*)mbs;  // 52 lines per record
    for (int mby = wv; mby < mbh; mby += NWD) {
        dec_recon_row<FUSE, false>(
            recs, quant, Y, U, V, flags, fp, f, mbw, mbh, ysz, csz, mby, W, LF, top_y, top_u, top_v,
            [&](int need) { dec_wait(progress, (mby - 1) % NWD, (mby - 1) * 65536 + need); },
            [&](int done) { dec_publish(progress, wv, mby * 65536 + done); });
    }
}

// Row-parallel reconstruction: one wave per workgroup, rows handed out by a
// per-frame ticket (a wave only ever waits for a row whose ticket an already
// running wave holds, so the grid cannot deadlock whatever the residency), the
// row-to-row hand-off through global memory (progress flags and the bottom
// pixel rows, sc1 both ways).  For one frame or a few, this spreads the x+2y
// wavefront over up to mbh CUs instead of one.
#define ZW_SPIN_MAX (1 << 22)
__device__ __forceinline__ int row_ticket(int* ticket)
{
    int t = 0;
    if ((threadIdx.x & 63) == 0) t = atomicAdd(ticket, 1);
    return __builtin_amdgcn_readfirstlane(__shfl(t, 0));
}
// Wait until *prog >= need.  seen caches the last value read: the row above
// usually runs ahead, so most waits cost no memory round trip.
__device__ __forceinline__ void row_wait(const int* prog, int need, int* err, int& seen)
{
    if (seen >= need) return;
    int it = 0;
    for (;;) {
        seen = __hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (seen >= need) break;
        __builtin_amdgcn_s_sleep(2);
        // never expected: after ZW_SPIN_MAX polls (or once any wave of the frame
        // gave up) report through *err instead of hanging the GPU
        if (++it > ZW_SPIN_MAX || ((it & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            if ((threadIdx.x & 63) == 0) atomicOr(err, 1);
            seen = 1 << 30;
            break;
        }
    }
}
__device__ __forceinline__ void row_publish(int* prog, int val)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are out
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(prog, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
}

// rowsync per frame: [0] recon ticket, [1] filter ticket, [2] error, [3] pad,
// then progress[2][mbh] (recon, filter), initialised to -1.
__device__ __forceinline__ int* rs_frame(int* rowsync, int f, int mbh) { return rowsync + (size_t)f * (4 + 2 * mbh); }

__global__ __launch_bounds__(64) void k_dec_recon_rows(const ZwDecMb* __restrict__ mbs,
                                                       const ZwDecQuant* __restrict__ quant, uint8_t* Y, uint8_t* U,
                                                       uint8_t* V, uint8_t* flags, int mbw, int mbh, size_t ysz,
                                                       size_t csz, int* rowsync, uint8_t* borders)
{
    __shared__ __attribute__((aligned(16))) DecLds Wl;
    DecLds* W = &Wl;
    const int f = blockIdx.y, lane = threadIdx.x;
    for (int i = lane; i < 160; i += 64) (&W->i4idx[0][0])[i] = (&d_I4_IDX[0][0])[i];
    if (lane < 24) ((int32_t*)W->q)[lane] = ((const int32_t*)(quant + (size_t)f * 4))[lane];
    int* rs = rs_frame(rowsync, f, mbh);
    int* prog = rs + 4;
    const size_t bsz = (size_t)mbw * 16 + 48 + 2 * ((size_t)mbw * 8 + 48);
    uint8_t* gty = borders + (size_t)f * bsz;
    uint8_t* gtu = gty + (size_t)mbw * 16 + 48;
    uint8_t* gtv = gtu + (size_t)mbw * 8 + 48;
    wsync();
    for (;;) {
        const int mby = row_ticket(&rs[0]);
        if (mby >= mbh) break;
        int seen = -1;
        dec_recon_row<false, true>(
            (const uint4*)mbs, W->q, Y, U, V, flags, nullptr, f, mbw, mbh, ysz, csz, mby, W, nullptr, gty, gtu, gtv,
            [&](int need) { row_wait(&prog[mby - 1], need, &rs[2], seen); },
            [&](int done) { row_publish(&prog[mby], done); });
    }
}

// Per wave, row by row: the MB's 16x16 / 8x8 interiors only change when the
// MB itself is filtered, so they are prefetched into registers one MB ahead.
extern "C" __global__ __launch_bounds__(WGD) void k_loopfilter(uint8_t* Y, uint8_t* U, uint8_t* V,
                                                               const uint8_t* __restrict__ flags,
                                                               const ZwFilterParams* __restrict__ fp, size_t ysz,
                                                               size_t csz)
{
    __shared__ __attribute__((aligned(16))) LfLds lds[NWD];
    __shared__ int progress[NWD];
    const int f = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const ZwFilterParams& F = fp[f];
    const int mbw = F.mbw, mbh = F.mbh, ys = mbw * 16, cs = mbw * 8;
    const size_t nmb = (size_t)mbw * mbh;
    if (threadIdx.x < NWD) progress[threadIdx.x] = -1;
    __syncthreads();
    LfLds* L = &lds[wv];
    uint8_t* Yf = Y + (size_t)f * ysz;
    uint8_t* Uf = U + (size_t)f * csz;
    uint8_t* Vf = V + (size_t)f * csz;
    const bool chroma = !F.filter_type;
    const int iy_r = lane >> 2, iy_w = lane & 3;
    const int ic_p = (lane >> 4) & 1, ic_r = (lane >> 1) & 7, ic_w = lane & 1;
    auto load_interior = [&](int mby, int mbx, uint32_t& py, uint32_t& pc) {
        py = *(const uint32_t*)(Yf + (size_t)(mby * 16 + iy_r) * ys + mbx * 16 + 4 * iy_w);
        pc = 0;
        if (chroma && lane < 32)
            pc = *(const uint32_t*)((ic_p ? Vf : Uf) + (size_t)(mby * 8 + ic_r) * cs + mbx * 8 + 4 * ic_w);
    };
    for (int mby = wv; mby < mbh; mby += NWD) {
        uint32_t ny, nc;
        load_interior(mby, 0, ny, nc);
        uint32_t nfl = *(const uint32_t*)(flags + ((size_t)f * nmb + (size_t)mby * mbw) * 4);
        for (int mbx = 0; mbx < mbw; mbx++) {
            const uint32_t cy = ny, cc = nc, fl = nfl;
            if (mbx + 1 < mbw) {
                load_interior(mby, mbx + 1, ny, nc);
                nfl = *(const uint32_t*)(flags + ((size_t)f * nmb + (size_t)mby * mbw + mbx + 1) * 4);
            }
            if (mby > 0) dec_wait(progress, (mby - 1) % NWD, (mby - 1) * 65536 + min(mbx + 2, mbw));
            lf_tile<false>(L, lane, F, Yf, Uf, Vf, ys, cs, mbx, mby, (fl & 255) == 4, (fl >> 8) & 255,
                           (fl >> 16) & 255, fl >> 24, cy, cc, false, [] {});
            dec_publish(progress, wv, mby * 65536 + mbx + 1);
        }
    }
}

// Row-parallel loop filter (see k_dec_recon_rows): every load and store of
// pixels another row hands over is sc1, including this row's own interior
// loads (MI355X_MICROARCH.md: every load of handed-off bytes must be one).
__global__ __launch_bounds__(64) void k_loopfilter_rows(uint8_t* Y, uint8_t* U, uint8_t* V,
                                                        const uint8_t* __restrict__ flags,
                                                        const ZwFilterParams* __restrict__ fp, size_t ysz, size_t csz,
                                                        int* rowsync)
{
    __shared__ __attribute__((aligned(16))) LfLds Ll;
    LfLds* L = &Ll;
    const int f = blockIdx.y, lane = threadIdx.x;
    const ZwFilterParams& F = fp[f];
    const int mbw = F.mbw, mbh = F.mbh, ys = mbw * 16, cs = mbw * 8;
    const size_t nmb = (size_t)mbw * mbh;
    int* rs = rs_frame(rowsync, f, mbh);
    int* prog = rs + 4 + mbh;
    uint8_t* Yf = Y + (size_t)f * ysz;
    uint8_t* Uf = U + (size_t)f * csz;
    uint8_t* Vf = V + (size_t)f * csz;
    const bool chroma = !F.filter_type;
    const int iy_r = lane >> 2, iy_w = lane & 3;
    const int ic_p = (lane >> 4) & 1, ic_r = (lane >> 1) & 7, ic_w = lane & 1;
    auto load_interior = [&](int mby, int mbx, uint32_t& py, uint32_t& pc) {
        py = ld_sc1(Yf + (size_t)(mby * 16 + iy_r) * ys + mbx * 16 + 4 * iy_w);
        pc = 0;
        if (chroma && lane < 32) pc = ld_sc1((ic_p ? Vf : Uf) + (size_t)(mby * 8 + ic_r) * cs + mbx * 8 + 4 * ic_w);
    };
    for (;;) {
        const int mby = row_ticket(&rs[1]);
        if (mby >= mbh) break;
        uint32_t ny, nc;
        load_interior(mby, 0, ny, nc);
        uint32_t nfl = *(const uint32_t*)(flags + ((size_t)f * nmb + (size_t)mby * mbw) * 4);
        int seen = -1;
        for (int mbx = 0; mbx < mbw; mbx++) {
            const uint32_t cy = ny, cc = nc, fl = nfl;
            if (mbx + 1 < mbw) {
                load_interior(mby, mbx + 1, ny, nc);
                nfl = *(const uint32_t*)(flags + ((size_t)f * nmb + (size_t)mby * mbw + mbx + 1) * 4);
            }
            if (mby > 0) row_wait(&prog[mby - 1], min(mbx + 2, mbw), &rs[2], seen);
            lf_tile<true>(L, lane, F, Yf, Uf, Vf, ys, cs, mbx, mby, (fl & 255) == 4, (fl >> 8) & 255,
                          (fl >> 16) & 255, fl >> 24, cy, cc, false, [&] { row_publish(&prog[mby], mbx + 1); });
        }
    }
}

// Row-parallel path scratch: rowsync ints and border rows for nframes frames.
extern "C" size_t zw_dec_rows_sync_bytes(int mbh, int nframes) { return (size_t)nframes * (4 + 2 * mbh) * 4; }
extern "C" size_t zw_dec_rows_border_bytes(int mbw, int nframes)
{
    return (size_t)nframes * ((size_t)mbw * 16 + 48 + 2 * ((size_t)mbw * 8 + 48));
}

// rowsync must hold zeros in [0..3] and -1 in the progress words of every
// frame (zw_dec_rows_sync_init); rows = workgroups (waves) per frame.
// phase 1: reconstruction, 2: loop filter.
extern "C" hipError_t zwk_dec_rows(hipStream_t s, int phase, const ZwDecMb* mbs, const void* quant, uint8_t* Y,
                                   uint8_t* U, uint8_t* V, uint8_t* flags, const ZwFilterParams* fp, int mbw, int mbh,
                                   size_t ysz, size_t csz, int nframes, int* rowsync, uint8_t* borders, int rows)
{
    const int R = rows < 1 ? 1 : (rows > mbh ? mbh : rows);
    if (phase == 1)
        hipLaunchKernelGGL(k_dec_recon_rows, dim3(R, nframes), dim3(64), 0, s, mbs, (const ZwDecQuant*)quant, Y, U,
                           V, flags, mbw, mbh, ysz, csz, rowsync, borders);
    else
        hipLaunchKernelGGL(k_loopfilter_rows, dim3(R, nframes), dim3(64), 0, s, Y, U, V, flags, fp, ysz, csz,
                           rowsync);
    return hipGetLastError();
}

// Sets the rowsync words: tickets / error 0, progress -1.
__global__ void k_dec_rows_init(int* rowsync, int mbh, int total)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < total) rowsync[i] = (i % (4 + 2 * mbh)) < 4 ? 0 : -1;
}
extern "C" hipError_t zwk_dec_rows_init(hipStream_t s, int* rowsync, int mbh, int nframes)
{
    const int total = nframes * (4 + 2 * mbh);
    hipLaunchKernelGGL(k_dec_rows_init, dim3((total + 255) / 256), dim3(256), 0, s, rowsync, mbh, total);
    return hipGetLastError();
}

extern "C" size_t zw_dec_lds_bytes(int mbw)
{
    size_t off = ((sizeof(DecLds) + 15) & ~(size_t)15) * NWD + 64;
    off += ((size_t)mbw * 16 + 48 + 15) & ~(size_t)15;
    off += 2 * (((size_t)mbw * 8 + 48 + 15) & ~(size_t)15);
    off += sizeof(LfLds) * NWD;
    return off;
}

// k_dec_expand: packed MB records (what crossed PCIe, zw_common.h ZW_DREC_*)
// -> full ZwDecMb records for k_dec_recon.  One wave per MB, fully parallel
// over the batch: the wavefront kernel keeps its one-MB-ahead prefetch of
// fixed-size records.  Slot sl = block (sl >> 4, 24 = Y2) x zigzag position.
extern "C" __global__ __launch_bounds__(256) void k_dec_expand(const uint8_t* __restrict__ recs,
                                                                 const uint32_t* __restrict__ moff,
                                                                 const uint64_t* __restrict__ fbase, ZwDecMb* mbs,
                                                                 int nmb)
{
    __shared__ uint4 raw[4][55];
    const int f = blockIdx.y, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + wv;
    if (i >= nmb) return;
    const uint32_t* fo = moff + (size_t)f * (nmb + 1);
    const uint32_t a = fo[i], e = fo[i + 1];
    if (a + 16u * (uint32_t)lane < e && lane < 55) raw[wv][lane] = *(const uint4*)(recs + fbase[f] + a + 16u * lane);
    wsync();
    const uint8_t* rb = (const uint8_t*)raw[wv];
    const uint16_t* st = (const uint16_t*)(rb + 16);
    const int16_t* lv = (const int16_t*)(rb + ZW_DREC_HDR);
    // the 832-byte record as 52 16-byte lines: lane l < 52 assembles line l
    // from 8 halfwords (line 0: header bytes and bpred, line 1..: y2/coeffs)
    uint4* out = (uint4*)(mbs + (size_t)f * nmb + i);
    if (lane < 52) {
        uint16_t h[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int byte = lane * 16 + q * 2;  // offset in ZwDecMb
            int v = 0;
            if (byte >= 24 && byte < 824) {  // y2[16] at 24, coeffs[24][16] at 56
                const int c = (byte - 24) >> 1, b = c < 16 ? 24 : (c - 16) >> 4, nat = c & 15;
                const int k = izz_of(nat), s0 = st[b], s1 = st[b + 1];
                v = s0 + k < s1 ? (int)(uint16_t)lv[s0 + k] : 0;
            } else if (byte < 24) {
                auto hb = [&](int o) -> int {
                    if (o == 0) return rb[0] & 7;
                    if (o == 1) return (rb[0] >> 3) & 3;
                    if (o == 2) return rb[1];
                    if (o == 3) return (rb[0] >> 5) & 1;
                    if (o < 20) return (rb[8 + ((o - 4) >> 1)] >> (4 * ((o - 4) & 1))) & 15;
                    return rb[4 + (o - 20)];  // nz_mask
                };
                v = hb(byte) | (hb(byte + 1) << 8);
            }
            h[q] = (uint16_t)v;
        }
        out[lane] = make_uint4(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16), h[4] | ((uint32_t)h[5] << 16),
                               h[6] | ((uint32_t)h[7] << 16));
    }
}

extern "C" hipError_t zwk_dec_expand(hipStream_t s, const uint8_t* recs, const uint32_t* moff, const uint64_t* fbase,
                                     ZwDecMb* mbs, int nmb, int nframes)
{
    hipLaunchKernelGGL(k_dec_expand, dim3((nmb + 3) / 4, nframes), dim3(256), 0, s, recs, moff, fbase, mbs, nmb);
    return hipGetLastError();
}

// fp == nullptr: reconstruction only (k_loopfilter follows); else the fused kernel.
extern "C" hipError_t zwk_dec_recon(hipStream_t s, const ZwDecMb* mbs, const void* quant, uint8_t* Y, uint8_t* U,
                                    uint8_t* V, uint8_t* flags, int mbw, int mbh, size_t ysz, size_t csz, int nframes,
                                    const ZwFilterParams* fp)
{
    static const bool attr = []() {
        (void)hipFuncSetAttribute((const void*)k_dec_recon<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_dec_recon<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    if (fp)
        hipLaunchKernelGGL(k_dec_recon<true>, dim3(nframes), dim3(WGD), zw_dec_lds_bytes(mbw), s, mbs,
                           (const ZwDecQuant*)quant, Y, U, V, flags, mbw, mbh, ysz, csz, fp);
    else
        hipLaunchKernelGGL(k_dec_recon<false>, dim3(nframes), dim3(WGD), zw_dec_lds_bytes(mbw), s, mbs,
                           (const ZwDecQuant*)quant, Y, U, V, flags, mbw, mbh, ysz, csz, fp);
    return hipGetLastError();
}

extern "C" hipError_t zwk_loopfilter(hipStream_t s, uint8_t* Y, uint8_t* U, uint8_t* V, const uint8_t* flags,
                                     const ZwFilterParams* fp, size_t ysz, size_t csz, int nframes)
{
    hipLaunchKernelGGL(k_loopfilter, dim3(nframes), dim3(WGD), 0, s, Y, U, V, flags, fp, ysz, csz);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// k_yuv2rgb: decoded YUV 4:2:0 planes -> packed RGB / RGBA (decoder/yuv.rs).
//
// FANCY: fill_rgb_buffer_fancy (yuv.rs:82-160) with its row helpers
// fill_row_fancy_with_2_uv_rows / _1_uv_row (:162-395).  Written per output
// pixel: chroma sample (main row mr, secondary row sr) x (main column mc,
// secondary column sc) and U = (9 m + 3 s1 + 3 s2 + t + 8) >> 4
// (get_fancy_chroma_value, :397).  Row r >= 1 pairs with chroma rows
// (r-1)/2 and (r+1)/2 (main = the nearer one); row 0 and the final row of an
// even-height image use one chroma row (sr = mr); columns likewise, with the
// first pixel and the final pixel of an even-width row on one chroma column.
// Every one of those special cases is the general formula with sr / sc
// clamped to the image's chroma extent.
// !FANCY: fill_rgb_buffer_simple (yuv.rs:402-515): U = u[r/2][x/2].
// yuv_to_r/g/b (:63-78): mulhi(v, c) = (v * c) >> 8, clip = clamp(v >> 6).
// BPP 4 writes alpha 255 (decode_rgba, decoder/api.rs:938-960).
//
// One thread per 4 consecutive pixels of the packed output (flat index, so
// the 12 / 16-byte stores stay 4-byte aligned for any width); frames on
// blockIdx.y.  Algorithmic bytes per pixel: 1 (Y) + 0.5 (U, V) read,
// BPP written.
// ---------------------------------------------------------------------------
// clip (yuv.rs:57-61).  Written as inline v_med3_i32: otherwise the gfx950
// backend fuses two neighbouring clips of the packed pixel into
// v_ashr_pk_u8_i32 and then ORs the third channel over bits 16-31 it assumes
// are zero; they are not (measured: blue read back as 255 whenever green
// clipped to 0).
__device__ __forceinline__ int yuv_clip(int v)
{
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(v >> 6), "v"(255));
    return r;
}
__device__ __forceinline__ uint32_t yuv_px(int y, int u, int v)
{
    const int yy = (y * 19077) >> 8;
    const int r = yuv_clip(yy + ((v * 26149) >> 8) - 14234);
    const int g = yuv_clip(yy - ((u * 6419) >> 8) - ((v * 13320) >> 8) + 8708);
    const int b = yuv_clip(yy + ((u * 33050) >> 8) - 17685);
    return (uint32_t)r | ((uint32_t)g << 8) | ((uint32_t)b << 16) | 0xff000000u;
}

// General per-pixel form (edges, odd widths): the chroma sample indices with
// their clamps, one byte load per sample.
template <bool FANCY>
__device__ __forceinline__ uint32_t yuv2rgb_px(const uint8_t* Y, const uint8_t* U, const uint8_t* V, int ys, int cs,
                                               int cw1, int ch1, int r, int x)
{
    const int yv = Y[(size_t)r * ys + x];
    int u, v;
    if (FANCY) {
        const int k = (r + 1) >> 1;
        const int mr = (r & 1) ? k - 1 : k, sr = max(min((r & 1) ? k : k - 1, ch1), 0);
        const int q = (x - 1) >> 1;  // x = 0: q = -1 -> mc = sc = 0
        const int mc = (x & 1) ? q : q + 1, sc = min(max((x & 1) ? q + 1 : q, 0), cw1);
        const uint8_t *um = U + (size_t)mr * cs, *us = U + (size_t)sr * cs;
        const uint8_t *vm = V + (size_t)mr * cs, *vs = V + (size_t)sr * cs;
        u = (9 * um[mc] + 3 * um[sc] + 3 * us[mc] + us[sc] + 8) >> 4;
        v = (9 * vm[mc] + 3 * vm[sc] + 3 * vs[mc] + vs[sc] + 8) >> 4;
    } else {
        u = U[(size_t)(r >> 1) * cs + (x >> 1)];
        v = V[(size_t)(r >> 1) * cs + (x >> 1)];
    }
    return yuv_px(yv, u, v);
}

__device__ __forceinline__ int byte_of(uint32_t w0, uint32_t w1, uint32_t w2, int i)  // i constant after unrolling
{
    const uint32_t w = i < 4 ? w0 : (i < 8 ? w1 : w2);
    return (int)((w >> (8 * (i & 3))) & 255u);
}

// One thread per 8 horizontally adjacent pixels of one output row (x = 8 *
// thread): Y as one 8-byte load, each chroma row as three aligned words
// covering columns x/2-4 .. x/2+7, so the interior does two vector loads per
// plane row and no per-sample addressing; the 8 pixels leave as two 16-byte
// (RGBA) or six 4-byte (RGB) stores.  Threads at the image edges, or whose
// row start is not 4-byte aligned in the packed RGB output, take the
// per-pixel form.
template <int BPP, bool FANCY>
__global__ __launch_bounds__(256) void k_yuv2rgb(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U,
                                                 const uint8_t* __restrict__ V, size_t ysz, size_t csz, int w, int h,
                                                 int ys, int cs, uint8_t* __restrict__ out)
{
    const int f = blockIdx.z, r = blockIdx.y;
    const int x = (int)(blockIdx.x * 256u + threadIdx.x) * 8;
    if (x >= w) return;
    Y += (size_t)f * ysz;
    U += (size_t)f * csz;
    V += (size_t)f * csz;
    uint8_t* o = out + ((size_t)f * h + r) * (size_t)w * BPP + (size_t)x * BPP;
    const int cw1 = ((w + 1) >> 1) - 1, ch1 = ((h + 1) >> 1) - 1;
    // (every full 8-pixel run takes the vector path; at the image's left / right
    // edge the fancy filter's outer chroma column is the edge column itself, so
    // the neighbour word is not loaded and the edge byte stands in for it)
    const bool fast = x + 8 <= w && (ys & 7) == 0 && (cs & 3) == 0 && ((uintptr_t)o & (BPP == 4 ? 15 : 3)) == 0;
    uint32_t px[8];
    if (fast) {
        const uint2 yy = *(const uint2*)(Y + (size_t)r * ys + x);
        const bool lok = x > 0, rok = (x >> 1) + 4 <= cw1;
        const int c1 = x >> 1, c0 = lok ? c1 - 4 : c1, c2 = rok ? c1 + 4 : c1;
        int mr, sr;
        if (FANCY) {
            const int k = (r + 1) >> 1;
            mr = (r & 1) ? k - 1 : k;
            sr = max(min((r & 1) ? k : k - 1, ch1), 0);
        } else {
            mr = sr = r >> 1;
        }
        auto row3 = [&](const uint8_t* P, int rr, int& b0, int& b5, uint32_t& mid) {
            const uint8_t* q = P + (size_t)rr * cs;
            const uint32_t a = *(const uint32_t*)(q + c0), m = *(const uint32_t*)(q + c1), z = *(const uint32_t*)(q + c2);
            b0 = (int)(lok ? a >> 24 : m & 255u);
            b5 = (int)(rok ? z & 255u : m >> 24);
            mid = m;
        };
        int um_l, um_r, vm_l, vm_r, us_l, us_r, vs_l, vs_r;
        uint32_t umw, vmw, usw, vsw;
        row3(U, mr, um_l, um_r, umw);
        row3(V, mr, vm_l, vm_r, vmw);
        if (FANCY) {
            row3(U, sr, us_l, us_r, usw);
            row3(V, sr, vs_l, vs_r, vsw);
        } else {
            us_l = um_l, us_r = um_r, usw = umw, vs_l = vm_l, vs_r = vm_r, vsw = vmw;
        }
        // fancy: 9 m + 3 s1 + 3 s2 + t = 3 (3 um + us)[mc] + (3 um + us)[sc], so
        // blend the two chroma rows once per column (local columns x/2-1 .. x/2+4)
        int tu[6], tv[6];
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const int um = j == 0 ? um_l : (j == 5 ? um_r : (int)((umw >> (8 * (j - 1))) & 255u));
            const int us = j == 0 ? us_l : (j == 5 ? us_r : (int)((usw >> (8 * (j - 1))) & 255u));
            const int vm = j == 0 ? vm_l : (j == 5 ? vm_r : (int)((vmw >> (8 * (j - 1))) & 255u));
            const int vs = j == 0 ? vs_l : (j == 5 ? vs_r : (int)((vsw >> (8 * (j - 1))) & 255u));
            if (FANCY) {
                tu[j] = 3 * um + us;
                tv[j] = 3 * vm + vs;
            } else {
                tu[j] = um;
                tv[j] = vm;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int yv = (int)(((i < 4 ? yy.x : yy.y) >> (8 * (i & 3))) & 255u);
            const int jm = 1 + (i >> 1);  // local chroma column (x + i) / 2 - 3
            int u, v;
            if (FANCY) {
                const int js = (i & 1) ? jm + 1 : jm - 1;
                u = (3 * tu[jm] + tu[js] + 8) >> 4;
                v = (3 * tv[jm] + tv[js] + 8) >> 4;
            } else {
                u = tu[jm];
                v = tv[jm];
            }
            px[i] = yuv_px(yv, u, v);
        }
        if (BPP == 4) {
            ((uint4*)o)[0] = make_uint4(px[0], px[1], px[2], px[3]);
            ((uint4*)o)[1] = make_uint4(px[4], px[5], px[6], px[7]);
        } else {
            uint32_t* d = (uint32_t*)o;
#pragma unroll
            for (int g = 0; g < 2; g++) {
                const uint32_t p0 = px[4 * g], p1 = px[4 * g + 1], p2 = px[4 * g + 2], p3 = px[4 * g + 3];
                d[3 * g + 0] = (p0 & 0xffffffu) | (p1 << 24);
                d[3 * g + 1] = ((p1 >> 8) & 0xffffu) | (p2 << 16);
                d[3 * g + 2] = ((p2 >> 16) & 0xffu) | ((p3 & 0xffffffu) << 8);
            }
        }
    } else {
        const int n = min(8, w - x);
        for (int i = 0; i < n; i++) {
            const uint32_t p = yuv2rgb_px<FANCY>(Y, U, V, ys, cs, cw1, ch1, r, x + i);
            for (int c = 0; c < BPP; c++) o[(size_t)i * BPP + c] = (uint8_t)(p >> (8 * c));
        }
    }
}

extern "C" hipError_t zwk_yuv2rgb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, size_t ysz,
                                  size_t csz, int w, int h, int ys, int cs, int bpp, int fancy, uint8_t* out,
                                  int nframes)
{
    const dim3 grid(((unsigned)w + 2047) / 2048, (unsigned)h, (unsigned)nframes);
    if (bpp == 4) {
        if (fancy) hipLaunchKernelGGL((k_yuv2rgb<4, true>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
        else hipLaunchKernelGGL((k_yuv2rgb<4, false>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
    } else {
        if (fancy) hipLaunchKernelGGL((k_yuv2rgb<3, true>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
        else hipLaunchKernelGGL((k_yuv2rgb<3, false>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
    }
    return hipGetLastError();
}
