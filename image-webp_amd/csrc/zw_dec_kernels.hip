// zw_dec_kernels.hip -- device half of the VP8 decoder (gfx950).
//
//   k_dec_recon    dequant + iWHT + iDCT (exact i16 SSE2 semantics) + intra
//                  prediction + residual add  (decoder/vp8.rs:736-870, :1060-1168)
//   k_loopfilter   in-loop deblocking filter   (decoder/vp8.rs:1172-1345,
//                  decoder/loop_filter.rs)
//
// Both kernels run one workgroup per frame; macroblock rows go round-robin to
// NWD waves and advance as an x+2y wavefront (MB x of row y starts once row
// y-1 has finished MB x+1).  Reconstruction works in quad form (lane = 4 block
// + pixel row: the iDCT's column pass in the lane, the transpose by DPP, the
// row as one word of the plane) from the unfiltered borders kept in LDS
// (vp8.rs:791-797); only I4 MBs chain through an LDS work area.  The loop
// filter stages each MB's 20x20 luma / 12x12 chroma neighbourhood in LDS,
// filters one row per lane across the vertical edges and then one column per
// lane across the horizontal ones (the reference's edge order, each line in
// registers), and writes it back; the wavefront order makes every overlapping
// access happen in raster order, as in the reference.
#include "zw_dev.h"

#ifndef ZW_NWD
#define ZW_NWD 16  // 16 rows of the x+2y wavefront in flight per frame
#endif
#define NWD ZW_NWD
#define WGD (NWD * 64)
#define ZW_DEC_TILE 384  // batch recon -> filter hand-over: one MB, luma 16 x 16 then U, V 8 x 8

struct ZwDecQuant {
    int32_t ydc, yac, y2dc, y2ac, uvdc, uvac;
};

struct DecLds {
    uint4 rec[55];  // the current MB's packed record (zw_common.h ZW_DREC_*, <= 880 B), prefetched one MB ahead
    uint8_t i4idx[10][16];
    uint8_t ws[17 * ZW_BPS];  // I4 MBs: the luma work area (border row / column + 16x16)
    uint8_t left_y[20], left_u[12], left_v[12];
    int16_t res4[16 * 16];  // I4 MBs: the 16 sub-blocks' residuals (block, row, column), computed up front
    uint32_t twy[8], twu[2], twv[2];  // row-parallel kernel: the row above's bottom pixels around this MB
    ZwDecQuant q[4];                  // row-parallel kernel: the frame's segment quantisers
};

// Row hand-off inside a workgroup.  Everything a row passes to the row below
// (border pixels, progress) lives in LDS, so publishing waits only for this
// wave's LDS writes (lgkmcnt), never for its global stores: those are written
// by one wave each and read by no other wave of the kernel.  LDS accesses are
// coherent across the CU's waves, so once the consumer has read the progress
// word its later LDS reads see every write made before it.
__device__ __forceinline__ void dec_wait(const int* progress, int w, int need)
{
    while (__hip_atomic_load(&progress[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void dec_publish(int* progress, int w, int val)
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(&progress[w], val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
}

// I4 edge offsets: E(j) of the sub-block whose top-left pixel is ws[base]
// (j < 4: the left column bottom-up, 4: the corner, 5..12: the row above and
// the above-right four; the d_I4_IDX value-vector order, zw_dev.h).
DI int i4_eoff(int j) { return j < 4 ? (3 - j) * ZW_BPS - 1 : (j == 4 ? -ZW_BPS - 1 : -ZW_BPS + (j - 5)); }


// Packed MB record (zw_common.h ZW_DREC_*, written by zw_dec_host.cpp
// parse_mbs or k_dec_tokl): byte 0 luma mode (bits 0-2), chroma mode (3-4),
// skip (5); byte 1 segment; bytes 4-7 the non-zero mask; 8-15 the I4 sub-modes
// as nibbles; halfwords 8.. the level start of each block 0-23 and (24) the
// end; from byte ZW_DREC_HDR the levels in zigzag order up to each block's last
// non-zero one, Y2's first ([0, start[0])).  drec_lv: the level at natural
// index n of the block whose levels are [s0, s1).
DI int drec_lv(const uint8_t* rb, int s0, int s1, int n)
{
    const int idx = s0 + izz_of(n);
    const int v = ((const int16_t*)(rb + ZW_DREC_HDR))[idx];  // (past the record: LDS garbage, masked)
    return idx < s1 ? v : 0;
}
DI int drec_start(const uint8_t* rb, int b) { return ((const uint16_t*)(rb + 16))[b]; }

// ---------------------------------------------------------------------------
// Loop filter (decoder/loop_filter.rs) on LDS-staged neighbourhoods.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int c8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
__device__ __forceinline__ int u2s(int v) { return v - 128; }
__device__ __forceinline__ uint8_t s2u(int v) { return (uint8_t)(c8(v) + 128); }

// One edge of one line, branch-free (loop_filter.rs): the eight pixels across
// the edge, p3 p2 p1 p0 | q0 q1 q2 q3, as unsigned values.  KIND 0: simple
// filter (simple_segment), 1: inner edge (subblock_filter), 2: macroblock edge
// (macroblock_filter).  en: the edge is filtered on this line at all.
template <int KIND>
__device__ __forceinline__ void lf_edge(bool en, int ht, int il, int el, int& p3, int& p2, int& p1, int& p0, int& q0,
                                        int& q1, int& q2, int& q3)
{
    const int P1 = u2s(p1), P0 = u2s(p0), Q0 = u2s(q0), Q1 = u2s(q1);
    const bool th = iabs(p0 - q0) * 2 + (iabs(p1 - q1) >> 1) <= el;
    bool on = en && th;
    bool hev = false;
    if (KIND != 0) {
        on = on && iabs(p3 - p2) <= il && iabs(p2 - p1) <= il && iabs(p1 - p0) <= il && iabs(q3 - q2) <= il &&
             iabs(q2 - q1) <= il && iabs(q1 - q0) <= il;
        hev = iabs(p1 - p0) > ht || iabs(q1 - q0) > ht;
    }
    // common_adjust (use_outer_taps = simple || hev || the mb edge's hev branch)
    const bool outer = KIND == 0 || hev;
    int a = c8(csel(outer, c8(P1 - Q1), 0) + 3 * (Q0 - P0));
    const int b3 = c8(a + 3) >> 3;
    a = c8(a + 4) >> 3;
    int n_p0 = s2u(P0 + b3), n_q0 = s2u(Q0 - a), n_p1 = p1, n_q1 = q1, n_p2 = p2, n_q2 = q2;
    if (KIND == 1) {
        const int a2 = (a + 1) >> 1;
        n_p1 = csel(hev, p1, s2u(P1 + a2));
        n_q1 = csel(hev, q1, s2u(Q1 - a2));
    } else if (KIND == 2) {
        const int w = c8(c8(P1 - Q1) + 3 * (Q0 - P0));
        const int a27 = c8((27 * w + 63) >> 7), a18 = c8((18 * w + 63) >> 7), a9 = c8((9 * w + 63) >> 7);
        n_p0 = csel(hev, n_p0, s2u(P0 + a27));
        n_q0 = csel(hev, n_q0, s2u(Q0 - a27));
        n_p1 = csel(hev, p1, s2u(P1 + a18));
        n_q1 = csel(hev, q1, s2u(Q1 - a18));
        n_p2 = csel(hev, p2, s2u(u2s(p2) + a9));
        n_q2 = csel(hev, q2, s2u(u2s(q2) - a9));
    }
    p0 = csel(on, n_p0, p0);
    q0 = csel(on, n_q0, q0);
    if (KIND != 0) {
        p1 = csel(on, n_p1, p1);
        q1 = csel(on, n_q1, q1);
    }
    if (KIND == 2) {
        p2 = csel(on, n_p2, p2);
        q2 = csel(on, n_q2, q2);
    }
}

// The edges of one line in the reference's order: v[i] is the pixel at offset
// i - 4 from the MB origin along the line (the 4 before it belong to the
// left / upper neighbour).  The MB edge sits at 4, the inner edges at 8, 12, 16
// (chroma: 8 only, en12 false).
template <bool SIMPLE>
__device__ __forceinline__ void lf_line(int* v, bool en_mb, bool en_in, bool en12, int ht, int il, int mbe, int sube)
{
    if (SIMPLE) {
        lf_edge<0>(en_mb, ht, il, mbe, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
        for (int e = 8; e <= 16; e += 4)
            lf_edge<0>(en_in && (e == 8 || en12), ht, il, sube, v[e - 4], v[e - 3], v[e - 2], v[e - 1], v[e], v[e + 1],
                       v[e + 2], v[e + 3]);
    } else {
        lf_edge<2>(en_mb, ht, il, mbe, v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
#pragma unroll
        for (int e = 8; e <= 16; e += 4)
            lf_edge<1>(en_in && (e == 8 || en12), ht, il, sube, v[e - 4], v[e - 3], v[e - 2], v[e - 1], v[e], v[e + 1],
                       v[e + 2], v[e + 3]);
    }
}

#define LFY 20   // luma staging: rows/cols -4..15 around the MB
#define LFC 12   // chroma staging: -4..7

struct LfLds {
    uint8_t y[LFY * LFY];
    uint8_t u[LFC * LFC], v[LFC * LFC];
    uint8_t pad[8];  // the last chroma row's 5-word read stays inside the tile
};

// The filtering of one staged tile by 32 lanes (hl = lane in the group):
// lines 0..15 luma, 16..23 U, 24..31 V.  Phase A: the vertical edges (left MB
// edge, then x = 4, 8, 12), one row per lane; phase B: the horizontal edges
// (top MB edge, then y = 4, 8, 12), one column per lane.  en: this group filters
// (lanes with en false run the same code on a valid line and store nothing).
__device__ __forceinline__ void lf_filter_tile(LfLds* L, int hl, bool en, bool simple, bool chroma, bool left_edge,
                                               bool top_edge, bool inner, int ht, int il, int mbe, int sube)
{
    const bool isy = hl < 16, isu = hl >= 16 && hl < 24;
    const bool act = en && (isy || chroma);
    const int li = isy ? hl : (hl - 16) & 7;
    uint8_t* buf = isy ? L->y : (isu ? L->u : L->v);
    const int W_ = isy ? LFY : LFC;
    {
        uint32_t* row = (uint32_t*)(buf + (li + 4) * W_);
        uint32_t w[5];
#pragma unroll
        for (int k = 0; k < 5; k++) w[k] = row[k];  // (chroma: words 3-4 are the next row's, never filtered)
        int v[20];
#pragma unroll
        for (int k = 0; k < 20; k++) v[k] = (int)((w[k >> 2] >> (8 * (k & 3))) & 255u);
        if (simple) lf_line<true>(v, act && left_edge, act && inner, isy, ht, il, mbe, sube);
        else lf_line<false>(v, act && left_edge, act && inner, isy, ht, il, mbe, sube);
#pragma unroll
        for (int k = 0; k < 5; k++)
            w[k] = (uint32_t)v[4 * k] | ((uint32_t)v[4 * k + 1] << 8) | ((uint32_t)v[4 * k + 2] << 16) |
                   ((uint32_t)v[4 * k + 3] << 24);
        if (act) {
            row[0] = w[0];
            row[1] = w[1];
            row[2] = w[2];
            if (isy) {
                row[3] = w[3];
                row[4] = w[4];
            }
        }
    }
    wsync();
    {
        uint8_t* col = buf + 4 + li;
        const int kmax = isy ? 19 : 11;
        int v[20];
#pragma unroll
        for (int k = 0; k < 20; k++) v[k] = col[min(k, kmax) * W_];
        if (simple) lf_line<true>(v, act && top_edge, act && inner, isy, ht, il, mbe, sube);
        else lf_line<false>(v, act && top_edge, act && inner, isy, ht, il, mbe, sube);
        if (act) {
#pragma unroll
            for (int k = 1; k <= 17; k++)
                if (k <= 9 || isy) col[k * W_] = (uint8_t)v[k];
        }
    }
    wsync();
}

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
// (buffer-op helpers brsrc / bld* / bst* and ZW_OOB: zw_dev.h)

// pub() runs once the rows the MB row below reads (luma 12..15, chroma 4..7 of
// this tile) are stored; the rest of the write-back follows it.
// !XCU: those rows go to the workgroup's LDS hand-off rows hy / hu / hv (4 rows
// each, plane-wide) instead of global memory, and the row below writes them
// out as its rows -4..-1 (always, filtered or not); only the frame's last MB row
// (last) stores its own rows 12..15.  So no two waves store the same bytes.
template <bool XCU, class PUB>
__device__ __forceinline__ void lf_tile(LfLds* L, int lane, const ZwFilterParams& F, uint8_t* Yf, uint8_t* Uf,
                                        uint8_t* Vf, int ys, int cs, int mbx, int mby, int i4, int seg, int skip,
                                        int nzd, uint32_t cy, uint32_t cc, uint8_t* hy, uint8_t* hu, uint8_t* hv,
                                        bool last, PUB&& pub)
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
            ((uint32_t*)(L->y + r * LFY + 4))[w] =
                XCU ? ld(Yf + (size_t)(y0 - 4 + r) * ys + x0 + 4 * w) : *(const uint32_t*)(hy + r * ys + x0 + 4 * w);
        } else if (chroma && lane >= 32 && lane < 48) {
            const int t = lane - 32, pl = t >> 3, r = (t >> 1) & 3, w = t & 1;
            ((uint32_t*)((pl ? L->v : L->u) + r * LFC + 4))[w] =
                XCU ? ld((pl ? Vf : Uf) + (size_t)(mby * 8 - 4 + r) * cs + mbx * 8 + 4 * w)
                    : *(const uint32_t*)((pl ? hv : hu) + r * cs + mbx * 8 + 4 * w);
        }
    }
    wsync();
    if (lvl != 0)
        lf_filter_tile(L, lane & 31, lane < 32, F.filter_type != 0, chroma, mbx > 0, mby > 0, i4 || (!skip && nzd), ht, il,
                       (lvl + 2) * 2 + il, lvl * 2 + il);
    const bool wb = lvl != 0;
    auto tile_y = [&](int r, int w) { return ((const uint32_t*)(L->y + (r + 4) * LFY))[w + 1]; };
    auto tile_c = [&](int pl, int r, int w) { return ((const uint32_t*)((pl ? L->v : L->u) + (r + 4) * LFC))[w + 1]; };
    if (XCU) {
        // write back: luma 20 rows x 5 words, chroma 2 x 12 rows x 3 words (inside the frame);
        // part 0: the rows the MB row below reads, part 1: the others
        for (int part = 0; part < 2; part++) {
            if (wb) {
                for (int t = lane; t < LFY * 5; t += 64) {
                    const int r = t / 5 - 4, w = t % 5 - 1;
                    if ((r >= 12) == (part == 0) && y0 + r >= 0 && x0 + 4 * w >= 0)
                        st(Yf + (size_t)(y0 + r) * ys + x0 + 4 * w, tile_y(r, w));
                }
                if (chroma) {  // (the simple filter leaves chroma alone)
                    for (int t = lane; t < 2 * LFC * 3; t += 64) {
                        const int pl = t / (LFC * 3), rr = t % (LFC * 3), r = rr / 3 - 4, w = rr % 3 - 1;
                        if ((r >= 4) == (part == 0) && mby * 8 + r >= 0 && mbx * 8 + 4 * w >= 0)
                            st((pl ? Vf : Uf) + (size_t)(mby * 8 + r) * cs + mbx * 8 + 4 * w, tile_c(pl, r, w));
                    }
                }
            }
            if (part == 0) pub();
        }
    } else {
        // hand-off rows (luma rows 12..15, chroma 4..7 with the carried columns), then publish
        if (lane < 20) {
            const int r = 12 + lane / 5, w = lane % 5 - 1;
            if (x0 + 4 * w >= 0) *(uint32_t*)(hy + (r - 12) * ys + x0 + 4 * w) = tile_y(r, w);
        } else if (chroma && lane >= 32 && lane < 56) {
            const int t = lane - 32, pl = t / 12, rr = t % 12, r = 4 + rr / 3, w = rr % 3 - 1;
            if (mbx * 8 + 4 * w >= 0) *(uint32_t*)((pl ? hv : hu) + (r - 4) * cs + mbx * 8 + 4 * w) = tile_c(pl, r, w);
        }
        pub();
        // global: rows -4..-1 always (the row above left them to this row), rows 0..11 when
        // filtered, rows 12..15 when filtered in the last MB row
        for (int t = lane; t < LFY * 5; t += 64) {
            const int r = t / 5 - 4, w = t % 5 - 1;
            const bool need = r < 0 ? mby > 0 : (wb && (r < 12 || last));
            if (need && x0 + 4 * w >= 0) st(Yf + (size_t)(y0 + r) * ys + x0 + 4 * w, tile_y(r, w));
        }
        if (chroma) {
            for (int t = lane; t < 2 * LFC * 3; t += 64) {
                const int pl = t / (LFC * 3), rr = t % (LFC * 3), r = rr / 3 - 4, w = rr % 3 - 1;
                const bool need = r < 0 ? mby > 0 : (wb && (r < 4 || last));
                if (need && mbx * 8 + 4 * w >= 0)
                    st((pl ? Vf : Uf) + (size_t)(mby * 8 + r) * cs + mbx * 8 + 4 * w, tile_c(pl, r, w));
            }
        }
    }
    wsync();
}

// idct16_exact (zw_dev.h; transform_simd_intrinsics.rs:478, exact i16
// semantics) in quad form: lane q of the quad holds column q of the block
// (x_r = element (r, q)) and gets row q of the result.  The column pass runs in
// the lane; the transpose is the quad's i16 pairs broadcast by DPP.
DI void idct_quad_exact(int x0, int x1, int x2, int x3, int q, int o[4])
{
    x0 = sat16(x0);
    x1 = sat16(x1);
    x2 = sat16(x2);
    x3 = sat16(x3);
    const int a = w16(x0 + x2), bb = w16(x0 - x2);
    const int c = w16(w16(x1 - x3) + w16(mulhi16(x1, -30068) - mulhi16(x3, 20091)));
    const int d = w16(w16(x1 + x3) + w16(mulhi16(x1, 20091) + mulhi16(x3, -30068)));
    // rows 0, 1 of column q in lo, rows 2, 3 in hi (pack_lo keeps the low 16 bits: the i16 wrap)
    const uint32_t lo = pack_lo(a + d, bb + c), hi = pack_lo(bb - c, a - d);
    const bool upper = q >= 2;
    const uint32_t off = 16u * (uint32_t)(q & 1);
    // (csel, not ?: -- a select of two DPP results may be folded into one DPP of a select)
    const int y0 = __builtin_amdgcn_sbfe(csel(upper, qb0((int)hi), qb0((int)lo)), off, 16);
    const int y1 = __builtin_amdgcn_sbfe(csel(upper, qb1((int)hi), qb1((int)lo)), off, 16);
    const int y2 = __builtin_amdgcn_sbfe(csel(upper, qb2((int)hi), qb2((int)lo)), off, 16);
    const int y3 = __builtin_amdgcn_sbfe(csel(upper, qb3((int)hi), qb3((int)lo)), off, 16);
    const int dc = w16(y0 + 4);
    const int A = w16(dc + y2), B = w16(dc - y2);
    const int C = w16(w16(y1 - y3) + w16(mulhi16(y1, -30068) - mulhi16(y3, 20091)));
    const int D = w16(w16(y1 + y3) + w16(mulhi16(y1, 20091) + mulhi16(y3, -30068)));
    o[0] = w16(A + D) >> 3;
    o[1] = w16(B + C) >> 3;
    o[2] = w16(B - C) >> 3;
    o[3] = w16(A - D) >> 3;
}

// Row q of a 4x4 block: residual (full iDCT when the block's token run was
// non-empty, else the DC-only (c0 + 4) >> 3, vp8.rs:1110-1117) plus the
// prediction of mode m (0 DC, 1 V, 2 H, 3 TM; predict_* prediction.rs:164-324)
// from the top word T (the 4 pixels above the block's columns), the left pixel
// L of this row, the corner P and the DC value; returns the 4 pixels as a word.
// any_nz: some block of the wave has a non-empty run (else the iDCT is skipped).
DI uint32_t recon_row_quad(const int x[4], int q, bool nz, bool any_nz, int c0, int m, uint32_t T, int L, int P, int dcv)
{
    int o[4] = {0, 0, 0, 0};
    if (any_nz) idct_quad_exact(x[0], x[1], x[2], x[3], q, o);
    const int d = (c0 + 4) >> 3;
    const uint32_t R01 = nz ? pack_lo(o[0], o[1]) : pack_lo(d, d);
    const uint32_t R32 = nz ? pack_lo(o[3], o[2]) : pack_lo(d, d);
    const uint32_t t01 = __builtin_amdgcn_perm(0u, T, 0x0c010c00u), t32 = __builtin_amdgcn_perm(0u, T, 0x0c020c03u);
    uint32_t p01, p32;
    if (m == 0) {
        p01 = p32 = (uint32_t)dcv * 0x10001u;
    } else if (m == 1) {
        p01 = t01;
        p32 = t32;
    } else if (m == 2) {
        p01 = p32 = (uint32_t)L * 0x10001u;
    } else {
        const uint32_t dd = ((uint32_t)(L - P) & 0xffffu) * 0x10001u;
        p01 = clamp_pk(add_pk(t01, dd));
        p32 = clamp_pk(add_pk(t32, dd));
    }
    const uint32_t r01 = clamp_pk(add_pk(R01, p01)), r32 = clamp_pk(add_pk(R32, p32));
    return __builtin_amdgcn_perm(r32, r01, 0x04060200u);
}

// One MB row of the reconstruction (shared by the one-workgroup-per-frame
// kernel and the row-parallel one).  wait(n): block until the row above has
// finished n MBs; pub(n): this row has finished n MBs.  XCU: the row above may
// run on another CU / XCD, so its bottom pixels are exchanged through the
// global border rows gty/gtu/gtv with sc1 stores and loads; otherwise
// gty/gtu/gtv are the workgroup's LDS border rows.
//
// Lane layout (I16 luma, chroma): lane = 4 b + q, block b, pixel row q of the
// block; the lane's row is one word of the plane.  The borders come straight
// from the top row (words) and the left column; only I4 MBs, whose
// sub-blocks chain through their own reconstruction, build the LDS work area
// ws and run the 16 sub-blocks in turn.
template <bool XCU, class WAIT, class PUB>
__device__ __forceinline__ void dec_recon_row(const uint8_t* __restrict__ recs, const uint32_t* __restrict__ moff,
                                              const uint64_t* __restrict__ fbase, const ZwDecQuant* __restrict__ quant, uint8_t* Y,
                                              uint8_t* U, uint8_t* V, uint8_t* flags, int f, int mbw, int mbh,
                                              size_t ysz, size_t csz, int mby, DecLds* W, uint8_t* gty, uint8_t* gtu,
                                              uint8_t* gtv, uint8_t* tiles, WAIT&& wait, PUB&& pub)
{
    const int lane0 = threadIdx.x & 63;
    const int ys = mbw * 16, cs = mbw * 8;
    const size_t nmb = (size_t)mbw * mbh;
    const bool above = mby != 0;
    const int lane = lane0;  // (outside the MB loop)
    if (lane < 20) W->left_y[lane] = 129;
    if (lane < 12) W->left_u[lane] = W->left_v[lane] = 129;
    wsync();
    // packed records of this row: MB x spans [fmo[x], fmo[x + 1]) bytes of the frame's
    // records.  Every global access of an MB step is an unconditional buffer op (ZW_OOB
    // for the lanes that have nothing to move), so the step's stores never join the
    // wait for the next MB's prefetch.
    const uint32_t* fmo_f = moff + (size_t)f * (nmb + 1);
    const uint32_t fbytes = (uint32_t)__builtin_amdgcn_readfirstlane((int)fmo_f[nmb]);
    const __amdgpu_buffer_rsrc_t rrec = brsrc(recs + fbase[f], fbytes);
    const __amdgpu_buffer_rsrc_t rmo = brsrc(fmo_f, (uint32_t)(nmb + 1) * 4u);
    const __amdgpu_buffer_rsrc_t ryp = brsrc(Y + (size_t)f * ysz, (uint32_t)ysz);
    const __amdgpu_buffer_rsrc_t rup = brsrc(U + (size_t)f * csz, (uint32_t)csz);
    const __amdgpu_buffer_rsrc_t rvp = brsrc(V + (size_t)f * csz, (uint32_t)csz);
    const __amdgpu_buffer_rsrc_t rfl = brsrc(flags + (size_t)f * nmb * 4, (uint32_t)nmb * 4u);
    // !XCU: the MBs go to the frame's tiles (ZW_DEC_TILE bytes each: luma 16 x 16, U, V 8 x 8,
    // row-major), whole cache lines; k_loopfilter reads them and writes the planes
    const __amdgpu_buffer_rsrc_t rty = brsrc(XCU ? (const uint8_t*)Y : tiles + (size_t)f * nmb * ZW_DEC_TILE,
                                             XCU ? 0u : (uint32_t)(nmb * ZW_DEC_TILE));
    const uint32_t row0 = (uint32_t)(mby * mbw);
    auto load_rec = [&](int ln, uint32_t a, uint32_t e) -> uint4 {
        const uint32_t o = a + 16u * (uint32_t)ln;
        const zu4 v = bld128(rrec, ln < 55 && o < e ? o : ZW_OOB);
        return make_uint4(v.x, v.y, v.z, v.w);
    };
    uint32_t a1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)fmo_f[row0 + 1]);
    uint32_t a2 = mbw >= 2 ? (uint32_t)__builtin_amdgcn_readfirstlane((int)fmo_f[row0 + 2]) : 0u;
    uint4 nxt = load_rec(lane, (uint32_t)__builtin_amdgcn_readfirstlane((int)fmo_f[row0]), a1);
    for (int mbx = 0; mbx < mbw; mbx++) {
        // the lane's roles, recomputed per MB from an opaque copy of the lane id:
        // hoisted out of the loop, their exec masks were spilled to VGPR lanes
        // and reloaded with v_readlane every MB
        const int lane = pin(lane0);
        const uint4 cur = nxt;
        nxt = load_rec(mbx + 1 < mbw ? lane : 64, (uint32_t)__builtin_amdgcn_readfirstlane((int)a1),
                       (uint32_t)__builtin_amdgcn_readfirstlane((int)a2));  // MB x+1
        a1 = a2;
        // (a vector load: a scalar one would be waited for with lgkmcnt(0) by the
        // next LDS access, a full memory round trip per MB)
        a2 = bld32(rmo, mbx + 3 <= mbw ? (row0 + (uint32_t)mbx + 3u) * 4u : ZW_OOB);
#ifndef ZW_EXP_NO_WAIT
        if (mby > 0) wait(min(mbx + 2, mbw));
#endif
        if (XCU && mby > 0) {  // the row above's bottom pixels (written by another workgroup)
            if (lane < 8) W->twy[lane] = ld_sc1(gty + mbx * 16 + 4 * lane);
            else if (lane < 10) W->twu[lane - 8] = ld_sc1(gtu + mbx * 8 + 4 * (lane - 8));
            else if (lane < 12) W->twv[lane - 10] = ld_sc1(gtv + mbx * 8 + 4 * (lane - 10));
        }
        const uint8_t* top_y = XCU ? (const uint8_t*)W->twy : gty + mbx * 16;
        const uint8_t* top_u = XCU ? (const uint8_t*)W->twu : gtu + mbx * 8;
        const uint8_t* top_v = XCU ? (const uint8_t*)W->twv : gtv + mbx * 8;
        if (lane < 55) W->rec[lane] = cur;
        wsync();
        const int ln = lane;
        const int b = ln >> 2, q = ln & 3, bx = b & 3, by = b >> 2;
        // chroma: lanes 0..31 (lanes 32..63 mirror them and store nothing)
        const int pl = (ln >> 4) & 1, cb = (ln >> 2) & 3, cbx = cb & 1, cby = cb >> 1;
        const uint8_t* rb = (const uint8_t*)W->rec;
        const uint32_t h0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)((const uint32_t*)rb)[0]);
        const int seg = (int)((h0 >> 8) & 3u), skip = (int)((h0 >> 5) & 1u);
        const ZwDecQuant& Q = quant[seg];  // the frame's LDS copy
        const int lm = (int)(h0 & 7u);
        const uint32_t nzm = (uint32_t)__builtin_amdgcn_readfirstlane((int)((const uint32_t*)rb)[1]);
        const bool left = mbx != 0;
        // ---- luma ----
        const uint32_t TW = above ? ((const uint32_t*)top_y)[bx] : 0x7f7f7f7fu;
        const int corner_y = (int)((uint32_t)__builtin_amdgcn_readlane((int)TW, 12) >> 24);  // top pixel 15: the next MB's corner
        uint32_t RW;
        int nzdct;
#ifdef ZW_EXP_NO_I4
        if (true) {
#else
        if (lm != 4) {
#endif
            // Y2 in group form (lane k = block k's DC after the iWHT), moved to the quads
            const int k = lane & 15;
            const int y2e = __builtin_amdgcn_readfirstlane(drec_start(rb, 0));  // Y2's levels come first: [0, start[0])
            int dc = 0;
            if (!skip && y2e > 0) {
                const int y2v = drec_lv(rb, 0, y2e, k) * (k ? Q.y2ac : Q.y2dc);
                dc = __builtin_amdgcn_ds_bpermute(4 * b, iwht_g(y2v, k));
            }
            const int s0 = drec_start(rb, b), s1 = drec_start(rb, b + 1);
            int x[4];
#pragma unroll
            for (int r = 0; r < 4; r++) x[r] = drec_lv(rb, s0, s1, 4 * r + q) * Q.yac;
            x[0] = csel(q == 0, dc, x[0]);
            const int L = left ? (int)W->left_y[1 + 4 * by + q] : 129;
            const int P = above ? (left ? (int)W->left_y[0] : 129) : 127;
            int dcv = 128;
            if (lm == 0) {  // DC predictor: the top row (lanes of blocks 0..3, q = 0) and the left column (bx = 0)
                int sv = (above && b < 4 && q == 0 ? (int)__builtin_amdgcn_sad_u8(TW, 0u, 0u) : 0) + (left && bx == 0 ? L : 0);
                sv = red16(sv);
                const int su = __builtin_amdgcn_readlane(sv, 0) + __builtin_amdgcn_readlane(sv, 16) +
                               __builtin_amdgcn_readlane(sv, 32) + __builtin_amdgcn_readlane(sv, 48);
                const int shf = 3 + above + left;
                if (above || left) dcv = (su + (1 << (shf - 1))) >> shf;
            }
            const bool nz = (nzm >> b) & 1u;
            RW = recon_row_quad(x, q, nz, (nzm & 0xffffu) != 0u, dc, lm, TW, L, P, dcv);
            nzdct = __any(dc != 0 || nz) ? 1 : 0;
        } else {
            // --- the 16 residuals in quad form first (they do not depend on the
            // prediction), then the sub-blocks' predictions in raster order ---
            {
                const int s0 = drec_start(rb, b), s1 = drec_start(rb, b + 1);
                int x[4];
#pragma unroll
                for (int r = 0; r < 4; r++) x[r] = drec_lv(rb, s0, s1, 4 * r + q) * (r == 0 && q == 0 ? Q.ydc : Q.yac);
                const int c0 = qb0(x[0]);
                const bool nz = (nzm >> b) & 1u;
                int o[4] = {0, 0, 0, 0};
                if ((nzm & 0xffffu) != 0u) idct_quad_exact(x[0], x[1], x[2], x[3], q, o);
                const int d = (c0 + 4) >> 3;  // DC-only: (c0 + 4) >> 3 (0 for c0 = 0)
                uint32_t* rp = (uint32_t*)&W->res4[b * 16 + q * 4];
                rp[0] = nz ? pack_lo(o[0], o[1]) : pack_lo(d, d);
                rp[1] = nz ? pack_lo(o[2], o[3]) : pack_lo(d, d);
                nzdct = __any(nz || c0 != 0) ? 1 : 0;
            }
            uint8_t* ws = W->ws;
            const uint8_t* ty = top_y - mbx * 16;
            if (lane < 32) {  // luma border (create_border_luma)
                int v;
                if (lane == 0) v = mby == 0 ? 127 : (mbx == 0 ? 129 : W->left_y[0]);
                else if (mby == 0) v = 127;
                else if (lane <= 16) v = ty[mbx * 16 + lane - 1];
                else if (mbx == mbw - 1) v = ty[mbx * 16 + 15];
                else v = ty[mbx * 16 + lane - 1];
                ws[lane] = (uint8_t)v;
                if (lane >= 17 && lane < 21) ws[4 * ZW_BPS + lane] = ws[8 * ZW_BPS + lane] = ws[12 * ZW_BPS + lane] = (uint8_t)v;
            } else if (lane < 48) {
                ws[(lane - 31) * ZW_BPS] = mbx == 0 ? 129 : W->left_y[lane - 31];
            }
            wsync();
            // value vector V (lane l < 39 holds V[l]): E(a) + wb E(b) + wc E(c) rounded, or the DC sum
            int ja = lane, jb = 0, jc = 0, wb = 0, wc = 0, rnd = 0, sh = 0;
            if (lane >= 13 && lane < 24) { ja = lane - 13; jb = ja + 1; jc = ja + 2; wb = 2; wc = 1; rnd = 2; sh = 2; }
            else if (lane >= 24 && lane < 36) { ja = lane - 24; jb = ja + 1; wb = 1; rnd = 1; sh = 1; }
            else if (lane == 36) { ja = 11; jb = 12; wb = 3; rnd = 2; sh = 2; }
            else if (lane == 37) { ja = 1; jb = 0; wb = 3; rnd = 2; sh = 2; }
            else if (lane >= 38) ja = 0;
            const int oa = i4_eoff(ja), ob = i4_eoff(jb), oc = i4_eoff(jc);
            const bool dcl = lane < 4 || (lane >= 5 && lane < 9);
            const int k = lane & 15;
            const uint64_t bp = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((const uint32_t*)rb)[2]) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((const uint32_t*)rb)[3]) << 32);
            for (int i = 0; i < 16; i++) {
                const int x0 = (i & 3) * 4 + 1, y0 = (i >> 2) * 4 + 1, base = y0 * ZW_BPS + x0;
                const int mode = (int)((bp >> (4 * i)) & 15u);
                const int idx = W->i4idx[mode][k];
                const int res = W->res4[i * 16 + k];
                const int ea = ws[base + oa], eb = ws[base + ob], ec = ws[base + oc];
                const int V = (ea + wb * eb + wc * ec + rnd) >> sh;
                const int dsum = red16(dcl ? ea : 0);
                const int dcv = (__builtin_amdgcn_readlane(dsum, 0) + 4) >> 3;
                const int vi = __builtin_amdgcn_ds_bpermute(4 * (idx >= 254 ? 0 : idx), V);
                const int tl = __builtin_amdgcn_ds_bpermute(4 * (3 - (k >> 2)), V);
                const int tt = __builtin_amdgcn_ds_bpermute(4 * (5 + (k & 3)), V);
                const int P = __builtin_amdgcn_readlane(V, 4);
                const int pred = idx == 254 ? clamp255(tl + tt - P) : (idx == 255 ? dcv : vi);
                if (lane < 16) ws[base + (k >> 2) * ZW_BPS + (k & 3)] = (uint8_t)clamp255(pred + res);
                wsync();
            }
            const uint8_t* pr = ws + (4 * by + q + 1) * ZW_BPS + 1 + 4 * bx;
            RW = (uint32_t)pr[0] | ((uint32_t)pr[1] << 8) | ((uint32_t)pr[2] << 16) | ((uint32_t)pr[3] << 24);
        }
        // ---- chroma ----
        uint32_t RC;
        {
            const uint8_t* tc = pl ? top_v : top_u;
            const uint8_t* lc = pl ? W->left_v : W->left_u;
            const uint32_t TC = above ? ((const uint32_t*)tc)[cbx] : 0x7f7f7f7fu;
            const int L = left ? (int)lc[1 + 4 * cby + q] : 129;
            const int P = above ? (left ? (int)lc[0] : 129) : 127;
            const int cm = (int)((h0 >> 3) & 3u);
            int dcv = 128;
            if (cm == 0) {
                int sv = (above && cby == 0 && q == 0 ? (int)__builtin_amdgcn_sad_u8(TC, 0u, 0u) : 0) + (left && cbx == 0 ? L : 0);
                sv = red16(sv);  // the plane's 16-lane group
                const int shf = 2 + above + left;
                if (above || left) dcv = (sv + (1 << (shf - 1))) >> shf;
            }
            const int cbk = 16 + 4 * pl + cb;
            const int s0 = drec_start(rb, cbk), s1 = drec_start(rb, cbk + 1);
            int x[4];
#pragma unroll
            for (int r = 0; r < 4; r++) x[r] = drec_lv(rb, s0, s1, 4 * r + q) * (r == 0 && q == 0 ? Q.uvdc : Q.uvac);
            const int c0 = qb0(x[0]);
            const bool nz = (nzm >> cbk) & 1u;
            RC = recon_row_quad(x, q, nz, (nzm >> 16) != 0u, c0, cm, TC, L, P, dcv);
            nzdct |= __any(lane < 32 && (c0 != 0 || nz)) ? 1 : 0;
        }
        const int corner_u = (int)((uint32_t)__builtin_amdgcn_readlane(above ? (int)((const uint32_t*)top_u)[1] : 0x7f7f7f7f, 0) >> 24);
        const int corner_v = (int)((uint32_t)__builtin_amdgcn_readlane(above ? (int)((const uint32_t*)top_v)[1] : 0x7f7f7f7f, 0) >> 24);
        wsync();
        // ---- borders for the next MB and the row below, output ----
        if (bx == 3) W->left_y[1 + 4 * by + q] = (uint8_t)(RW >> 24);
        if (lane == 0) {
            W->left_y[0] = (uint8_t)corner_y;
            W->left_u[0] = (uint8_t)corner_u;
            W->left_v[0] = (uint8_t)corner_v;
        }
        if (lane < 32 && cbx == 1) (pl ? W->left_v : W->left_u)[1 + 4 * cby + q] = (uint8_t)(RC >> 24);
        if (XCU) {  // bottom rows for the row below (sc1), then publish, then the planes
            if (by == 3 && q == 3) st_sc1(gty + mbx * 16 + 4 * bx, RW);
            if (lane < 32 && cby == 1 && q == 3) st_sc1((pl ? gtv : gtu) + mbx * 8 + 4 * cbx, RC);
            pub(mbx + 1);  // the row below needs only the border: publish before the plane stores
        } else {  // LDS border rows; the publish waits for LDS only, not for the plane stores
            if (by == 3 && q == 3) *(uint32_t*)(gty + mbx * 16 + 4 * bx) = RW;
            if (lane < 32 && cby == 1 && q == 3) *(uint32_t*)((pl ? gtv : gtu) + mbx * 8 + 4 * cbx) = RC;
            pub(mbx + 1);
        }
        if (XCU) {
            const uint32_t oy = (uint32_t)((mby * 16 + 4 * by + q) * ys + mbx * 16 + 4 * bx);
            const uint32_t oc = (uint32_t)((mby * 8 + 4 * cby + q) * cs + mbx * 8 + 4 * cbx);
            bst32(RW, ryp, oy);
            bst32(RC, rup, lane < 32 && !pl ? oc : ZW_OOB);
            bst32(RC, rvp, lane < 32 && pl ? oc : ZW_OOB);
        } else {
            const uint32_t tb = (row0 + (uint32_t)mbx) * ZW_DEC_TILE;
            bst32(RW, rty, tb + (uint32_t)((4 * by + q) * 16 + 4 * bx));
            bst32(RC, rty, lane < 32 ? tb + 256u + (uint32_t)(pl * 64 + (4 * cby + q) * 8 + 4 * cbx) : ZW_OOB);
        }
        {
            const int v = lane == 0 ? lm : (lane == 1 ? seg : (lane == 2 ? skip : nzdct));
            bst8((uint32_t)v, rfl, lane < 4 ? (row0 + (uint32_t)mbx) * 4u + (uint32_t)lane : ZW_OOB);
        }
        wsync();
    }
}

__global__ __launch_bounds__(WGD) __attribute__((amdgpu_waves_per_eu(NWD / 4, NWD / 4))) void k_dec_recon(const uint8_t* __restrict__ recs,
                                                              const uint32_t* __restrict__ moff,
                                                              const uint64_t* __restrict__ fbase,
                                                              const ZwDecQuant* __restrict__ quant, uint8_t* Y, uint8_t* U,
                                                              uint8_t* V, uint8_t* flags, int mbw, int mbh, size_t ysz,
                                                              size_t csz, uint8_t* tiles)
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
    DecLds* W = (DecLds*)((uint8_t*)Wall + ((sizeof(DecLds) + 15) & ~(size_t)15) * wv);
    for (int i = lane; i < 160; i += 64) (&W->i4idx[0][0])[i] = (&d_I4_IDX[0][0])[i];
    if (lane < 24) ((int32_t*)W->q)[lane] = ((const int32_t*)(quant + (size_t)f * 4))[lane];
    for (int i = threadIdx.x; i < mbw * 16 + 48; i += WGD) top_y[i] = 127;
    for (int i = threadIdx.x; i < mbw * 8 + 48; i += WGD) top_u[i] = top_v[i] = 127;
    if (threadIdx.x < NWD) progress[threadIdx.x] = -1;
    __syncthreads();
    for (int mby = wv; mby < mbh; mby += NWD) {
        dec_recon_row<false>(
            recs, moff, fbase, W->q, Y, U, V, flags, f, mbw, mbh, ysz, csz, mby, W, top_y, top_u, top_v, tiles,
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

__global__ __launch_bounds__(64) void k_dec_recon_rows(const uint8_t* __restrict__ recs,
                                                       const uint32_t* __restrict__ moff,
                                                       const uint64_t* __restrict__ fbase,
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
        dec_recon_row<true>(
            recs, moff, fbase, W->q, Y, U, V, flags, f, mbw, mbh, ysz, csz, mby, W, gty, gtu, gtv, nullptr,
            [&](int need) { row_wait(&prog[mby - 1], need, &rs[2], seen); },
            [&](int done) { row_publish(&prog[mby], done); });
    }
}

// One MB of the batch loop filter on one half-wave (hl = lane in the half,
// 0..31; on: the half has an MB this step).  The tile is assembled from the
// prefetched interior (luma words hl and hl + 32: row w >> 2, word w & 3;
// chroma word hl: plane hl >> 4, row (hl >> 1) & 7, word hl & 1), the carried
// left columns and the LDS hand-off rows above; filtered; its rows 12..15
// (chroma 4..7) go to the hand-off rows, the rest to the planes (rows -4..-1
// always: the row above left them to this row; the last MB row also stores its
// own rows 12..15).  No two waves store the same bytes.
template <class PF>
// cmove: chroma is moved (tile -> planes) even when the simple filter leaves it alone.
__device__ __forceinline__ void lf_half(LfLds* L, int hl, bool on, const ZwFilterParams& F, __amdgpu_buffer_rsrc_t ry,
                                        __amdgpu_buffer_rsrc_t ru, __amdgpu_buffer_rsrc_t rv, int ys, int cs, int mbx,
                                        int mby, uint32_t fl, uint32_t cy0, uint32_t cy1, uint32_t cc, uint8_t* hy,
                                        uint8_t* hu, uint8_t* hv, bool last, bool cmove, PF&& prefetch)
{
    const bool chroma = cmove;  // (staging, hand-off and stores; the filter itself takes !F.filter_type)
    const int i4 = (fl & 255u) == 4u, seg = (int)((fl >> 8) & 3u), skip = (int)((fl >> 16) & 255u), nzd = (int)(fl >> 24);
    const int lvl = F.level[seg][i4], il = F.ilimit[seg][i4], ht = F.hev[seg][i4];
    const int x0 = mbx * 16, y0 = mby * 16;
    // ---- assemble the tile ----
    if (on && mbx > 0) {  // left 4 columns (rows -4..15) from the previous tile's columns 12..15
        if (hl < LFY) {
            uint32_t* row = (uint32_t*)(L->y + hl * LFY);
            row[0] = row[4];
        }
        if (chroma && hl < 2 * LFC) {
            uint32_t* row = (uint32_t*)((hl >= LFC ? L->v : L->u) + (hl % LFC) * LFC);
            row[0] = row[2];
        }
    }
    if (on) {
        ((uint32_t*)(L->y + (4 + (hl >> 2)) * LFY + 4))[hl & 3] = cy0;
        ((uint32_t*)(L->y + (12 + (hl >> 2)) * LFY + 4))[hl & 3] = cy1;
        if (chroma) ((uint32_t*)((((hl >> 4) & 1) ? L->v : L->u) + (4 + ((hl >> 1) & 7)) * LFC + 4))[hl & 1] = cc;
        if (mby > 0) {  // the 4 rows above from the hand-off rows: luma hl < 16, chroma hl >= 16
            if (hl < 16) {
                const int r = hl >> 2, w = hl & 3;
                ((uint32_t*)(L->y + r * LFY + 4))[w] = *(const uint32_t*)(hy + r * ys + x0 + 4 * w);
            } else if (chroma) {
                const int t = hl - 16, pl = t >> 3, r = (t >> 1) & 3, w = t & 1;
                ((uint32_t*)((pl ? L->v : L->u) + r * LFC + 4))[w] = *(const uint32_t*)((pl ? hv : hu) + r * cs + mbx * 8 + 4 * w);
            }
        }
    }
    prefetch();  // the next step's interior: issued once this one's is in LDS (fewer live registers)
    wsync();
#ifndef ZW_EXP_NO_LF
    lf_filter_tile(L, hl, on && lvl != 0, F.filter_type != 0, !F.filter_type, mbx > 0, mby > 0, i4 || (!skip && nzd),
                   ht, il, (lvl + 2) * 2 + il, lvl * 2 + il);
#endif
    auto tile_y = [&](int r, int w) { return ((const uint32_t*)(L->y + (r + 4) * LFY))[w + 1]; };
    auto tile_c = [&](int pl, int r, int w) { return ((const uint32_t*)((pl ? L->v : L->u) + (r + 4) * LFC))[w + 1]; };
    // hand-off rows: luma rows 12..15 (20 words with the carried columns), chroma 4..7 (24)
    if (on && hl < 20) {
        const int r = 12 + hl / 5, w = hl % 5 - 1;
        if (x0 + 4 * w >= 0) *(uint32_t*)(hy + (r - 12) * ys + x0 + 4 * w) = tile_y(r, w);
    }
    if (on && chroma && hl < 24) {
        const int pl = hl / 12, rr = hl % 12, r = 4 + rr / 3, w = rr % 3 - 1;
        if (mbx * 8 + 4 * w >= 0) *(uint32_t*)((pl ? hv : hu) + (r - 4) * cs + mbx * 8 + 4 * w) = tile_c(pl, r, w);
    }
    const bool wb = lvl != 0;
#ifdef ZW_EXP_NO_WB
    return;
#endif
    // the planes, one tile row per lane (luma: a word for the carried columns + 16 bytes;
    // chroma: a word + 8 bytes): rows -4..-1 always (the row above left them to this
    // row), rows 0..11 (chroma 0..3) always (the planes get every byte from here), 12..15
    // (4..7) in the last MB row.  Every lane issues every store; the ones not wanted go to
    // ZW_OOB.
    (void)wb;
    {
        const int lr = min(hl, LFY - 1), r = lr - 4;
        const bool need = on && hl < LFY && (r < 0 ? mby > 0 : (r < 12 || last));
        const uint32_t* row = (const uint32_t*)(L->y + lr * LFY);
        const zu4 wv = {row[1], row[2], row[3], row[4]};
        const uint32_t off = (uint32_t)((y0 + r) * ys + x0);
        bst32(row[0], ry, need && mbx > 0 ? off - 4 : ZW_OOB);
        bst128(wv, ry, need ? off : ZW_OOB);
    }
    {
        const int lr = min(hl, 2 * LFC - 1), pl = lr >= LFC, rr = lr - LFC * pl, r = rr - 4;
        const bool need = on && chroma && hl < 2 * LFC && (r < 0 ? mby > 0 : (r < 4 || last));
        const uint32_t* row = (const uint32_t*)((pl ? L->v : L->u) + rr * LFC);
        const zu2 wv = {row[1], row[2]};
        const uint32_t off = (uint32_t)((mby * 8 + r) * cs + mbx * 8);
        bst32(row[0], ru, need && !pl && mbx > 0 ? off - 4 : ZW_OOB);
        bst64(wv, ru, need && !pl ? off : ZW_OOB);
        bst32(row[0], rv, need && pl && mbx > 0 ? off - 4 : ZW_OOB);
        bst64(wv, rv, need && pl ? off : ZW_OOB);
    }
}

// Batch loop filter: one workgroup per frame, NWD waves; wave wv takes MB-row
// pairs wv, wv + NWD, ...  A pair runs as one stream of steps: at step s the
// upper row (lanes 0..31) filters MB s and the lower row (lanes 32..63) MB
// s - 2 -- the x+2y wavefront inside the wave; the two tiles never overlap.
// Every lane does useful work, so a frame costs half the instructions and half
// the serial steps of one row per wave.  The next pair's upper row waits on the
// lower row's progress.  The rows hand over through LDS (hy/hu/hv: the last
// filtered MB row's bottom 4 rows, plane-wide).
// tiles: the batch reconstruction's MB tiles (ZW_DEC_TILE bytes per MB), or nullptr:
// the planes hold the unfiltered frame (the loop-filter-only entry point).
extern "C" __global__ __launch_bounds__(WGD) void k_loopfilter(uint8_t* Y, uint8_t* U, uint8_t* V,
                                                               const uint8_t* __restrict__ flags,
                                                               const ZwFilterParams* __restrict__ fp, size_t ysz,
                                                               size_t csz, const uint8_t* __restrict__ tiles)
{
    __shared__ __attribute__((aligned(16))) LfLds lds[NWD][2];
    __shared__ int progress[NWD];
    __shared__ ZwFilterParams Fs;
    extern __shared__ __attribute__((aligned(16))) uint8_t hand[];  // hand-off rows: 4 luma + 2 x 4 chroma
    const int f = blockIdx.x, wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, hl = lane & 31;
    if (threadIdx.x < sizeof(ZwFilterParams) / 4) ((uint32_t*)&Fs)[threadIdx.x] = ((const uint32_t*)(fp + f))[threadIdx.x];
    if (threadIdx.x < NWD) progress[threadIdx.x] = -1;
    __syncthreads();
    const ZwFilterParams& F = Fs;
    const int mbw = F.mbw, mbh = F.mbh, ys = mbw * 16, cs = mbw * 8;
    const size_t nmb = (size_t)mbw * mbh;
    uint8_t* hy = hand;
    uint8_t* hu = hand + 4 * ys;
    uint8_t* hv = hu + 4 * cs;
    LfLds* L = &lds[wv][h];
    uint8_t* Yf = Y + (size_t)f * ysz;
    uint8_t* Uf = U + (size_t)f * csz;
    uint8_t* Vf = V + (size_t)f * csz;
    const bool chroma = !F.filter_type || tiles != nullptr;  // chroma staged and stored (see lf_half)
    const __amdgpu_buffer_rsrc_t ry = brsrc(Yf, (uint32_t)ysz), ru = brsrc(Uf, (uint32_t)csz), rv = brsrc(Vf, (uint32_t)csz);
    const __amdgpu_buffer_rsrc_t rt = brsrc(tiles ? tiles + (size_t)f * nmb * ZW_DEC_TILE : (const uint8_t*)Yf,
                                            tiles ? (uint32_t)(nmb * ZW_DEC_TILE) : 0u);
    const __amdgpu_buffer_rsrc_t rf = brsrc(flags + (size_t)f * nmb * 4, (uint32_t)(nmb * 4));
    // the interior words and the flags of MB (mx, my) (every lane loads; invalid -> ZW_OOB -> 0)
    auto load = [&](bool valid, int my, int mx, uint32_t& y0w, uint32_t& y1w, uint32_t& cw, uint32_t& flw) {
#ifdef ZW_EXP_NO_LOAD
        y0w = y1w = cw = (uint32_t)(mx * 77 + hl); flw = 0x01000000u | (uint32_t)(mx & 1);
        return;
#endif
        // tiles: whole lines (luma words hl, hl + 32: rows hl >> 2 and 8 + (hl >> 2); chroma
        // word hl); else the planes.  The same four loads either way (a uniform choice of
        // resource and offsets, no branch: the waits stay counted)
        const bool t = tiles != nullptr, pv = (hl >> 4) & 1, cv = valid && chroma;
        const uint32_t tb = (uint32_t)(my * mbw + mx) * ZW_DEC_TILE + 4u * (uint32_t)hl;
        const uint32_t oy = (uint32_t)((my * 16 + (hl >> 2)) * ys + mx * 16 + 4 * (hl & 3));
        const uint32_t oc = (uint32_t)((my * 8 + ((hl >> 1) & 7)) * cs + mx * 8 + 4 * (hl & 1));
        y0w = bld32(t ? rt : ry, !valid ? ZW_OOB : (t ? tb : oy));
        y1w = bld32(t ? rt : ry, !valid ? ZW_OOB : (t ? tb + 128u : oy + 8u * (uint32_t)ys));
        cw = bld32(t ? rt : ru, !cv ? ZW_OOB : (t ? tb + 256u : (!pv ? oc : ZW_OOB))) |
             bld32(rv, cv && !t && pv ? oc : ZW_OOB);
        flw = bld32(rf, valid ? (uint32_t)((my * mbw + mx) * 4) : ZW_OOB);
    };
    for (int pr = wv; 2 * pr < mbh; pr += NWD) {
        const int my = 2 * pr + h;  // this half's MB row
        const bool rowok = my < mbh;
        uint32_t ny0 = 0, ny1 = 0, nc = 0, nfl = 0;
        load(rowok && h == 0, my, 0, ny0, ny1, nc, nfl);  // step 0: the lower half starts at step 2
        for (int st = 0; st < mbw + 2; st++) {
            const int mx = st - 2 * h;
            const bool on = rowok && mx >= 0 && mx < mbw;
            const uint32_t cy0 = ny0, cy1 = ny1, cc = nc, fl = nfl;
#ifndef ZW_EXP_NO_WAIT
            if (pr > 0 && st < mbw) dec_wait(progress, (pr - 1) % NWD, (pr - 1) * 65536 + min(st + 2, mbw));
#endif
            load(rowok && mx + 1 >= 0 && mx + 1 < mbw, my, mx + 1, ny0, ny1, nc, nfl);
            lf_half(L, hl, on, F, ry, ru, rv, ys, cs, mx, my, fl, cy0, cy1, cc, hy, hu, hv, my == mbh - 1, chroma, [] {});
            wsync();
            if (st >= 2) dec_publish(progress, wv, pr * 65536 + st - 1);  // the lower row has finished st - 1 MBs
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
                          (fl >> 16) & 255, fl >> 24, cy, cc, nullptr, nullptr, nullptr, false,
                          [&] { row_publish(&prog[mby], mbx + 1); });
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
// recs / moff / fbase: the packed MB records (zw_common.h ZW_DREC_*), each
// frame's MB byte offsets (nmb + 1 per frame) and each frame's base offset.
extern "C" hipError_t zwk_dec_rows(hipStream_t s, int phase, const uint8_t* recs, const uint32_t* moff,
                                   const uint64_t* fbase, const void* quant, uint8_t* Y, uint8_t* U, uint8_t* V,
                                   uint8_t* flags, const ZwFilterParams* fp, int mbw, int mbh, size_t ysz, size_t csz,
                                   int nframes, int* rowsync, uint8_t* borders, int rows)
{
    const int R = rows < 1 ? 1 : (rows > mbh ? mbh : rows);
    if (phase == 1)
        hipLaunchKernelGGL(k_dec_recon_rows, dim3(R, nframes), dim3(64), 0, s, recs, moff, fbase,
                           (const ZwDecQuant*)quant, Y, U, V, flags, mbw, mbh, ysz, csz, rowsync, borders);
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
    return off;
}

// tiles: nframes * mbw * mbh * ZW_DEC_TILE bytes (k_loopfilter's input; the planes
// are written by the filter)
extern "C" hipError_t zwk_dec_recon(hipStream_t s, const uint8_t* recs, const uint32_t* moff, const uint64_t* fbase,
                                    const void* quant, uint8_t* Y, uint8_t* U, uint8_t* V, uint8_t* flags, int mbw,
                                    int mbh, size_t ysz, size_t csz, int nframes, uint8_t* tiles)
{
    static const bool attr = []() {
        (void)hipFuncSetAttribute((const void*)k_dec_recon, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    hipLaunchKernelGGL(k_dec_recon, dim3(nframes), dim3(WGD), zw_dec_lds_bytes(mbw), s, recs, moff, fbase,
                       (const ZwDecQuant*)quant, Y, U, V, flags, mbw, mbh, ysz, csz, tiles);
    return hipGetLastError();
}

// mbw: the frames' width in MBs (every frame of a launch has the same size)
extern "C" hipError_t zwk_loopfilter(hipStream_t s, uint8_t* Y, uint8_t* U, uint8_t* V, const uint8_t* flags,
                                     const ZwFilterParams* fp, size_t ysz, size_t csz, int nframes, int mbw,
                                     const uint8_t* tiles)
{
    static const bool attr = []() {
        (void)hipFuncSetAttribute((const void*)k_loopfilter, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024 - (int)(sizeof(LfLds) * 2 * NWD + 4 * NWD + sizeof(ZwFilterParams)));
        return true;
    }();
    (void)attr;
    hipLaunchKernelGGL(k_loopfilter, dim3(nframes), dim3(WGD), (size_t)mbw * 128, s, Y, U, V, flags, fp, ysz, csz, tiles);
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

// yuv_px for a pixel pair on u16 halves (v_pk_*): mulhi(v, c) = (v * c) >> 8 is
// v * (c >> 8) + ((v * (c & 255)) >> 8), every term below 2^16; clip(t - k) for
// t = the positive part, k = 64 a + b, is min(sat(sat(t - b) >> 6 - a), 255).
// Exhaustively equal to yuv_px over all 2^24 (y, u, v).
typedef unsigned short zh2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void yuv_px2(zh2 Y, zh2 U, zh2 V, uint32_t& p0, uint32_t& p1)
{
    const zh2 yy = Y * (zh2)74 + ((Y * (zh2)133) >> (zh2)8);   // (y * 19077) >> 8
    const zh2 rv = V * (zh2)102 + ((V * (zh2)37) >> (zh2)8);   // (v * 26149) >> 8
    const zh2 gu = U * (zh2)25 + ((U * (zh2)19) >> (zh2)8);    // (u * 6419) >> 8
    const zh2 gv = V * (zh2)52 + (V >> (zh2)5);                // (v * 13320) >> 8
    const zh2 bu = U * (zh2)129 + ((U * (zh2)26) >> (zh2)8);   // (u * 33050) >> 8
    const zh2 k255 = (zh2)255;
    const zh2 r = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(yy + rv, (zh2)26) >> (zh2)6, (zh2)222), k255);
    const zh2 g = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat((zh2)(yy + (zh2)19716 - gu - gv) >> (zh2)6, (zh2)172), k255);
    const zh2 b = __builtin_elementwise_min(
        __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(yy + bu, (zh2)21) >> (zh2)6, (zh2)276), k255);
    const uint32_t rg = __builtin_bit_cast(uint32_t, r) | (__builtin_bit_cast(uint32_t, g) << 8);
    const uint32_t ba = __builtin_bit_cast(uint32_t, b) | 0xff00ff00u;
    p0 = __builtin_amdgcn_perm(ba, rg, 0x05040100u);
    p1 = __builtin_amdgcn_perm(ba, rg, 0x07060302u);
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

// One thread per 8 horizontally adjacent pixels of an output ROW PAIR: rows
// 2j-1 and 2j blend the same two chroma rows (j-1 and j, clamped), with their
// main / secondary roles swapped (fancy) or one each (simple), so the pair
// shares one set of chroma loads.  Y is one 8-byte load per row, each chroma
// row three aligned words covering columns x/2-4 .. x/2+7; the 8 pixels of a
// row leave as two 16-byte nontemporal stores (RGBA; the output is written
// once and not read back here) or six 4-byte stores (RGB); a row that does not
// start aligned in the packed output is stored bytewise.  The pixel arithmetic
// runs on u16 pairs (yuv_px2).  Threads at the image's right edge (a partial
// run) take the per-pixel form.  Measured per 256 1080p RGBA frames: 0.61 ms,
// 0.55 ms for the same loads and stores without the arithmetic (ZW_Y2R_NOCOMP);
// two row pairs per thread (ZW_Y2R_RP = 2: three chroma rows for four output
// rows) 0.635 ms, XCD-contiguous row blocks 0.66 ms, lane pairs swapping
// halves so each store instruction covers whole 64-byte granules 0.66 ms.
#ifndef ZW_Y2R_RP
#define ZW_Y2R_RP 1  // row pairs per thread (pairs j0 .. j0+RP-1 share RP+1 chroma rows)
#endif
#ifndef ZW_Y2R_PK
#define ZW_Y2R_PK 1  // the pixel arithmetic on u16 pairs (yuv_px2)
#endif
#ifndef ZW_Y2R_NOCOMP
#define ZW_Y2R_NOCOMP 0  // calibration: the same loads and stores, pixels not computed
#endif
template <int BPP, bool FANCY>
__global__ __launch_bounds__(256) void k_yuv2rgb(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U,
                                                 const uint8_t* __restrict__ V, size_t ysz, size_t csz, int w, int h,
                                                 int ys, int cs, uint8_t* __restrict__ out)
{
    const int f = blockIdx.z;
    const int j0 = (int)blockIdx.y * ZW_Y2R_RP;
    const int x = (int)(blockIdx.x * 256u + threadIdx.x) * 8;
    if (x >= w) return;
    Y += (size_t)f * ysz;
    U += (size_t)f * csz;
    V += (size_t)f * csz;
    const int cw1 = ((w + 1) >> 1) - 1, ch1 = ((h + 1) >> 1) - 1;
    const uintptr_t am = BPP == 4 ? 15 : 3;
    auto orow = [&](int r) { return out + ((size_t)f * h + (size_t)r) * (size_t)w * BPP + (size_t)x * BPP; };
    // (every full 8-pixel run takes the vector path; at the image's left / right
    // edge the fancy filter's outer chroma column is the edge column itself, so
    // the neighbour word is not loaded and the edge byte stands in for it)
    const bool fast = x + 8 <= w && (ys & 7) == 0 && (cs & 3) == 0;
    if (fast) {
        const bool lok = x > 0, rok = (x >> 1) + 4 <= cw1;
        const int c1 = x >> 1, c0 = lok ? c1 - 4 : c1, c2 = rok ? c1 + 4 : c1;
        // the six local chroma columns x/2-1 .. x/2+4 of one plane row
        auto cols = [&](const uint8_t* P, int rr, int* c6) {
            const uint8_t* q = P + (size_t)rr * cs;
            const uint32_t a = *(const uint32_t*)(q + c0), m = *(const uint32_t*)(q + c1), z = *(const uint32_t*)(q + c2);
            c6[0] = (int)(lok ? a >> 24 : m & 255u);
            c6[5] = (int)(rok ? z & 255u : m >> 24);
#pragma unroll
            for (int k = 1; k < 5; k++) c6[k] = (int)((m >> (8 * (k - 1))) & 255u);
        };
        // chroma rows j0-1 .. j0+RP-1 (clamped): pair j0+p blends rows p (main of its
        // upper row 2j-1) and p+1 (main of its lower row 2j)
        int uc[ZW_Y2R_RP + 1][6], vc[ZW_Y2R_RP + 1][6];
#pragma unroll
        for (int i = 0; i <= ZW_Y2R_RP; i++) {
            const int cr = min(max(j0 - 1 + i, 0), ch1);
            cols(U, cr, uc[i]);
            cols(V, cr, vc[i]);
        }
        auto row8 = [&](uint2 yy, const int* uM, const int* uS, const int* vM, const int* vS, uint32_t* px) {
            // fancy: 9 m + 3 s1 + 3 s2 + t = 3 (3 m + s)[mc] + (3 m + s)[sc] per column pair
            int tu[6], tv[6];
#pragma unroll
            for (int k = 0; k < 6; k++) {
                tu[k] = FANCY ? 3 * uM[k] + uS[k] : uM[k];
                tv[k] = FANCY ? 3 * vM[k] + vS[k] : vM[k];
            }
            int uu[8], vv[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int jm = 1 + (i >> 1);  // local chroma column of pixel x + i
                if (FANCY) {
                    const int js = (i & 1) ? jm + 1 : jm - 1;
                    uu[i] = (3 * tu[jm] + tu[js] + 8) >> 4;
                    vv[i] = (3 * tv[jm] + tv[js] + 8) >> 4;
                } else {
                    uu[i] = tu[jm];
                    vv[i] = tv[jm];
                }
            }
#if ZW_Y2R_PK
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const uint32_t yw = i < 4 ? yy.x : yy.y;
                const uint32_t y2 = __builtin_amdgcn_perm(0u, yw, (i & 2) ? 0x0c030c02u : 0x0c010c00u);
                yuv_px2(__builtin_bit_cast(zh2, y2), __builtin_bit_cast(zh2, pack_lo(uu[i], uu[i + 1])),
                        __builtin_bit_cast(zh2, pack_lo(vv[i], vv[i + 1])), px[i], px[i + 1]);
            }
#else
#pragma unroll
            for (int i = 0; i < 8; i++)
                px[i] = yuv_px((int)(((i < 4 ? yy.x : yy.y) >> (8 * (i & 3))) & 255u), uu[i], vv[i]);
#endif
        };
        auto store8 = [&](uint8_t* o, const uint32_t* px) {
            if (BPP == 4) {
                __builtin_nontemporal_store(zu4{px[0], px[1], px[2], px[3]}, (zu4*)o);
                __builtin_nontemporal_store(zu4{px[4], px[5], px[6], px[7]}, (zu4*)o + 1);
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
        };
        // the Y words of every row first (all loads in flight before the arithmetic)
        uint2 yw[2 * ZW_Y2R_RP];
#pragma unroll
        for (int i = 0; i < 2 * ZW_Y2R_RP; i++) {
            const int r = 2 * j0 - 1 + i;
            yw[i] = *(const uint2*)(Y + (size_t)min(max(r, 0), h - 1) * ys + x);
        }
#pragma unroll
        for (int i = 0; i < 2 * ZW_Y2R_RP; i++) {
            const int r = 2 * j0 - 1 + i, p = i >> 1;
            if (r < 0 || r >= h) continue;
            uint32_t px[8];
            if (ZW_Y2R_NOCOMP) {
#pragma unroll
                for (int k = 0; k < 8; k++)
                    px[k] = yw[i].x ^ (yw[i].y << k) ^ (uint32_t)(uc[p][k % 6] + vc[p + 1][k % 6]);
            } else if (i & 1) {
                row8(yw[i], uc[p + 1], uc[p], vc[p + 1], vc[p], px);  // row 2j: main chroma row j
            } else {
                row8(yw[i], uc[p], uc[p + 1], vc[p], vc[p + 1], px);  // row 2j-1: main chroma row j-1
            }
            uint8_t* o = orow(r);
            if (((uintptr_t)o & am) == 0) store8(o, px);
            else  // (a packed row that does not start aligned)
                for (int k = 0; k < 8 * BPP; k++) o[k] = (uint8_t)(px[k / BPP] >> (8 * (k % BPP)));
        }
    } else {
        const int n = min(8, w - x);
        for (int i = 0; i < 2 * ZW_Y2R_RP; i++) {
            const int r = 2 * j0 - 1 + i;
            if (r < 0 || r >= h) continue;
            uint8_t* o = orow(r);
            for (int k = 0; k < n; k++) {
                const uint32_t p = yuv2rgb_px<FANCY>(Y, U, V, ys, cs, cw1, ch1, r, x + k);
                for (int c = 0; c < BPP; c++) o[(size_t)k * BPP + c] = (uint8_t)(p >> (8 * c));
            }
        }
    }
}

extern "C" hipError_t zwk_yuv2rgb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, size_t ysz,
                                  size_t csz, int w, int h, int ys, int cs, int bpp, int fancy, uint8_t* out,
                                  int nframes)
{
    // row pairs (2j-1, 2j), ZW_Y2R_RP per thread
    const unsigned gy = ((unsigned)h / 2 + ZW_Y2R_RP) / ZW_Y2R_RP;
    const dim3 grid(((unsigned)w + 2047) / 2048, gy, (unsigned)nframes);
    if (bpp == 4) {
        if (fancy) hipLaunchKernelGGL((k_yuv2rgb<4, true>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
        else hipLaunchKernelGGL((k_yuv2rgb<4, false>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
    } else {
        if (fancy) hipLaunchKernelGGL((k_yuv2rgb<3, true>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
        else hipLaunchKernelGGL((k_yuv2rgb<3, false>), grid, dim3(256), 0, s, Y, U, V, ysz, csz, w, h, ys, cs, out);
    }
    return hipGetLastError();
}
