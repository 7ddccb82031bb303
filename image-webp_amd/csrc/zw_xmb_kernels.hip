// zw_xmb_kernels.hip -- the streaming DCT+quant pass over per-macroblock
// records (the HBM-roofline pass of 8(d)).
//
// Per MB, exactly the arithmetic of the encoder's final transform with the
// trellis off:
//   transform_luma_block        encoder/vp8.rs:2647-2780  (I16: prediction,
//                               fDCT x16, WHT -> Y2 quant/dequant -> iWHT,
//                               Y1 AC quant/dequant, iDCT, add_residue)
//   transform_luma_blocks_4x4   :2785-2916  (I4: the 16 sub-blocks in
//                               dependency order, each predicted from the
//                               reconstruction of its neighbours)
//   transform_chroma_blocks     :3039-3121  (+ apply_chroma_error_diffusion
//                               :572-647 on the four DCs of each plane)
// Everything the encoder takes from its running state -- the borders that
// create_border_luma / create_border_chroma build (common/prediction.rs:15-130),
// the incoming top/left error-diffusion terms -- comes from the MB's 96-byte
// record, so MBs are independent and the pass streams (layout: include/zwebp.h,
// zw_transform_quant_mbs).  The prediction is built in registers from the
// record's edge bytes, as the decoder's k_dec_recon does.
//
// Shape: one wave per 8 consecutive MBs of an MB row.  The wave stages the 8
// records, the 16x128-byte luma tile and the two 8x64-byte chroma tiles in
// LDS with 16-byte row-coalesced loads, then
//   luma, twice (MBs 0-3, 4-7): lane = 16*mb + block (the 16 blocks of an MB
//        are one DPP row, so the Y2 WHT/iWHT run as row butterflies);
//   chroma: lane = 8*mb + 4*plane + block (a quad per plane: the error
//        diffusion chain is three DPP quad broadcasts);
// and writes the levels (25 x 16 i16 per MB, zigzag, the ZwMbOut order) and
// the reconstruction tiles back with 16-byte stores.  I4 MBs run their 16
// sub-blocks along the x+2y anti-diagonals (10 steps) in an LDS work buffer
// with the reference's 32-byte stride; I16 lanes of the same wave are done
// after step 0.
// HBM per MB: 96 B record + 384 B source in, 800 B levels + 384 B recon out
// (1 568 B of it algorithmic).
#include "zw_dev.h"

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

// quantize_coeff as (c*iq + (c < 0 ? bn : bp)) >> 17, [0] DC, [1] AC (see zw_xform_kernels.hip)
struct XmbMat {
    int32_t iq[2], bp[2], bn[2], q[2];
};
struct XmbSeg {
    XmbMat y1, y2, uv;
};

#define XMB_MBS 8  // MBs per wave
#ifndef XMB_WAVES
#define XMB_WAVES 2  // waves per workgroup (LDS: 10.6 KB per wave)
#endif

#define XMB_LEVW 200  // words of levels per MB (25 x 16 i16)
#ifndef XMB_STAGE_LEV
// 1: levels staged in LDS, stored as one contiguous run; 0: stored from the lanes;
// -1 (default): staged for RGB(A) sources, from the lanes for Y/U/V planes (measured:
// staging 1.38-1.40 vs 1.43-1.44 ms per 256 RGBA frames; from the lanes 1.10 vs
// 1.15-1.16 ms from planes, whose occupancy the 6.4 KB of staging then no longer caps)
#define XMB_STAGE_LEV -1
#endif
#ifndef XMB_HALF_STAGE
// 1: the staged forms hold half the group's levels at a time (MBs 0-3, then 4-7: the
// chroma pass runs first and keeps its packed levels in registers until its half
// leaves), so the staging buffer is 3.2 instead of 6.4 KB a wave
#define XMB_HALF_STAGE 1
#endif
#ifndef XMB_PLANES_HALF
#define XMB_PLANES_HALF 0  // 1: the Y/U/V-planes form half-stages its levels too (else from the lanes)
#endif
template <int NL>
struct XmbLev {
    uint32_t lev[NL][XMB_LEVW];  // NL MBs' levels, laid out as in HBM (one contiguous store run)
};
template <>
struct XmbLev<0> {
};
template <int NL>
struct XmbLds : XmbLev<NL> {
    uint32_t rec[XMB_MBS][24];      // the 8 records
    uint32_t yt[16][36];            // luma tile: 16 rows x 8 MBs x 16 B (source, then reconstruction), rows padded
                                    // to 144 B: the lanes of a block row (4 MBs x 4 block rows x 4 columns) hit 64 banks
    uint32_t ct[2][8][20];          // U, V tiles: 8 rows x 8 MBs x 8 B, rows padded to 80 B (64 banks, as yt)
    XmbSeg seg[4];                  // the frame's four segment matrices (per-lane segment reads hit LDS, not HBM)
};

// k_xform_mb_i4: one I4 MB per lane.  Queue
// layout (u32 words): [0], [1] the counts of the queue's even / odd launches
// (k_xform_mb appends to count qp), [64..] global MB indexes.  Both counts
// are zero before a queue's first launch; each launch's drain kernel zeroes
// the other parity's count -- the previous launch's, whose drain has finished
// (stream order) and which the next launch uses -- so no kernel needs to
// know when every workgroup of the launch is done.
#define XI4_LIST 64
// The drain kernel's count read is relaxed: the queue entries come from the
// previous kernel on the stream, whose writes the launch boundary makes
// visible (an acquire at agent scope costs an L2 invalidate in every
// workgroup).
#define XI4_ACQ __ATOMIC_RELAXED
#ifndef XI4_QUAD
#define XI4_QUAD 1  // 1: k_xform_mb_i4q drains the queue; 0: k_xform_mb_i4 (one MB per lane)
#endif

DI int qz(int c, const XmbMat& m, int t) { return (__mul24(c, m.iq[t]) + (c < 0 ? m.bn[t] : m.bp[t])) >> 17; }
// A lane's quantiser matrix from LDS into registers (two 16-byte reads, pinned):
// read through the reference, each coefficient's bias became a load at a
// selected address (an LDS round trip per coefficient) instead of a select
DI XmbMat ld_mat(const XmbMat& m)
{
    v4u a = *(const v4u*)&m, b = *((const v4u*)&m + 1);
    asm volatile("" : "+v"(a), "+v"(b));
    XmbMat r;
    r.iq[0] = (int)a.x; r.iq[1] = (int)a.y; r.bp[0] = (int)a.z; r.bp[1] = (int)a.w;
    r.bn[0] = (int)b.x; r.bn[1] = (int)b.y; r.q[0] = (int)b.z; r.q[1] = (int)b.w;
    return r;
}
DI uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }

// byte pairs (b0, b1) and (b3, b2) of a row word as i16 pairs
DI uint32_t pr01(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c010c00u); }
DI uint32_t pr32(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c020c03u); }
// residual rows (src - pred, 4 bytes a row) -> dct4x4 (transform.rs:176): the
// residual pairs are formed packed (v_perm + v_pk_sub_i16) and fed straight to
// the packed-i16 row stage of fdct16_pk
DI void fdct_words(const uint32_t* sw, const uint32_t* pw, int* c)
{
    const zs2 k8p = {8, 8}, k8m = {8, -8}, k1a = {10704, 4434}, k1b = {4434, -10704};
    int o[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 R01 = as_zs2(sub_pk(pr01(sw[i]), pr01(pw[i]))), R32 = as_zs2(sub_pk(pr32(sw[i]), pr32(pw[i])));
        const zs2 A = R01 + R32, D = R01 - R32;
        o[4 * i] = dot2(A, k8p, 0);
        o[4 * i + 2] = dot2(A, k8m, 0);
        o[4 * i + 1] = dot2(D, k1a, 3625) >> 10;
        o[4 * i + 3] = dot2(D, k1b, 1875) >> 10;
    }
    const zs2 k1p = {1, 1}, k1m = {1, -1}, k2a = {5352, 2217}, k2b = {2217, -5352};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 X01 = as_zs2(pack_lo(o[i], o[4 + i])), X32 = as_zs2(pack_lo(o[12 + i], o[8 + i]));
        const zs2 A = X01 + X32, D = X01 - X32;
        c[i] = dot2(A, k1p, 7) >> 4;
        c[8 + i] = dot2(A, k1m, 7) >> 4;
        c[4 + i] = (dot2(D, k2a, 12000) >> 16) + ((as_zu(D) & 0xffffu) != 0u ? 1 : 0);
        c[12 + i] = dot2(D, k2b, 51000) >> 16;
    }
}
// iDCT (transform.rs:19) + add_residue (prediction.rs:138): reconstruction rows,
// the add and the [0, 255] clamp on i16 pairs (residuals of encoder-made levels
// stay far inside i16)
DI void recon_words(int* c, const uint32_t* pw, uint32_t* rw)
{
    idct16(c);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t r01 = clamp_pk(add_pk(pack_lo(c[4 * i], c[4 * i + 1]), pr01(pw[i])));
        const uint32_t r32 = clamp_pk(add_pk(pack_lo(c[4 * i + 3], c[4 * i + 2]), pr32(pw[i])));
        rw[i] = __builtin_amdgcn_perm(r32, r01, 0x04060200u);
    }
}
// 32 bytes into LDS as two 16-byte writes, the second half first when `swap`:
// lanes whose 32-byte slots are 256 bytes apart (the same 64 banks) then write
// different halves in each instruction (no 2-way bank conflict)
DI void lds_put32(uint32_t* o, const uint32_t* lw, bool swap)
{
    const v4u a = v4u{lw[0], lw[1], lw[2], lw[3]}, b = v4u{lw[4], lw[5], lw[6], lw[7]};
    const int h = swap ? 4 : 0;
    *(v4u*)(o + h) = swap ? b : a;
    *(v4u*)(o + 4 - h) = swap ? a : b;
}
// a block's 16 levels in zigzag order as 8 words of i16 pairs, into LDS
DI void stage_levels(uint32_t* o, const int* lv, bool swap)
{
    uint32_t lw[8];
#pragma unroll
    for (int q = 0; q < 8; q++) lw[q] = pack_lo(lv[kZZ(2 * q)], lv[kZZ(2 * q + 1)]);
    lds_put32(o, lw, swap);
}
DI void store_levels(int16_t* out, const int* lv)
{
    uint32_t lw[8];
#pragma unroll
    for (int q = 0; q < 8; q++) lw[q] = pack_lo(lv[kZZ(2 * q)], lv[kZZ(2 * q + 1)]);
    v4u* o = (v4u*)out;
    __builtin_nontemporal_store(v4u{lw[0], lw[1], lw[2], lw[3]}, o);
    __builtin_nontemporal_store(v4u{lw[4], lw[5], lw[6], lw[7]}, o + 1);
}
// predict_dcpred (prediction.rs:182-211): shift 3 (16x16) / 2 (8x8) plus one per available edge
DI uint32_t dc_word(uint32_t sum_top, uint32_t sum_left, int has_top, int has_left, int shf0)
{
    const int shf = shf0 + has_top + has_left;
    const uint32_t s = (has_top ? sum_top : 0u) + (has_left ? sum_left : 0u);
    const uint32_t dc = (!has_top && !has_left) ? 128u : ((s + (1u << (shf - 1))) >> shf);
    return dc * 0x01010101u;
}
DI uint32_t bsum(uint32_t w) { return __builtin_amdgcn_sad_u8(w, 0u, 0u); }
// V / H / TM / DC prediction rows of the 4x4 block at (bx, by) of a 16x16 or 8x8 block
// (predict_vpred / hpred / tmpred / dcpred, prediction.rs:164-324).  Branches:
// the MBs of a wave mostly share a mode (measured: a branch-free select of all
// four was 4 % slower from Y/U/V planes).  TM on i16 pairs: clamp(L + T[j] - P).
DI void pred_rows(int mode, uint32_t T, const uint8_t* left /* 4 bytes of this block's rows */, int P, uint32_t dcw,
                  uint32_t* pw)
{
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int L = left[r];
        uint32_t w;
        if (mode == 1) {
            w = T;
        } else if (mode == 2) {
            w = (uint32_t)L * 0x01010101u;
        } else if (mode == 3) {
            const uint32_t d = (uint32_t)(L - P) & 0xffffu, dd = d | (d << 16);
            const uint32_t r01 = clamp_pk(add_pk(__builtin_amdgcn_perm(0u, T, 0x0c010c00u), dd));
            const uint32_t r32 = clamp_pk(add_pk(__builtin_amdgcn_perm(0u, T, 0x0c020c03u), dd));
            w = __builtin_amdgcn_perm(r32, r01, 0x04060200u);
        } else {
            w = dcw;
        }
        pw[r] = w;
    }
}

// apply_chroma_error_diffusion's diffuse_dc (vp8.rs:589-609): adjusted DC and the error term
DI int diffuse_err(int dc, const XmbMat& m)
{
    const int level = iabs(qz(dc, m, 0));
    const int err = iabs(dc) - m24(level, m.q[0]);
    const int se = dc < 0 ? -err : err;
    const int e = se >> 1;
    return e < -127 ? -127 : (e > 127 ? 127 : e);
}
DI int adj_dc(int dc, int te, int le) { return dc + ((7 * te + 8 * le) >> 3); }

#ifndef XMB_OCC
#define XMB_OCC 0  // >0: waves per SIMD the main pass is compiled for (amdgpu_waves_per_eu)
#endif
#if XMB_OCC > 0
#define XMB_ATTR __attribute__((amdgpu_waves_per_eu(XMB_OCC)))
#else
#define XMB_ATTR
#endif

// RGB(A) source (SRC = 3 / 4): convert_image_yuv (yuv.rs:656-804) of the
// group's 16 x 128 luma pixels / 2 x 8 x 64 chroma samples straight into the
// tiles, with the MB padding of the encoder's planes (edge replication: luma
// pixel (x, y) is pixel (min(x, w-1), min(y, h-1)); chroma sample (cx, cy) is
// the 2x2 average at (min(cx, cw-1), min(cy, ch-1)), its pixel pairs clamped
// likewise).  Item = 8 pixels x 2 rows (4 chroma samples per plane).
template <int BPP>
DI uint32_t px_at(const uint8_t* img, int w, int x, int y)
{
    const uint8_t* p = img + ((size_t)y * w + x) * BPP;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
}
template <int BPP>
DI void rgb_item(const uint8_t* __restrict__ img, int w, int h, bool runs, int px0, int cy, uint32_t ya[2],
                 uint32_t yb[2], uint32_t& uw, uint32_t& vw)
{
    uint32_t a[8], b[8], ca[8], cb[8];  // luma rows 2cy, 2cy+1; chroma rows
    const int ch = (h + 1) / 2, cw = (w + 1) / 2;
    if (runs && px0 + 8 <= w && 2 * cy + 1 < h) {
        // interior: the two rows' 8-pixel runs, 16-byte (RGBA) / 8-byte (RGB) loads
        const uint8_t* ra = img + ((size_t)(2 * cy) * w + px0) * BPP;
        const uint8_t* rb = ra + (size_t)w * BPP;
        if (BPP == 4) {
            const v4u a0 = __builtin_nontemporal_load((const v4u*)ra), a1 = __builtin_nontemporal_load((const v4u*)ra + 1);
            const v4u b0 = __builtin_nontemporal_load((const v4u*)rb), b1 = __builtin_nontemporal_load((const v4u*)rb + 1);
            a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
            b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
        } else {
#pragma unroll
            for (int r = 0; r < 2; r++) {
                const uint8_t* row = r ? rb : ra;
                const v2u x0 = __builtin_nontemporal_load((const v2u*)row), x1 = __builtin_nontemporal_load((const v2u*)(row + 8));
                const v2u x2 = __builtin_nontemporal_load((const v2u*)(row + 16));
                const uint32_t wd[6] = {x0.x, x0.y, x1.x, x1.y, x2.x, x2.y};
                uint32_t* o = r ? b : a;
#pragma unroll
                for (int q = 0; q < 2; q++) {  // 4 pixels in 3 words
                    const uint32_t w0 = wd[3 * q], w1 = wd[3 * q + 1], w2 = wd[3 * q + 2];
                    o[4 * q] = w0;
                    o[4 * q + 1] = __builtin_amdgcn_alignbyte(w1, w0, 3);
                    o[4 * q + 2] = __builtin_amdgcn_alignbyte(w2, w1, 2);
                    o[4 * q + 3] = w2 >> 8;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            ca[i] = a[i];
            cb[i] = b[i];
        }
    } else {
        // edges and padding: every pixel at its clamped coordinates
        const int y0 = min(2 * cy, h - 1), y1 = min(2 * cy + 1, h - 1);
        const int ccy = min(cy, ch - 1), cy0 = 2 * ccy, cy1 = min(2 * ccy + 1, h - 1);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = min(px0 + i, w - 1);
            a[i] = px_at<BPP>(img, w, x, y0);
            b[i] = px_at<BPP>(img, w, x, y1);
            const int ccx = min((px0 >> 1) + (i >> 1), cw - 1);
            const int cxx = (i & 1) ? min(2 * ccx + 1, w - 1) : 2 * ccx;
            ca[i] = px_at<BPP>(img, w, cxx, cy0);
            cb[i] = px_at<BPP>(img, w, cxx, cy1);
        }
    }
    uw = vw = 0;
    ya[0] = pk_y4(a[0], a[1], a[2], a[3]);
    ya[1] = pk_y4(a[4], a[5], a[6], a[7]);
    yb[0] = pk_y4(b[0], b[1], b[2], b[3]);
    yb[1] = pk_y4(b[4], b[5], b[6], b[7]);
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t u, v;
        pk_uv4(ca[2 * j], ca[2 * j + 1], cb[2 * j], cb[2 * j + 1], u, v);
        uw |= u << (8 * j);
        vw |= v << (8 * j);
    }
}

// SRC: 0 = Y/U/V planes (MB-padded), 3 / 4 = RGB / RGBA pixels at Y (frame f at
// Y + f * img_stride; w, h the image size; runs: every 8-pixel run is aligned
// for its 16-byte (RGBA) / 8-byte (RGB) loads, else all pixels go the per-pixel
// way).  CV: 0 = the pass; 99 = the copy calibration (the same loads and
// stores, no arithmetic); the per-stream calibrations move one stream alone:
// 94 the records in, 92 / 97 the RGB(A) pixels in (92 raw, folded into LDS with
// no conversion; 97 converted into the tiles as the pass does), 93 the same
// pixels in with every load instruction reading 64 x 16 contiguous bytes, 96
// the levels out, 95 the reconstruction out.
template <int SRC, int CV>
__global__ __launch_bounds__(64 * XMB_WAVES) XMB_ATTR void k_xform_mb(
    const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U, const uint8_t* __restrict__ V, int w, int h,
    size_t img_stride, bool runs, const uint8_t* __restrict__ recs, const XmbSeg* __restrict__ segs, int mbw, int mbh, int nframes,
    int16_t* __restrict__ levels, uint8_t* __restrict__ RY, uint8_t* __restrict__ RU, uint8_t* __restrict__ RV,
    uint32_t* __restrict__ i4q, int qp, uint32_t* __restrict__ qerr)
{
    // (the copy calibration always stages: the same bytes in and out, levels as one
    // contiguous run -- the ceiling for moving them)
    constexpr bool COPY = CV != 0;
    constexpr bool REC_IN = CV == 0 || CV == 99 || CV == 94;
    constexpr bool PIX_IN = CV == 0 || CV == 99 || CV == 97;
    constexpr bool LEV_OUT = CV == 0 || CV == 99 || CV == 96;
    constexpr bool REC_OUT = CV == 0 || CV == 99 || CV == 95;
    constexpr bool STG = COPY || (XMB_STAGE_LEV < 0 ? (SRC != 0 || XMB_PLANES_HALF) : XMB_STAGE_LEV != 0);
    constexpr bool HALF = STG && !COPY && XMB_HALF_STAGE;
    constexpr int NL = !STG ? 0 : (HALF ? XMB_MBS / 2 : XMB_MBS);
    __shared__ XmbLds<NL> lds[XMB_WAVES];
    // (the wave's group index made wave-uniform, so its decomposition runs on the
    // scalar unit in 32 bits: as per-lane 64-bit divisions it cost ~180 VALU a wave)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    XmbLds<NL>& L = lds[wv];
    const uint32_t ngx = (uint32_t)(mbw + XMB_MBS - 1) / XMB_MBS;
    // (< 2^31: the host checks the group count)
    const uint32_t id = blockIdx.x * XMB_WAVES + (uint32_t)wv;
    if (id >= (uint32_t)nframes * (uint32_t)mbh * ngx) return;
    const int gx = (int)(id % ngx);
    const uint32_t rest = id / ngx;
    const int mby = (int)(rest % (uint32_t)mbh), f = (int)(rest / (uint32_t)mbh);
    const int x0 = gx * XMB_MBS, nact = min(XMB_MBS, mbw - x0);
    const int nmb = mbw * mbh;
    const size_t ys = (size_t)mbw * 16, cs = (size_t)mbw * 8;
    const size_t ysz = ys * mbh * 16, csz = cs * mbh * 8;
    const size_t mb0 = (size_t)f * nmb + (size_t)mby * mbw + x0;  // first MB of the group
    // chroma 16-byte pieces: plane cp, row cr, piece cq (MBs 2cq, 2cq+1)
    const int cp = lane >> 5, cr = (lane >> 2) & 7, cq = lane & 3;
    const int cn = min(max(nact - 2 * cq, 0), 2);  // MBs of the piece inside the group

    // ---- stage: records (48 lanes x 16 B), the source tiles, the segment table
    {
        const int rm = lane / 6, rq = lane % 6;
        v4u r4 = {0u, 0u, 0u, 0u};
        if (REC_IN && lane < 48 && rm < nact) r4 = __builtin_nontemporal_load((const v4u*)(recs + (mb0 + rm) * 96) + rq);
        v4u s4 = {0u, 0u, 0u, 0u};
        if (!COPY && lane >= 40) s4 = *((const v4u*)(segs + (size_t)f * 4) + (lane - 40));
        if (SRC != 0 && (CV == 92 || CV == 93)) {
            // raw pixel reads, folded into one word per lane (kept in LDS so they stay)
            const uint8_t* img = Y + (size_t)f * img_stride + ((size_t)mby * 16 * w + (size_t)x0 * 16) * SRC;
            const int rowb = nact * 16 * SRC;  // bytes of the group's row
            uint32_t acc = 0;
            if (CV == 92) {  // the pass's item pattern: lane = 8 px x 2 rows, 32 B per row
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const int g = lane >> 4, pr = (((g & 1) << 2) | ((g >> 1) << 1)) + k, xr = lane & 15;
                    if ((xr >> 1) < nact && mby * 16 + 2 * pr + 1 < h) {
                        const uint8_t* ra = img + ((size_t)(2 * pr) * w) * SRC + (size_t)xr * 32;
                        const v4u a0 = __builtin_nontemporal_load((const v4u*)ra), a1 = __builtin_nontemporal_load((const v4u*)ra + 1);
                        const v4u b0 = __builtin_nontemporal_load((const v4u*)(ra + (size_t)w * SRC));
                        const v4u b1 = __builtin_nontemporal_load((const v4u*)(ra + (size_t)w * SRC) + 1);
                        acc ^= a0.x ^ a0.y ^ a0.z ^ a0.w ^ a1.x ^ a1.y ^ a1.z ^ a1.w ^ b0.x ^ b0.y ^ b0.z ^ b0.w ^ b1.x ^ b1.y ^ b1.z ^ b1.w;
                    }
                }
            } else {  // contiguous: instruction j reads rows 2j, 2j+1, 32 lanes x 16 B each
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int r = 2 * j + (lane >> 5), c = (lane & 31) * 16;
                    if (c < rowb && mby * 16 + r < h) {
                        const v4u a = __builtin_nontemporal_load((const v4u*)(img + (size_t)r * w * SRC + c));
                        acc ^= a.x ^ a.y ^ a.z ^ a.w;
                    }
                }
            }
            (&L.yt[0][0])[lane] = acc;
        } else if (!PIX_IN) {
        } else if (SRC == 0) {
            const uint8_t* Yf = Y + f * ysz + (size_t)mby * 16 * ys + x0 * 16;
            const int yc = lane & 7, yr = lane >> 3;
            v4u y0 = {0u, 0u, 0u, 0u}, y1 = y0;
            if (yc < nact) {
                y0 = __builtin_nontemporal_load((const v4u*)(Yf + yr * ys + yc * 16));
                y1 = __builtin_nontemporal_load((const v4u*)(Yf + (yr + 8) * ys + yc * 16));
            }
            const uint8_t* Cf = (cp ? V : U) + f * csz + (size_t)(mby * 8 + cr) * cs + (x0 + 2 * cq) * 8;
            v4u c4 = {0u, 0u, 0u, 0u};
            if (cn == 2) c4 = __builtin_nontemporal_load((const v4u*)Cf);
            else if (cn == 1) {
                const v2u c2 = __builtin_nontemporal_load((const v2u*)Cf);
                c4.x = c2.x;
                c4.y = c2.y;
            }
            *(v4u*)&L.yt[yr][4 * yc] = y0;
            *(v4u*)&L.yt[yr + 8][4 * yc] = y1;
            *(v4u*)&L.ct[cp][cr][4 * cq] = c4;
        } else {
            const uint8_t* img = Y + (size_t)f * img_stride;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                // chroma row pr of the item: pass k, 16-lane group g takes rows
                // {0, 4, 2, 6} / {1, 5, 3, 7}, so the two groups of each half-wave
                // write luma rows 2 pr 288 bytes apart (disjoint banks) instead of 144
                const int g = lane >> 4, pr = (((g & 1) << 2) | ((g >> 1) << 1)) + k, xr = lane & 15;
                if ((xr >> 1) < nact) {
                    uint32_t ya[2], yb[2], uw, vw;
                    rgb_item<SRC>(img, w, h, runs, (x0 + (xr >> 1)) * 16 + 8 * (xr & 1), mby * 8 + pr, ya, yb, uw, vw);
                    *(v2u*)&L.yt[2 * pr][2 * xr] = v2u{ya[0], ya[1]};
                    *(v2u*)&L.yt[2 * pr + 1][2 * xr] = v2u{yb[0], yb[1]};
                    L.ct[0][pr][xr] = uw;
                    L.ct[1][pr][xr] = vw;
                }
            }
        }
        if (lane < 48) *(v4u*)&L.rec[rm][4 * rq] = r4;
        if (!COPY && lane >= 40) *((v4u*)L.seg + (lane - 40)) = s4;
        wsync();
    }
    const XmbSeg* S = L.seg;

    if (COPY) {
        // calibration: levels staged from the records, no arithmetic
        if constexpr (!LEV_OUT) {
        } else if constexpr (STG) {
            for (int i = lane; i < XMB_MBS * XMB_LEVW; i += 64) (&L.lev[0][0])[i] = (&L.rec[0][0])[i % (XMB_MBS * 24)];
        } else {
            for (int k = 0; k < 3; k++) {
                const int m = (lane >> 3), b = (lane & 7) + 8 * k;  // 24 blocks of every MB, 8 lanes per MB
                int lv[16];
#pragma unroll
                for (int j = 0; j < 16; j++) lv[j] = (int)L.rec[m][j] + b;
                if (m < nact) store_levels(levels + ((mb0 + m) * 25 + b + (b >= 16)) * 16, lv);
            }
        }
        wsync();
    } else {
        // the group's I4 MBs go on k_xform_mb_i4's queue (their luma is left to it)
        {
            const bool i4 = lane < nact && (L.rec[lane & 7][0] & 255u) == 4u;
            const unsigned long long b = __ballot(i4);
            if (b) {
                uint32_t base = 0;
                if (lane == 0)
                    base = __hip_atomic_fetch_add(&i4q[qp], (uint32_t)__popcll(b), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                base = (uint32_t)__shfl((int)base, 0);
                const int rank = __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u);
                // bounded: the queue holds one launch's MBs.  A count past that
                // would mean a shared or stale queue, which the host rules out;
                // should it happen, the MB's luma is not transformed and the
                // host-visible error word makes the context's calls fail
                if (i4 && base + rank < (uint32_t)nframes * (uint32_t)(mbw * mbh))
                    i4q[XI4_LIST + base + rank] = (uint32_t)(mb0 + lane);
                else if (i4)
                    __hip_atomic_store(qerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        // ---- chroma: lane = 8*mb + 4*plane + block (quad = one plane of one MB);
        // the block's 16 levels leave as 8 packed words in clw
        const int cm = lane >> 3, cplane = (lane >> 2) & 1, csub = lane & 3;
        uint32_t clw[8];
        auto chroma = [&]() {
            const int m = cm, plane = cplane, sub = csub, bx = sub & 1, by = sub >> 1;
            const uint32_t* R = L.rec[m];
            const uint8_t* Rb = (const uint8_t*)R;
            const int mode = (int)((R[0] >> 8) & 255u);
            const int seg = (int)((R[0] >> 16) & 3u);
            const int has_top = (int)((R[0] >> 24) & 1u), has_left = (int)((R[0] >> 25) & 1u);
            // (in registers for the RGB(A) forms; the planes form keeps its 5 waves a SIMD)
            XmbMat muv_r;
            if constexpr (SRC != 0) muv_r = ld_mat(S[seg].uv);
            const XmbMat& muv = SRC != 0 ? muv_r : S[seg].uv;
            const uint32_t* Tw = R + 16 + 4 * plane;  // top 8 at bytes 64 + 16*plane, left 8 right after
            const uint32_t st = bsum(Tw[0]) + bsum(Tw[1]), sl = bsum(Tw[2]) + bsum(Tw[3]);
            uint32_t pw[4], sw[4];
            pred_rows(mode, Tw[bx], Rb + 72 + 16 * plane + by * 4, Rb[21 + plane], dc_word(st, sl, has_top, has_left, 2),
                      pw);
#pragma unroll
            for (int r = 0; r < 4; r++) sw[r] = L.ct[plane][by * 4 + r][m * 2 + bx];
            int c[16];
            fdct_words(sw, pw, c);
            // error diffusion over the plane's four DCs: block 0 <- (top0, left0); 1 <- (top1, e0);
            // 2 <- (e0, left1); 3 <- (e1, e2)
            const int8_t* d = (const int8_t*)(Rb + 12 + 4 * plane);
            const int dc = c[0];
            const int dc0 = adj_dc(dc, d[0], d[2]);
            const int e0 = qb0(diffuse_err(dc0, muv));
            const int te = sub == 1 ? (int)d[1] : e0, le = sub == 1 ? e0 : (int)d[3];
            const int dc12 = adj_dc(dc, te, le);
            const int e12 = diffuse_err(dc12, muv);
            const int e1 = qb1(e12), e2 = qb2(e12);
            const int dc3 = adj_dc(dc, e1, e2);
            c[0] = sub == 0 ? dc0 : (sub == 3 ? dc3 : dc12);
            int lv[16];
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int tk = k > 0;
                lv[k] = qz(c[k], muv, tk);
                c[k] = m24(lv[k], muv.q[tk]);
            }
#pragma unroll
            for (int q = 0; q < 8; q++) clw[q] = pack_lo(lv[kZZ(2 * q)], lv[kZZ(2 * q + 1)]);
            uint32_t rw[4];
            recon_words(c, pw, rw);
#pragma unroll
            for (int r = 0; r < 4; r++) L.ct[plane][by * 4 + r][m * 2 + bx] = rw[r];
        };
        if constexpr (HALF) {
            // MBs 0-3's chroma levels join their luma in the staging buffer; MBs 4-7's
            // leave from the lanes (256 B a MB), so no level is held across the luma
            chroma();
            if (cm < XMB_MBS / 2) {
                lds_put32(&L.lev[cm][136 + 8 * (4 * cplane + csub)], clw, cm & 1);
            } else if (cm < nact) {
                v4u* o = (v4u*)(levels + ((mb0 + cm) * 25 + 17 + 4 * cplane + csub) * 16);
                __builtin_nontemporal_store(v4u{clw[0], clw[1], clw[2], clw[3]}, o);
                __builtin_nontemporal_store(v4u{clw[4], clw[5], clw[6], clw[7]}, o + 1);
            }
        }

        // ---- luma of the I16 MBs: MBs 0-3, then 4-7; lane = 16*mb + block
        const int blk = lane & 15, bx = blk & 3, by = blk >> 2;
#pragma unroll 1
        for (int hh = 0; hh < 2; hh++) {
            const int m = 4 * hh + (lane >> 4);
            const int ml = HALF ? (m & 3) : m;  // the MB's staging slot
            const uint32_t* R = L.rec[m];
            const int mode = (int)(R[0] & 255u);
            const int seg = (int)((R[0] >> 16) & 3u);
            const int has_top = (int)((R[0] >> 24) & 1u), has_left = (int)((R[0] >> 25) & 1u);
            XmbMat my1_r;
            if constexpr (SRC != 0) my1_r = ld_mat(S[seg].y1);
            const XmbMat& my1 = SRC != 0 ? my1_r : S[seg].y1;
            int y2l = 0;
            if (mode != 4) {
                uint32_t sw[4];
#pragma unroll
                for (int r = 0; r < 4; r++) sw[r] = L.yt[by * 4 + r][m * 4 + bx];
                // I16 (transform_luma_block): prediction of this lane's 4x4 from the record's edges
                const uint8_t* Rb = (const uint8_t*)R;
                const uint32_t T = R[6 + bx];
                const uint32_t st = bsum(R[6]) + bsum(R[7]) + bsum(R[8]) + bsum(R[9]);
                const uint32_t sl = bsum(R[11]) + bsum(R[12]) + bsum(R[13]) + bsum(R[14]);
                uint32_t pw[4];
                pred_rows(mode, T, Rb + 44 + by * 4, Rb[20], dc_word(st, sl, has_top, has_left, 3), pw);
                int c[16];
                fdct_words(sw, pw, c);
                // Y2: WHT of the 16 DCs (lane blk = block blk = Y2 position blk), quant, dequant, iWHT
                const XmbMat& my2 = S[seg].y2;
                const int t2 = blk > 0;
                const int y2c = wht_g(c[0], blk);
                y2l = qz(y2c, my2, t2);
                const int dcv = iwht_g(m24(y2l, my2.q[t2]), blk);
                int lv[16];
                lv[0] = 0;
#pragma unroll
                for (int k = 1; k < 16; k++) {
                    lv[k] = qz(c[k], my1, 1);
                    c[k] = m24(lv[k], my1.q[1]);
                }
                c[0] = dcv;
                if constexpr (STG) stage_levels(&L.lev[ml][8 * blk], lv, blk >= 8);
                else if (m < nact) store_levels(levels + ((mb0 + m) * 25 + blk) * 16, lv);
                uint32_t rw[4];
                recon_words(c, pw, rw);
#pragma unroll
                for (int r = 0; r < 4; r++) L.yt[by * 4 + r][m * 4 + bx] = rw[r];
            }
            // Y2 levels in zigzag order (zeros for I4 MBs)
            const int zsrc = (lane & ~15) | kZZ(blk);
            const int zv = __shfl(y2l, zsrc);
            const int zn = __shfl_down(zv, 1);
            if constexpr (STG) {
                if ((blk & 1) == 0) L.lev[ml][128 + (blk >> 1)] = pack_lo(zv, zn);
            } else {
                if ((blk & 1) == 0 && m < nact) *(uint32_t*)(levels + ((mb0 + m) * 25 + 16) * 16 + blk) = pack_lo(zv, zn);
            }
            if constexpr (HALF) {
                wsync();
                if (hh == 0) {
                    // MBs 0-3 whole (their chroma was staged first): one contiguous run of 4 x 800 B
                    const int nch = min(nact, XMB_MBS / 2) * (XMB_LEVW / 4);
                    v4u* lo = (v4u*)(levels + mb0 * 400);
#pragma unroll
                    for (int k = 0; k < (XMB_MBS / 2 * XMB_LEVW / 4 + 63) / 64; k++) {
                        const int c = 64 * k + lane;
                        if (c < nch) __builtin_nontemporal_store(*((const v4u*)&L.lev[0][0] + c), lo + c);
                    }
                } else {
                    // MBs 4-7: Y1 + Y2 (544 B a MB; their chroma left from the lanes)
                    const int nch = max(nact - XMB_MBS / 2, 0) * 34;
#pragma unroll
                    for (int k = 0; k < (XMB_MBS / 2 * 34 + 63) / 64; k++) {
                        const int c = 64 * k + lane, mm = c / 34, q = c - 34 * mm;
                        if (c < nch)
                            __builtin_nontemporal_store(*(const v4u*)&L.lev[mm][4 * q],
                                                        (v4u*)(levels + (mb0 + XMB_MBS / 2 + mm) * 400) + q);
                    }
                }
                wsync();
            }
        }

        if constexpr (!HALF) {
            chroma();
            const int m = cm;
            if constexpr (STG) {
                lds_put32(&L.lev[m][136 + 8 * (4 * cplane + csub)], clw, m & 1);
            } else if (m < nact) {
                v4u* o = (v4u*)(levels + ((mb0 + m) * 25 + 17 + 4 * cplane + csub) * 16);
                __builtin_nontemporal_store(v4u{clw[0], clw[1], clw[2], clw[3]}, o);
                __builtin_nontemporal_store(v4u{clw[4], clw[5], clw[6], clw[7]}, o + 1);
            }
        }
        wsync();
    }

    // ---- out: the group's levels as one contiguous run (nact x 800 B, 16 B a
    // lane; the half-staged form has sent them already), the reconstruction tiles
    // row-coalesced (an I4 MB's luma tile still holds its source: k_xform_mb_i4,
    // next on the stream, reads it there and overwrites it with the reconstruction)
    {
        if constexpr (STG && !HALF && LEV_OUT) {
            const int nch = nact * (XMB_LEVW / 4);
            v4u* lo = (v4u*)(levels + mb0 * 400);
#pragma unroll
            for (int k = 0; k < (XMB_MBS * XMB_LEVW / 4 + 63) / 64; k++) {
                const int c = 64 * k + lane;
                if (c < nch) __builtin_nontemporal_store(*((const v4u*)&L.lev[0][0] + c), lo + c);
            }
        }
        uint8_t* RYf = RY + f * ysz + (size_t)mby * 16 * ys + x0 * 16;
        const int yc = lane & 7, yr = lane >> 3;
        if (REC_OUT && yc < nact) {
            __builtin_nontemporal_store(*(const v4u*)&L.yt[yr][4 * yc], (v4u*)(RYf + yr * ys + yc * 16));
            __builtin_nontemporal_store(*(const v4u*)&L.yt[yr + 8][4 * yc], (v4u*)(RYf + (yr + 8) * ys + yc * 16));
        }
        uint8_t* Cf = (cp ? RV : RU) + f * csz + (size_t)(mby * 8 + cr) * cs + (x0 + 2 * cq) * 8;
        const v4u c4 = *(const v4u*)&L.ct[cp][cr][4 * cq];
#ifndef XMB_CHROMA_NT
#define XMB_CHROMA_NT (SRC == 0)  // measured: RGBA 1.300-1.303 vs 1.310-1.316 ms plain; planes 1.04 vs 1.06-1.08 NT
#endif
        if (XMB_CHROMA_NT) {
            if (REC_OUT && cn == 2) __builtin_nontemporal_store(c4, (v4u*)Cf);
            else if (REC_OUT && cn == 1) __builtin_nontemporal_store(v2u{c4.x, c4.y}, (v2u*)Cf);
        } else {
            // (64-byte row pieces: the other half of each 128-byte line is the
            // neighbouring group's, so the stores may merge in L2)
            if (REC_OUT && cn == 2) *(v4u*)Cf = c4;
            else if (REC_OUT && cn == 1) *(v2u*)Cf = v2u{c4.x, c4.y};
        }
    }
}

// The I4 MBs' luma (transform_luma_blocks_4x4, vp8.rs:2785-2916), after
// k_xform_mb: the queue it filled runs ONE MB PER LANE, 64 per wave, each lane
// walking its MB's 16 sub-blocks in raster order with the running edges in
// registers (top row of each block column, the left column, the corner):
// every wave-instruction does 64 MBs' work, where a lane-per-block layout
// would leave all but the 1-2 blocks of the current anti-diagonal idle.  I4
// MBs are rare (2-20 % at Q75 m4) and cluster in textured regions, so the
// queue balances them over the whole grid and the main pass never waits on
// their serial chains.
__global__ __launch_bounds__(64 * XMB_WAVES) void k_xform_mb_i4(const uint8_t* __restrict__ recs,
                                                              const XmbSeg* __restrict__ segs, int mbw, int mbh,
                                                              int nframes, int16_t* __restrict__ levels,
                                                              uint8_t* __restrict__ RY, uint32_t* __restrict__ i4q, int qp)
{
    __shared__ uint32_t vvs[XMB_WAVES][10][64];  // per lane: the 39-value vector (word q of lane l at [q][l])
    __shared__ uint8_t i4idx[10][16];            // d_I4_IDX
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < 40) ((uint32_t*)i4idx)[threadIdx.x] = ((const uint32_t*)d_I4_IDX)[threadIdx.x];
    __syncthreads();
    const uint8_t* vvb = (const uint8_t*)&vvs[wv][0][0];
    const int nmb = mbw * mbh;
    const uint32_t cap = (uint32_t)((long long)nframes * nmb);
    // an overflowed count (a stale or shared queue: k_xform_mb flagged it) or an
    // entry outside this launch is not trusted: nothing is read through it
    const uint32_t cnt = __hip_atomic_load(&i4q[qp], XI4_ACQ, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(&i4q[qp ^ 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t n = cnt > cap ? 0u : cnt;
    const size_t ys = (size_t)mbw * 16, ysz = ys * mbh * 16;
    const uint32_t nwaves = gridDim.x * XMB_WAVES;
#pragma unroll 1
    for (uint32_t k = 64 * (blockIdx.x * XMB_WAVES + wv); k < n; k += 64 * nwaves) {
        if (k + lane >= n) continue;  // (no cross-lane operations below)
        const size_t gm = i4q[XI4_LIST + k + lane];
        if (gm >= cap) continue;
        const int f = (int)(gm / nmb), rr = (int)(gm % nmb), mby = rr / mbw, x = rr % mbw;
        // record words 0..15: modes/segment, bpred, corner, top 16 + top-right 4, left 16
        uint32_t R[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const v4u r4 = *((const v4u*)(recs + gm * 96) + q);
            R[4 * q] = r4.x; R[4 * q + 1] = r4.y; R[4 * q + 2] = r4.z; R[4 * q + 3] = r4.w;
        }
        const int seg = (int)((R[0] >> 16) & 3u);
        XmbMat my1;
        {
            const v4u m0 = *((const v4u*)&segs[(size_t)f * 4 + seg].y1), m1 = *((const v4u*)&segs[(size_t)f * 4 + seg].y1 + 1);
            my1.iq[0] = (int)m0.x; my1.iq[1] = (int)m0.y; my1.bp[0] = (int)m0.z; my1.bp[1] = (int)m0.w;
            my1.bn[0] = (int)m1.x; my1.bn[1] = (int)m1.y; my1.q[0] = (int)m1.z; my1.q[1] = (int)m1.w;
        }
        // k_xform_mb left the MB's source luma in its reconstruction tile
        uint8_t* ymb = RY + f * ysz + (size_t)mby * 16 * ys + (size_t)x * 16;
        uint32_t top[4] = {R[6], R[7], R[8], R[9]};  // bottom row above each block column
        uint32_t lc[4] = {R[11], R[12], R[13], R[14]};  // the MB's left column, 4 rows a word
        uint32_t pc0 = R[5] & 255u;                      // corner of block (0, by)
#pragma unroll 1
        for (int by = 0; by < 4; by++) {
            uint32_t src[4][4], rec[4][4];  // [row][block column]
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const v4u v = *(const v4u*)(ymb + (size_t)(4 * by + r) * ys);
                src[r][0] = v.x; src[r][1] = v.y; src[r][2] = v.z; src[r][3] = v.w;
            }
            const uint32_t bpw = (by < 2 ? R[1] : R[2]) >> (16 * (by & 1));
            uint32_t L = lc[0], P = pc0;
#pragma unroll
            for (int bx = 0; bx < 4; bx++) {
                const uint32_t T = top[bx], TR = bx < 3 ? top[bx + 1] : R[10];
                const int sm = (int)((bpw >> (4 * bx)) & 15u);
                // the 13 edges: left column bottom-up, corner, top 4 + top-right 4
                int E[13];
#pragma unroll
                for (int j = 0; j < 4; j++) E[j] = (int)byte_of(L, 3 - j);
                E[4] = (int)P;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    E[5 + j] = (int)byte_of(T, j);
                    E[9 + j] = (int)byte_of(TR, j);
                }
                // the 39-value vector (k_dec_recon's dec_i4_values), then this mode's pixels
#pragma unroll
                for (int q = 0; q < 10; q++) {
                    uint32_t wd = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int i = 4 * q + j;
                        int v;
                        if (i < 13) v = E[i];
                        else if (i < 24) v = (E[i - 13] + 2 * E[i - 12] + E[i - 11] + 2) >> 2;
                        else if (i < 36) v = (E[i - 24] + E[i - 23] + 1) >> 1;
                        else if (i == 36) v = (E[11] + 3 * E[12] + 2) >> 2;
                        else if (i == 37) v = (E[1] + 3 * E[0] + 2) >> 2;
                        else if (i == 38) v = (4 + E[0] + E[1] + E[2] + E[3] + E[5] + E[6] + E[7] + E[8]) >> 3;
                        else v = 0;
                        wd |= (uint32_t)v << (8 * j);
                    }
                    vvs[wv][q][lane] = wd;
                }
                uint32_t pw[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    uint32_t wd = 0;
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int idx = i4idx[sm][4 * r + j];
                        int v;
                        if (idx == 254) v = clamp255(E[3 - r] + E[5 + j] - E[4]);
                        else {
                            const int ii = idx == 255 ? 38 : idx;
                            v = vvb[((ii >> 2) * 64 + lane) * 4 + (ii & 3)];
                        }
                        wd |= (uint32_t)v << (8 * j);
                    }
                    pw[r] = wd;
                }
                uint32_t s4[4];
#pragma unroll
                for (int r = 0; r < 4; r++) s4[r] = src[r][bx];
                int cf[16], lv[16];
                fdct_words(s4, pw, cf);
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    const int tk = j > 0;
                    lv[j] = qz(cf[j], my1, tk);
                    cf[j] = m24(lv[j], my1.q[tk]);
                }
                store_levels(levels + (gm * 25 + 4 * by + bx) * 16, lv);
                uint32_t rw[4];
                recon_words(cf, pw, rw);
#pragma unroll
                for (int r = 0; r < 4; r++) rec[r][bx] = rw[r];
                // the next block's edges: this block's right column, the corner above it
                P = T >> 24;
                L = (rw[0] >> 24) | ((rw[1] >> 24) << 8) | ((rw[2] >> 24) << 16) | (rw[3] & 0xff000000u);
                top[bx] = rw[3];
            }
#pragma unroll
            for (int r = 0; r < 4; r++)
                __builtin_nontemporal_store(v4u{rec[r][0], rec[r][1], rec[r][2], rec[r][3]},
                                            (v4u*)(ymb + (size_t)(4 * by + r) * ys));
            pc0 = lc[0] >> 24;
            lc[0] = lc[1];
            lc[1] = lc[2];
            lc[2] = lc[3];
        }
    }
}

// The same I4 MBs in quad form (the default, XI4_QUAD): 8 MBs a wave, 8 lanes
// an MB -- two quads, one per block of the current x+2y anti-diagonal, lane q
// of a quad holding row q of the block's pixels and column q of its
// coefficients (uvq_fdct / uvq_idct_recon, the encoder's I4 candidate form).
// An MB's chain is 10 steps of a quarter block each instead of 16 whole
// blocks, and the queue's MBs spread over 8x the waves: the one-MB-per-lane
// form above is bound by that chain (one wave a SIMD issuing a serial
// 16-block walk), this one by issue.  Per MB in LDS: the reconstruction with
// its borders (row 0 the pixels above, byte column 8 + x for pixel x, so a
// block's row is one aligned word and its left neighbour byte 3 of the word
// before), the source luma, the 16 blocks' levels as they leave, the record.
#define XQ_MBS 8
struct XqMb {
    uint32_t buf[17][8];  // cols 7 (left / corner), 8..23 (the MB), 24..27 (above-right)
    uint32_t src[16][4];
    uint32_t lev[16][8];  // blocks 0..15, zigzag i16 pairs (the first 512 B of the MB's levels)
    uint32_t rec[16];     // record words 0..15
};
__global__ __launch_bounds__(64 * XMB_WAVES) void k_xform_mb_i4q(const uint8_t* __restrict__ recs,
                                                               const XmbSeg* __restrict__ segs, int mbw, int mbh,
                                                               int nframes, int16_t* __restrict__ levels,
                                                               uint8_t* __restrict__ RY, uint32_t* __restrict__ i4q, int qp)
{
    __shared__ XqMb qm[XMB_WAVES][XQ_MBS];
    __shared__ uint32_t vvs[XMB_WAVES][10][64];  // per lane: the 39-value vector (word w of lane l at [w][l])
    __shared__ uint8_t i4idx[10][16];            // d_I4_IDX
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x < 40) ((uint32_t*)i4idx)[threadIdx.x] = ((const uint32_t*)d_I4_IDX)[threadIdx.x];
    __syncthreads();
    const uint8_t* vvb = (const uint8_t*)&vvs[wv][0][0];
    const int mi = lane >> 3, j8 = lane & 7, slot = (lane >> 2) & 1, q = lane & 3;
    XqMb& M = qm[wv][mi];
    const int nmb = mbw * mbh;
    const uint32_t cap = (uint32_t)((long long)nframes * nmb);
    const uint32_t cnt = __hip_atomic_load(&i4q[qp], XI4_ACQ, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(&i4q[qp ^ 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t n = cnt > cap ? 0u : cnt;
    const size_t ys = (size_t)mbw * 16, ysz = ys * mbh * 16;
    const uint32_t nwaves = gridDim.x * XMB_WAVES;
#pragma unroll 1
    for (uint32_t k = XQ_MBS * (blockIdx.x * XMB_WAVES + wv); k < n; k += XQ_MBS * nwaves) {
        // every lane runs every step (the quads' DPP reads need their whole quad);
        // an MB slot past the queue's end or with an entry outside the launch
        // computes on zeros and stores nothing
        const bool have = k + mi < n;
        uint32_t gm = have ? i4q[XI4_LIST + k + mi] : 0u;
        const bool valid = have && gm < cap;
        gm = valid ? gm : 0u;
        const int f = (int)(gm / nmb), rr = (int)(gm % nmb), mby = rr / mbw, x = rr % mbw;
        uint8_t* ymb = RY + f * ysz + (size_t)mby * 16 * ys + (size_t)x * 16;
        {
            v4u r4 = {0u, 0u, 0u, 0u}, s0 = r4, s1 = r4;
            if (valid) {
                if (j8 < 4) r4 = *((const v4u*)(recs + (size_t)gm * 96) + j8);
                s0 = *(const v4u*)(ymb + (size_t)(2 * j8) * ys);  // (k_xform_mb left the source luma here)
                s1 = *(const v4u*)(ymb + (size_t)(2 * j8 + 1) * ys);
            }
            if (j8 < 4) *(v4u*)&M.rec[4 * j8] = r4;
            *(v4u*)M.src[2 * j8] = s0;
            *(v4u*)M.src[2 * j8 + 1] = s1;
        }
        wsync();
        // borders: row 0 = corner, the 16 pixels above, the 4 above-right; the
        // left column down col 7; blocks (3, by > 0) read the above-right 4 too
        // (rows 4, 8, 12), as the reference's top-right of the right column
        if (j8 == 0) M.buf[0][1] = (M.rec[5] & 255u) << 24;
        if (j8 < 4) M.buf[0][2 + j8] = M.rec[6 + j8];
        if (j8 == 4) M.buf[0][6] = M.rec[10];
        if (j8 > 4) M.buf[4 * (j8 - 4)][6] = M.rec[10];
#pragma unroll
        for (int t = 0; t < 2; t++) {
            const int r = 2 * j8 + t;
            M.buf[1 + r][1] = ((M.rec[11 + (r >> 2)] >> (8 * (r & 3))) & 255u) << 24;
        }
        const int seg = (int)((M.rec[0] >> 16) & 3u);
        XmbMat my1;
        {
            const v4u m0 = *((const v4u*)&segs[(size_t)f * 4 + seg].y1), m1 = *((const v4u*)&segs[(size_t)f * 4 + seg].y1 + 1);
            my1.iq[0] = (int)m0.x; my1.iq[1] = (int)m0.y; my1.bp[0] = (int)m0.z; my1.bp[1] = (int)m0.w;
            my1.bn[0] = (int)m1.x; my1.bn[1] = (int)m1.y; my1.q[0] = (int)m1.z; my1.q[1] = (int)m1.w;
        }
        const uint32_t bp01 = M.rec[1], bp23 = M.rec[2];
        wsync();
#pragma unroll 1
        for (int s = 0; s < 10; s++) {
            const int sbyA = s < 4 ? 0 : (s - 2) >> 1, sbxA = s - 2 * sbyA;
            const bool act = slot == 0 || (s >= 2 && s <= 7);
            const int bx = act ? (slot ? sbxA - 2 : sbxA) : 0, by = act ? (slot ? sbyA + 1 : sbyA) : 0;
            const int sm = (int)((((by < 2 ? bp01 : bp23) >> (16 * (by & 1))) >> (4 * bx)) & 15u);
            // the 13 edges: left column bottom-up, corner, top 4 + top-right 4
            const uint32_t* ra = M.buf[4 * by];
            const uint32_t wc = ra[1 + bx], T = ra[2 + bx], TR = ra[3 + bx];
            uint32_t Lr[4];
#pragma unroll
            for (int r = 0; r < 4; r++) Lr[r] = M.buf[1 + 4 * by + r][1 + bx] >> 24;
            const uint32_t sw = M.src[4 * by + q][bx];
            int E[13];
#pragma unroll
            for (int t = 0; t < 4; t++) E[t] = (int)Lr[3 - t];
            E[4] = (int)(wc >> 24);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                E[5 + t] = (int)byte_of(T, t);
                E[9 + t] = (int)byte_of(TR, t);
            }
#pragma unroll
            for (int w = 0; w < 10; w++) {
                uint32_t wd = 0;
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const int i = 4 * w + t;
                    int v;
                    if (i < 13) v = E[i];
                    else if (i < 24) v = (E[i - 13] + 2 * E[i - 12] + E[i - 11] + 2) >> 2;
                    else if (i < 36) v = (E[i - 24] + E[i - 23] + 1) >> 1;
                    else if (i == 36) v = (E[11] + 3 * E[12] + 2) >> 2;
                    else if (i == 37) v = (E[1] + 3 * E[0] + 2) >> 2;
                    else if (i == 38) v = (4 + E[0] + E[1] + E[2] + E[3] + E[5] + E[6] + E[7] + E[8]) >> 3;
                    else v = 0;
                    wd |= (uint32_t)v << (8 * t);
                }
                vvs[wv][w][lane] = wd;
            }
            // row q of the prediction (TrueMotion: clamp(L[q] + T[t] - corner))
            const int Lq = sel4(q, (int)Lr[0], (int)Lr[1], (int)Lr[2], (int)Lr[3]);
            uint32_t pw = 0;
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int idx = i4idx[sm][4 * q + t];
                int v;
                if (idx == 254) v = clamp255(Lq + E[5 + t] - E[4]);
                else {
                    const int ii = idx == 255 ? 38 : idx;
                    v = vvb[((ii >> 2) * 64 + lane) * 4 + (ii & 3)];
                }
                pw |= (uint32_t)v << (8 * t);
            }
            const uint32_t p01 = __builtin_amdgcn_perm(0u, pw, 0x0c010c00u), p32 = __builtin_amdgcn_perm(0u, pw, 0x0c020c03u);
            const uint32_t R01 = sub_pk(pr01(sw), p01), R32 = sub_pk(pr32(sw), p32);
            int cf[4];
            uvq_fdct(add_pk(R01, R32), sub_pk(R01, R32), q, cf);  // cf[r]: coefficient (r, q), natural index 4 r + q
            int lv[4], dq[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                // (selects, not my1.x[tk]: a lane-varying index would put my1 in scratch)
                const bool dc = r == 0 && q == 0;
                const int c = cf[r];
                const int iq = dc ? my1.iq[0] : my1.iq[1], bp = dc ? my1.bp[0] : my1.bp[1];
                const int bn = dc ? my1.bn[0] : my1.bn[1], qq = dc ? my1.q[0] : my1.q[1];
                lv[r] = (__mul24(c, iq) + (c < 0 ? bn : bp)) >> 17;
                dq[r] = m24(lv[r], qq);
            }
            uint32_t r01, r32;
            uvq_idct_recon(dq, p01, p32, q, r01, r32);
            if (act) {
                M.buf[1 + 4 * by + q][2 + bx] = __builtin_amdgcn_perm(r32, r01, 0x04060200u);
                int16_t* lp = (int16_t*)M.lev[4 * by + bx];
#pragma unroll
                for (int r = 0; r < 4; r++) lp[izz_of(4 * r + q)] = (int16_t)lv[r];
            }
            wsync();
        }
        if (valid) {
            v4u* lo = (v4u*)(levels + (size_t)gm * 400);
#pragma unroll
            for (int t = 0; t < 4; t++) __builtin_nontemporal_store(*((const v4u*)&M.lev[0][0] + 4 * j8 + t), lo + 4 * j8 + t);
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const int r = 2 * j8 + t;
                const v2u a = *(const v2u*)&M.buf[1 + r][2], b = *(const v2u*)&M.buf[1 + r][4];
                __builtin_nontemporal_store(v4u{a.x, a.y, b.x, b.y}, (v4u*)(ymb + (size_t)r * ys));
            }
        }
        wsync();
    }
}

extern "C" size_t zwk_xform_mb_seg_bytes(void) { return sizeof(XmbSeg) * 4; }
// Bytes of the I4 queue (k_xform_mb appends, k_xform_mb_i4 drains); its
// first 8 bytes must be zero before the first launch.
extern "C" size_t zwk_xform_mb_queue_bytes(int mbw, int mbh, int nframes)
{
    return 4 * (XI4_LIST + (size_t)nframes * mbw * mbh);
}

// segs: per frame 4 x (y1, y2, uv) as {q_dc, q_ac, iq_dc, iq_ac, bias_dc, bias_ac} host-built ZwMatrix
// triples, converted here into the branch-free quantiser form.  variant 99: copy calibration.
extern "C" void zwk_xform_mb_pack_segs(const ZwMatrix* m /* [n][4][3] */, int n, void* out)
{
    XmbSeg* o = (XmbSeg*)out;
    for (int i = 0; i < n * 4; i++) {
        XmbMat* dst[3] = {&o[i].y1, &o[i].y2, &o[i].uv};
        for (int k = 0; k < 3; k++) {
            const ZwMatrix& s = m[i * 3 + k];
            for (int t = 0; t < 2; t++) {
                dst[k]->iq[t] = (int32_t)s.iq[t];
                dst[k]->bp[t] = (int32_t)s.bias[t];
                dst[k]->bn[t] = (int32_t)((1u << 17) - 1 - s.bias[t]);
                dst[k]->q[t] = (int32_t)s.q[t];
            }
        }
    }
}

// queue: zwk_xform_mb_queue_bytes of device memory whose two counters are zero
// (as every launch leaves them); qerr: a host-visible word the kernel sets to 1
// if the queue overflowed (never cleared here).  src_bpp: 0 = Y/U/V planes; 3 / 4 = RGB / RGBA
// pixels at Y (frame stride img_stride, image w x h).
extern "C" hipError_t zwk_xform_mb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, int src_bpp,
                                   int w, int h, size_t img_stride, const uint8_t* recs, const void* segs, int mbw,
                                   int mbh, int nframes, int16_t* levels, uint8_t* RY, uint8_t* RU, uint8_t* RV,
                                   uint32_t* queue, int qp, uint32_t* qerr, int variant)
{
    const long long waves = (long long)nframes * mbh * ((mbw + XMB_MBS - 1) / XMB_MBS);
    const unsigned grid = (unsigned)((waves + XMB_WAVES - 1) / XMB_WAVES);
    if (grid == 0) return hipSuccess;
    if (waves >= (1LL << 31)) return hipErrorInvalidValue;  // (k_xform_mb indexes its groups in 32 bits)
    if (src_bpp != 0 && src_bpp != 3 && src_bpp != 4) return hipErrorInvalidValue;
    const XmbSeg* sg = (const XmbSeg*)segs;
    const bool copy = variant != 0;
    if (copy && variant != 99 && (src_bpp == 0 || (variant != 92 && variant != 93 && (variant < 94 || variant > 97))))
        return hipErrorInvalidValue;
    const int ra = src_bpp == 4 ? 16 : 8;
    const bool runs = src_bpp != 0 && (uintptr_t)Y % ra == 0 && img_stride % ra == 0 && ((size_t)w * src_bpp) % ra == 0;
#define XMB_LAUNCH(SRC, CP)                                                                                         \
    hipLaunchKernelGGL((k_xform_mb<SRC, CP>), dim3(grid), dim3(64 * XMB_WAVES), 0, s, Y, U, V, w, h, img_stride, runs,  \
                       recs, sg, mbw, mbh, nframes, levels, RY, RU, RV, queue, qp, qerr)
    if (src_bpp == 0) {
        if (copy) XMB_LAUNCH(0, 99);
        else XMB_LAUNCH(0, 0);
    } else if (src_bpp == 3) {
        if (copy) XMB_LAUNCH(3, 99);
        else XMB_LAUNCH(3, 0);
    } else {
        switch (variant) {
        case 0: XMB_LAUNCH(4, 0); break;
        case 92: XMB_LAUNCH(4, 92); break;
        case 93: XMB_LAUNCH(4, 93); break;
        case 94: XMB_LAUNCH(4, 94); break;
        case 95: XMB_LAUNCH(4, 95); break;
        case 96: XMB_LAUNCH(4, 96); break;
        case 97: XMB_LAUNCH(4, 97); break;
        default: XMB_LAUNCH(4, 99); break;
        }
    }
#undef XMB_LAUNCH
    if (copy) return hipGetLastError();
    // the I4 queue: waves of XQ_MBS (quad form) / 64 MBs; grid for an I4 share up
    // to 1/16 in one pass over it, at most 4096 / 1024 workgroups
    const long long nmbs = (long long)nframes * mbw * mbh;
    if (XI4_QUAD) {
        const unsigned g4 = (unsigned)min((nmbs + XQ_MBS * 16 * XMB_WAVES - 1) / (XQ_MBS * 16 * XMB_WAVES), 4096LL);
        hipLaunchKernelGGL(k_xform_mb_i4q, dim3(g4), dim3(64 * XMB_WAVES), 0, s, recs, sg, mbw, mbh, nframes, levels,
                           RY, queue, qp);
    } else {
        const unsigned g4 = (unsigned)min((nmbs + 64 * 16 * XMB_WAVES - 1) / (64 * 16 * XMB_WAVES), 1024LL);
        hipLaunchKernelGGL(k_xform_mb_i4, dim3(g4), dim3(64 * XMB_WAVES), 0, s, recs, sg, mbw, mbh, nframes, levels,
                           RY, queue, qp);
    }
    return hipGetLastError();
}
