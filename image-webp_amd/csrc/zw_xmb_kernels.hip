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
#define XMB_WAVES 4

struct XmbLds {
    uint32_t rec[XMB_MBS][24];   // the 8 records
    uint32_t yt[16][32];         // luma tile: 16 rows x 8 MBs x 16 B (source, then reconstruction)
    uint32_t ct[2][8][16];       // U, V tiles: 8 rows x 8 MBs x 8 B
    uint8_t ws[4][17 * ZW_BPS + 4];  // I4 work buffers (origin at byte 3: row pixels dword aligned)
    uint8_t vv[64][40];          // per-lane I4 value vectors (dec_i4_values layout)
    XmbSeg seg[4];               // the frame's four segment matrices (per-lane segment reads hit LDS, not HBM)
};

DI int qz(int c, const XmbMat& m, int t) { return (__mul24(c, m.iq[t]) + (c < 0 ? m.bn[t] : m.bp[t])) >> 17; }
DI uint32_t byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255u; }

// residual rows (src - pred, 4 bytes a row) -> dct4x4 (transform.rs:176), packed-i16 form
DI void fdct_words(const uint32_t* sw, const uint32_t* pw, int* c)
{
    int r[16];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) r[4 * i + j] = (int)byte_of(sw[i], j) - (int)byte_of(pw[i], j);
    fdct16_pk(r, c);
}
// iDCT (transform.rs:19) + add_residue (prediction.rs:138): reconstruction rows
DI void recon_words(int* c, const uint32_t* pw, uint32_t* rw)
{
    idct16(c);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) w |= (uint32_t)clamp255(c[4 * i + j] + (int)byte_of(pw[i], j)) << (8 * j);
        rw[i] = w;
    }
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
            w = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) w |= (uint32_t)clamp255(L + (int)byte_of(T, j) - P) << (8 * j);
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
    const int err = iabs(dc) - level * m.q[0];
    const int se = dc < 0 ? -err : err;
    const int e = se >> 1;
    return e < -127 ? -127 : (e > 127 ? 127 : e);
}
DI int adj_dc(int dc, int te, int le) { return dc + ((7 * te + 8 * le) >> 3); }

template <bool COPY>
__global__ __launch_bounds__(64 * XMB_WAVES) void k_xform_mb(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U,
                                                           const uint8_t* __restrict__ V, const uint8_t* __restrict__ recs,
                                                           const XmbSeg* __restrict__ segs, int mbw, int mbh, int nframes,
                                                           int16_t* __restrict__ levels, uint8_t* __restrict__ RY,
                                                           uint8_t* __restrict__ RU, uint8_t* __restrict__ RV)
{
    __shared__ XmbLds lds[XMB_WAVES];
    __shared__ uint8_t i4idx[10][16];  // d_I4_IDX
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (!COPY && threadIdx.x < 40) ((uint32_t*)i4idx)[threadIdx.x] = ((const uint32_t*)d_I4_IDX)[threadIdx.x];
    __syncthreads();
    XmbLds& L = lds[wv];
    const int ngx = (mbw + XMB_MBS - 1) / XMB_MBS;
    const long long id = (long long)blockIdx.x * XMB_WAVES + wv;
    if (id >= (long long)nframes * mbh * ngx) return;
    const int gx = (int)(id % ngx);
    const long long rest = id / ngx;
    const int mby = (int)(rest % mbh), f = (int)(rest / mbh);
    const int x0 = gx * XMB_MBS, nact = min(XMB_MBS, mbw - x0);
    const int nmb = mbw * mbh;
    const size_t ys = (size_t)mbw * 16, cs = (size_t)mbw * 8;
    const size_t ysz = ys * mbh * 16, csz = cs * mbh * 8;
    const size_t mb0 = (size_t)f * nmb + (size_t)mby * mbw + x0;  // first MB of the group
    const uint8_t* Yf = Y + f * ysz + (size_t)mby * 16 * ys + x0 * 16;
    const uint8_t* Uf = U + f * csz + (size_t)mby * 8 * cs + x0 * 8;
    const uint8_t* Vf = V + f * csz + (size_t)mby * 8 * cs + x0 * 8;

    // ---- stage: records (48 lanes x 16 B), luma rows (2 x 16 B), chroma rows (2 x 8 B)
    {
        const int rm = lane / 6, rq = lane % 6;
        v4u r4 = {0u, 0u, 0u, 0u};
        if (lane < 48 && rm < nact) r4 = __builtin_nontemporal_load((const v4u*)(recs + (mb0 + rm) * 96) + rq);
        const int yc = lane & 7, yr = lane >> 3;
        v4u y0 = {0u, 0u, 0u, 0u}, y1 = y0;
        if (yc < nact) {
            y0 = __builtin_nontemporal_load((const v4u*)(Yf + yr * ys + yc * 16));
            y1 = __builtin_nontemporal_load((const v4u*)(Yf + (yr + 8) * ys + yc * 16));
        }
        // chroma: 128 8-byte pieces (plane, row, MB), two per lane
        v2u c0 = {0u, 0u}, c1 = c0;
        const int cm = lane & 7, cr = (lane >> 3) & 7;
        if (cm < nact) {
            c0 = __builtin_nontemporal_load((const v2u*)(Uf + cr * cs + cm * 8));
            c1 = __builtin_nontemporal_load((const v2u*)(Vf + cr * cs + cm * 8));
        }
        // the frame's segment table: 4 x 96 B = 24 lines of 16 B
        v4u s4 = {0u, 0u, 0u, 0u};
        if (!COPY && lane >= 40) s4 = *((const v4u*)(segs + (size_t)f * 4) + (lane - 40));
        if (lane < 48) *(v4u*)&L.rec[rm][4 * rq] = r4;
        if (!COPY && lane >= 40) *((v4u*)L.seg + (lane - 40)) = s4;
        *(v4u*)&L.yt[yr][4 * yc] = y0;
        *(v4u*)&L.yt[yr + 8][4 * yc] = y1;
        *(v2u*)&L.ct[0][cr][2 * cm] = c0;
        *(v2u*)&L.ct[1][cr][2 * cm] = c1;
        wsync();
    }
    const XmbSeg* S = L.seg;

    if (COPY) {
        // calibration: the same loads and stores, no arithmetic
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int m = 4 * h + (lane >> 4), blk = lane & 15;
            if (m < nact) {
                int lv[16];
#pragma unroll
                for (int k = 0; k < 16; k++) lv[k] = (int)L.rec[m][k] + blk;
                store_levels(levels + ((mb0 + m) * 25 + blk) * 16, lv);
                if (blk < 8) *(uint32_t*)(levels + ((mb0 + m) * 25 + 16) * 16 + 2 * blk) = L.rec[m][blk];
            }
        }
        {
            const int m = lane >> 3, b = lane & 7;
            if (m < nact) {
                int lv[16];
#pragma unroll
                for (int k = 0; k < 16; k++) lv[k] = (int)L.rec[m][k + 8] + b;
                store_levels(levels + ((mb0 + m) * 25 + 17 + b) * 16, lv);
            }
        }
    } else {
        // ---- luma: MBs 0-3, then 4-7; lane = 16*mb + block
        const int blk = lane & 15, bx = blk & 3, by = blk >> 2;
#pragma unroll 1
        for (int h = 0; h < 2; h++) {
            const int m = 4 * h + (lane >> 4);
            const uint32_t* R = L.rec[m];
            const int mode = (int)(R[0] & 255u);
            const int seg = (int)((R[0] >> 16) & 3u);
            const int has_top = (int)((R[0] >> 24) & 1u), has_left = (int)((R[0] >> 25) & 1u);
            const XmbMat& my1 = S[seg].y1;
            uint32_t sw[4];
#pragma unroll
            for (int r = 0; r < 4; r++) sw[r] = L.yt[by * 4 + r][m * 4 + bx];
            int y2l = 0;
            if (mode != 4) {
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
                const int dcv = iwht_g(y2l * my2.q[t2], blk);
                int lv[16];
                lv[0] = 0;
#pragma unroll
                for (int k = 1; k < 16; k++) {
                    lv[k] = qz(c[k], my1, 1);
                    c[k] = lv[k] * my1.q[1];
                }
                c[0] = dcv;
                if (m < nact) store_levels(levels + ((mb0 + m) * 25 + blk) * 16, lv);
                uint32_t rw[4];
                recon_words(c, pw, rw);
#pragma unroll
                for (int r = 0; r < 4; r++) L.yt[by * 4 + r][m * 4 + bx] = rw[r];
            }
            // I4 MBs of this half (transform_luma_blocks_4x4): x+2y anti-diagonals
            const bool any_i4 = __builtin_amdgcn_ballot_w64(mode == 4) != 0;
            if (any_i4) {
                uint8_t* ws = L.ws[m & 3] + 3;
                if (mode == 4) {
                    // create_border_luma from the record: corner, top 16 + top-right 4, left 16,
                    // the top-right 4 copied to rows 4, 8, 12
                    if (blk < 5) *(uint32_t*)(ws + 1 + 4 * blk) = R[6 + blk];
                    if (blk == 5) ws[0] = (uint8_t)(R[5] & 255u);
                    if (blk >= 6 && blk < 9) *(uint32_t*)(ws + 4 * (blk - 5) * ZW_BPS + 17) = R[10];
                    ws[(blk + 1) * ZW_BPS] = ((const uint8_t*)R)[44 + blk];
                }
                wsync();
                const int sm = (int)((R[1 + (blk >> 3)] >> (4 * (blk & 7))) & 15u);  // bpred[blk]
                const int xo = bx * 4 + 1, yo = by * 4 + 1;
                uint8_t* vv = L.vv[lane];
#pragma unroll 1
                for (int t = 0; t < 10; t++) {
                    if (mode == 4 && bx + 2 * by == t) {
                        // the 39-value vector of this sub-block's edges (k_dec_recon's dec_i4_values)
                        int E[13];
#pragma unroll
                        for (int k = 0; k < 4; k++) E[k] = ws[(yo + 3 - k) * ZW_BPS + xo - 1];
                        E[4] = ws[(yo - 1) * ZW_BPS + xo - 1];
#pragma unroll
                        for (int k = 5; k < 13; k++) E[k] = ws[(yo - 1) * ZW_BPS + xo + (k - 5)];
                        uint32_t vw[10];
#pragma unroll
                        for (int q = 0; q < 10; q++) {
                            uint32_t w = 0;
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
                                w |= (uint32_t)v << (8 * j);
                            }
                            vw[q] = w;
                        }
#pragma unroll
                        for (int q = 0; q < 10; q++) *(uint32_t*)(vv + 4 * q) = vw[q];
                        uint32_t pw[4];
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            uint32_t w = 0;
#pragma unroll
                            for (int j = 0; j < 4; j++) {
                                const int idx = i4idx[sm][4 * r + j];
                                int v;
                                if (idx == 254) v = clamp255(E[3 - r] + E[5 + j] - E[4]);
                                else v = vv[idx == 255 ? 38 : idx];
                                w |= (uint32_t)v << (8 * j);
                            }
                            pw[r] = w;
                        }
                        uint32_t s4[4];
#pragma unroll
                        for (int r = 0; r < 4; r++) s4[r] = sw[r];
                        int c[16], lv[16];
                        fdct_words(s4, pw, c);
#pragma unroll
                        for (int k = 0; k < 16; k++) {
                            const int tk = k > 0;
                            lv[k] = qz(c[k], my1, tk);
                            c[k] = lv[k] * my1.q[tk];
                        }
                        if (m < nact) store_levels(levels + ((mb0 + m) * 25 + blk) * 16, lv);
                        uint32_t rw[4];
                        recon_words(c, pw, rw);
#pragma unroll
                        for (int r = 0; r < 4; r++) {
                            *(uint32_t*)(ws + (yo + r) * ZW_BPS + xo) = rw[r];
                            L.yt[by * 4 + r][m * 4 + bx] = rw[r];
                        }
                    }
                    wsync();
                }
            }
            // Y2 levels in zigzag order (zeros for I4 MBs): eight 4-byte stores per MB
            const int zsrc = (lane & ~15) | kZZ(blk);
            const int zv = __shfl(y2l, zsrc);
            const int zn = __shfl_down(zv, 1);
            if ((blk & 1) == 0 && m < nact)
                *(uint32_t*)(levels + ((mb0 + m) * 25 + 16) * 16 + blk) = pack_lo(zv, zn);
        }

        // ---- chroma: lane = 8*mb + 4*plane + block (quad = one plane of one MB)
        {
            const int m = lane >> 3, plane = (lane >> 2) & 1, sub = lane & 3, bx = sub & 1, by = sub >> 1;
            const uint32_t* R = L.rec[m];
            const uint8_t* Rb = (const uint8_t*)R;
            const int mode = (int)((R[0] >> 8) & 255u);
            const int seg = (int)((R[0] >> 16) & 3u);
            const int has_top = (int)((R[0] >> 24) & 1u), has_left = (int)((R[0] >> 25) & 1u);
            const XmbMat& muv = S[seg].uv;
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
                c[k] = lv[k] * muv.q[tk];
            }
            if (m < nact) store_levels(levels + ((mb0 + m) * 25 + 17 + 4 * plane + sub) * 16, lv);
            uint32_t rw[4];
            recon_words(c, pw, rw);
#pragma unroll
            for (int r = 0; r < 4; r++) L.ct[plane][by * 4 + r][m * 2 + bx] = rw[r];
        }
        wsync();
    }

    // ---- reconstruction tiles back to the planes
    {
        uint8_t* RYf = RY + f * ysz + (size_t)mby * 16 * ys + x0 * 16;
        uint8_t* RUf = RU + f * csz + (size_t)mby * 8 * cs + x0 * 8;
        uint8_t* RVf = RV + f * csz + (size_t)mby * 8 * cs + x0 * 8;
        const int yc = lane & 7, yr = lane >> 3;
        const int cm = lane & 7, cr = (lane >> 3) & 7;
        if (yc < nact) {
            __builtin_nontemporal_store(*(const v4u*)&L.yt[yr][4 * yc], (v4u*)(RYf + yr * ys + yc * 16));
            __builtin_nontemporal_store(*(const v4u*)&L.yt[yr + 8][4 * yc], (v4u*)(RYf + (yr + 8) * ys + yc * 16));
        }
        if (cm < nact) {
            __builtin_nontemporal_store(*(const v2u*)&L.ct[0][cr][2 * cm], (v2u*)(RUf + cr * cs + cm * 8));
            __builtin_nontemporal_store(*(const v2u*)&L.ct[1][cr][2 * cm], (v2u*)(RVf + cr * cs + cm * 8));
        }
    }
}

extern "C" size_t zwk_xform_mb_seg_bytes(void) { return sizeof(XmbSeg) * 4; }

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

extern "C" hipError_t zwk_xform_mb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V,
                                   const uint8_t* recs, const void* segs, int mbw, int mbh, int nframes,
                                   int16_t* levels, uint8_t* RY, uint8_t* RU, uint8_t* RV, int variant)
{
    const long long waves = (long long)nframes * mbh * ((mbw + XMB_MBS - 1) / XMB_MBS);
    const unsigned grid = (unsigned)((waves + XMB_WAVES - 1) / XMB_WAVES);
    if (grid == 0) return hipSuccess;
    const XmbSeg* sg = (const XmbSeg*)segs;
    if (variant == 99)
        hipLaunchKernelGGL((k_xform_mb<true>), dim3(grid), dim3(64 * XMB_WAVES), 0, s, Y, U, V, recs, sg, mbw, mbh,
                           nframes, levels, RY, RU, RV);
    else
        hipLaunchKernelGGL((k_xform_mb<false>), dim3(grid), dim3(64 * XMB_WAVES), 0, s, Y, U, V, recs, sg, mbw, mbh,
                           nframes, levels, RY, RU, RV);
    return hipGetLastError();
}
