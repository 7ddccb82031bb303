/* oracle/or_dsp.c -- TEST INFRASTRUCTURE ONLY (see or_internal.h).
 * Transforms, intra predictors, colour conversion and the VP8 loop filter,
 * restated from the reference crate zenwebp 0.2.0. */
#include "or_internal.h"

/* ------------------------------------------------------------------------ */
/* Transforms                                                               */
/* ------------------------------------------------------------------------ */

/* dct4x4_scalar, reference src/common/transform.rs:176-211 (i64 intermediates). */
void or_fdct(int32_t b[16])
{
    int64_t t[16];
    for (int i = 0; i < 16; i++) t[i] = b[i];
    for (int i = 0; i < 4; i++) {
        int64_t a = (t[i * 4] + t[i * 4 + 3]) * 8;
        int64_t bb = (t[i * 4 + 1] + t[i * 4 + 2]) * 8;
        int64_t c = (t[i * 4 + 1] - t[i * 4 + 2]) * 8;
        int64_t d = (t[i * 4] - t[i * 4 + 3]) * 8;
        t[i * 4] = (int32_t)(a + bb);
        t[i * 4 + 2] = (int32_t)(a - bb);
        t[i * 4 + 1] = (int32_t)((c * 2217 + d * 5352 + 14500) >> 12);
        t[i * 4 + 3] = (int32_t)((d * 2217 - c * 5352 + 7500) >> 12);
    }
    for (int i = 0; i < 4; i++) {
        int64_t a = t[i] + t[i + 12];
        int64_t bb = t[i + 4] + t[i + 8];
        int64_t c = t[i + 4] - t[i + 8];
        int64_t d = t[i] - t[i + 12];
        b[i] = (int32_t)((a + bb + 7) >> 4);
        b[i + 8] = (int32_t)((a - bb + 7) >> 4);
        b[i + 4] = (int32_t)(((c * 2217 + d * 5352 + 12000) >> 16) + (d != 0 ? 1 : 0));
        b[i + 12] = (int32_t)((d * 2217 - c * 5352 + 51000) >> 16);
    }
}

static inline int16_t w16(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
static inline int16_t sat16(int32_t v) { return (int16_t)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v)); }
static inline int16_t mulhi16(int16_t x, int k) { return (int16_t)(((int32_t)x * k) >> 16); }

/* dct4x4_sse2 (the default x86-64-v3 build of the reference), reference
 * src/common/transform_simd_intrinsics.rs:157-337: i16 lanes, madd to i32,
 * saturating packs, i16 column pass. */
void or_fdct_sse2(int32_t b[16])
{
    int16_t in[16], r[16];
    for (int i = 0; i < 16; i++) in[i] = (int16_t)b[i];
    for (int row = 0; row < 4; row++) {
        const int16_t *d = in + row * 4;
        int16_t a0 = w16(d[0] + d[3]), a1 = w16(d[1] + d[2]);
        int16_t a3 = w16(d[0] - d[3]), a2 = w16(d[1] - d[2]);
        int32_t t0 = a0 * 8 + a1 * 8;
        int32_t t2 = a0 * 8 - a1 * 8;
        int32_t t1 = (a3 * 5352 + a2 * 2217 + 1812) >> 9;
        int32_t t3 = (a3 * 2217 - a2 * 5352 + 937) >> 9;
        r[row * 4 + 0] = sat16(t0);
        r[row * 4 + 1] = sat16(t1);
        r[row * 4 + 2] = sat16(t2);
        r[row * 4 + 3] = sat16(t3);
    }
    for (int i = 0; i < 4; i++) {
        int16_t v0 = r[i], v1 = r[4 + i], v2 = r[8 + i], v3 = r[12 + i];
        int16_t a3 = w16(v0 - v3), a2 = w16(v1 - v2);
        int16_t a0 = w16(v0 + v3), a1 = w16(v1 + v2);
        int16_t c0 = w16(w16(a0 + 7) + a1), c2 = w16(w16(a0 + 7) - a1);
        int32_t e1 = (a3 * 5352 + a2 * 2217 + 12000 + 65536) >> 16;
        int32_t e3 = (a3 * 2217 - a2 * 5352 + 51000) >> 16;
        b[i] = (int16_t)(c0 >> 4);
        b[8 + i] = (int16_t)(c2 >> 4);
        b[4 + i] = w16(sat16(e1) + (a3 == 0 ? -1 : 0));
        b[12 + i] = sat16(e3);
    }
}

/* idct4x4_sse2 (default build), transform_simd_intrinsics.rs:478-632:
 * saturating i32->i16 pack, then both passes in wrapping i16 with
 * _mm_mulhi_epi16 by 20091 / -30068 and an i16 arithmetic >>3. */
void or_idct(int32_t b[16])
{
    int16_t x[16], t[16];
    for (int i = 0; i < 16; i++) x[i] = sat16(b[i]);
    for (int i = 0; i < 4; i++) {
        int16_t x0 = x[i], x1 = x[4 + i], x2 = x[8 + i], x3 = x[12 + i];
        int16_t a = w16(x0 + x2), bb = w16(x0 - x2);
        int16_t c = w16(w16(x1 - x3) + w16(mulhi16(x1, -30068) - mulhi16(x3, 20091)));
        int16_t d = w16(w16(x1 + x3) + w16(mulhi16(x1, 20091) + mulhi16(x3, -30068)));
        t[0 * 4 + i] = w16(a + d);
        t[1 * 4 + i] = w16(bb + c);
        t[2 * 4 + i] = w16(bb - c);
        t[3 * 4 + i] = w16(a - d);
    }
    for (int r = 0; r < 4; r++) {
        int16_t y0 = t[r * 4], y1 = t[r * 4 + 1], y2 = t[r * 4 + 2], y3 = t[r * 4 + 3];
        int16_t dc = w16(y0 + 4);
        int16_t a = w16(dc + y2), bb = w16(dc - y2);
        int16_t c = w16(w16(y1 - y3) + w16(mulhi16(y1, -30068) - mulhi16(y3, 20091)));
        int16_t d = w16(w16(y1 + y3) + w16(mulhi16(y1, 20091) + mulhi16(y3, -30068)));
        b[r * 4 + 0] = (int16_t)(w16(a + d) >> 3);
        b[r * 4 + 1] = (int16_t)(w16(bb + c) >> 3);
        b[r * 4 + 2] = (int16_t)(w16(bb - c) >> 3);
        b[r * 4 + 3] = (int16_t)(w16(a - d) >> 3);
    }
}

/* idct4x4_scalar, transform.rs:35-79 (i64). */
void or_idct_scalar(int32_t b[16])
{
    int64_t t[16];
    for (int i = 0; i < 16; i++) t[i] = b[i];
    for (int i = 0; i < 4; i++) {
        int64_t a1 = t[i] + t[8 + i], b1 = t[i] - t[8 + i];
        int64_t c1 = ((t[4 + i] * 35468) >> 16) - (t[12 + i] + ((t[12 + i] * 20091) >> 16));
        int64_t d1 = (t[4 + i] + ((t[4 + i] * 20091) >> 16)) + ((t[12 + i] * 35468) >> 16);
        t[i] = (int32_t)(a1 + d1);
        t[4 + i] = (int32_t)(b1 + c1);
        t[12 + i] = (int32_t)(a1 - d1);
        t[8 + i] = (int32_t)(b1 - c1);
    }
    for (int i = 0; i < 4; i++) {
        int64_t a1 = t[4 * i] + t[4 * i + 2], b1 = t[4 * i] - t[4 * i + 2];
        int64_t c1 = ((t[4 * i + 1] * 35468) >> 16) - (t[4 * i + 3] + ((t[4 * i + 3] * 20091) >> 16));
        int64_t d1 = (t[4 * i + 1] + ((t[4 * i + 1] * 20091) >> 16)) + ((t[4 * i + 3] * 35468) >> 16);
        b[4 * i] = (int32_t)((a1 + d1 + 4) >> 3);
        b[4 * i + 3] = (int32_t)((a1 - d1 + 4) >> 3);
        b[4 * i + 1] = (int32_t)((b1 + c1 + 4) >> 3);
        b[4 * i + 2] = (int32_t)((b1 - c1 + 4) >> 3);
    }
}

/* idct4x4_dc, transform.rs:13-16 */
void or_idct_dc(int32_t b[16])
{
    int32_t dc = (b[0] + 4) >> 3;
    for (int i = 0; i < 16; i++) b[i] = dc;
}

/* wht4x4, transform.rs:116-156 */
void or_wht(int32_t b[16])
{
    int64_t t[16];
    for (int i = 0; i < 16; i++) t[i] = b[i];
    for (int i = 0; i < 4; i++) {
        int64_t a = t[i * 4] + t[i * 4 + 3], bb = t[i * 4 + 1] + t[i * 4 + 2];
        int64_t c = t[i * 4 + 1] - t[i * 4 + 2], d = t[i * 4] - t[i * 4 + 3];
        t[i * 4] = (int32_t)(a + bb);
        t[i * 4 + 1] = (int32_t)(c + d);
        t[i * 4 + 2] = (int32_t)(a - bb);
        t[i * 4 + 3] = (int32_t)(d - c);
    }
    for (int i = 0; i < 4; i++) {
        int64_t a1 = t[i] + t[i + 12], b1 = t[i + 4] + t[i + 8];
        int64_t c1 = t[i + 4] - t[i + 8], d1 = t[i] - t[i + 12];
        int64_t a2 = a1 + b1, b2 = c1 + d1, c2 = a1 - b1, d2 = d1 - c1;
        /* Rust integer '/' truncates toward zero, as C does. */
        b[i] = (int32_t)((a2 + (a2 > 0 ? 1 : 0)) / 2);
        b[i + 4] = (int32_t)((b2 + (b2 > 0 ? 1 : 0)) / 2);
        b[i + 8] = (int32_t)((c2 + (c2 > 0 ? 1 : 0)) / 2);
        b[i + 12] = (int32_t)((d2 + (d2 > 0 ? 1 : 0)) / 2);
    }
}

/* iwht4x4, transform.rs:82-114 */
void or_iwht(int32_t b[16])
{
    for (int i = 0; i < 4; i++) {
        int32_t a1 = b[i] + b[12 + i], b1 = b[4 + i] + b[8 + i];
        int32_t c1 = b[4 + i] - b[8 + i], d1 = b[i] - b[12 + i];
        b[i] = a1 + b1;
        b[4 + i] = c1 + d1;
        b[8 + i] = a1 - b1;
        b[12 + i] = d1 - c1;
    }
    for (int r = 0; r < 4; r++) {
        int32_t *q = b + 4 * r;
        int32_t a1 = q[0] + q[3], b1 = q[1] + q[2], c1 = q[1] - q[2], d1 = q[0] - q[3];
        int32_t a2 = a1 + b1, b2 = c1 + d1, c2 = a1 - b1, d2 = d1 - c1;
        q[0] = (a2 + 3) >> 3;
        q[1] = (b2 + 3) >> 3;
        q[2] = (c2 + 3) >> 3;
        q[3] = (d2 + 3) >> 3;
    }
}

/* forward_dct_4x4, encoder/analysis.rs:172-209 (FTransform_C, result as i16). */
void or_ftransform_analysis(const uint8_t *src, const uint8_t *pred, int ss, int ps, int16_t out[16])
{
    int32_t tmp[16];
    for (int i = 0; i < 4; i++) {
        int d0 = src[i * ss] - pred[i * ps];
        int d1 = src[i * ss + 1] - pred[i * ps + 1];
        int d2 = src[i * ss + 2] - pred[i * ps + 2];
        int d3 = src[i * ss + 3] - pred[i * ps + 3];
        int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
        tmp[0 + i * 4] = (a0 + a1) * 8;
        tmp[2 + i * 4] = (a0 - a1) * 8;
        tmp[1 + i * 4] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
        tmp[3 + i * 4] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
    }
    for (int i = 0; i < 4; i++) {
        int a0 = tmp[0 + i] + tmp[12 + i], a1 = tmp[4 + i] + tmp[8 + i];
        int a2 = tmp[4 + i] - tmp[8 + i], a3 = tmp[0 + i] - tmp[12 + i];
        out[0 + i] = (int16_t)((a0 + a1 + 7) >> 4);
        out[8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
        out[4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0 ? 1 : 0));
        out[12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
    }
}

/* ------------------------------------------------------------------------ */
/* Prediction (common/prediction.rs)                                         */
/* ------------------------------------------------------------------------ */

/* create_border_luma, prediction.rs:15-74 */
void or_border_luma(uint8_t ws[OR_LUMA_WS], int mbx, int mby, int mbw, const uint8_t *top, const uint8_t *left)
{
    const int s = OR_BPS;
    memset(ws, 0, OR_LUMA_WS);
    if (mby == 0) {
        for (int i = 1; i < s; i++) ws[i] = 127;
    } else {
        for (int i = 0; i < 16; i++) ws[1 + i] = top[mbx * 16 + i];
        if (mbx == mbw - 1) {
            for (int i = 16; i < s - 1; i++) ws[1 + i] = top[mbx * 16 + 15];
        } else {
            /* zip(&top[mbx*16+16..]) over above[16..] (15 entries), bounded by top length */
            for (int i = 16; i < s - 1; i++) ws[1 + i] = top[mbx * 16 + i];
        }
    }
    for (int i = 17; i < 21; i++) {
        ws[4 * s + i] = ws[i];
        ws[8 * s + i] = ws[i];
        ws[12 * s + i] = ws[i];
    }
    if (mbx == 0) {
        for (int i = 0; i < 16; i++) ws[(i + 1) * s] = 129;
    } else {
        for (int i = 0; i < 16; i++) ws[(i + 1) * s] = left[1 + i];
    }
    ws[0] = mby == 0 ? 127 : (mbx == 0 ? 129 : left[0]);
}

/* create_border_chroma, prediction.rs:85-130 */
void or_border_chroma(uint8_t ws[OR_CHROMA_WS], int mbx, int mby, const uint8_t *top, const uint8_t *left)
{
    const int s = OR_BPS;
    memset(ws, 0, OR_CHROMA_WS);
    if (mby == 0) {
        for (int i = 1; i < s; i++) ws[i] = 127;
    } else {
        /* zip(&top[mbx*8..]): the chroma top border holds exactly mbw*8 bytes;
         * callers pass buffers padded so reading past 8 is harmless and only
         * [1..9) is ever consumed by the 8x8 predictors. */
        for (int i = 0; i < 8; i++) ws[1 + i] = top[mbx * 8 + i];
    }
    if (mbx == 0) {
        for (int y = 0; y < 8; y++) ws[(y + 1) * s] = 129;
    } else {
        for (int y = 0; y < 8; y++) ws[(y + 1) * s] = left[1 + y];
    }
    ws[0] = mby == 0 ? 127 : (mbx == 0 ? 129 : left[0]);
}

/* add_residue, prediction.rs:138-153 */
void or_add_residue(uint8_t *ws, const int32_t r[16], int y0, int x0, int stride)
{
    int pos = y0 * stride + x0;
    for (int row = 0; row < 4; row++) {
        for (int k = 0; k < 4; k++) ws[pos + k] = (uint8_t)or_clamp(r[row * 4 + k] + ws[pos + k], 0, 255);
        pos += stride;
    }
}

static inline uint8_t avg3(int l, int t, int r) { return (uint8_t)((l + 2 * t + r + 2) >> 2); }
static inline uint8_t avg2(int t, int r) { return (uint8_t)((t + r + 1) >> 1); }
/* KAT entry points: avg3 / avg2 (prediction.rs:154-161) and the edge gathers
 * top_pixels (:349) / edge_pixels (:373) as or_i4_preds below reads them. */
int or_avg3(int l, int t, int r) { return avg3(l, t, r); }
int or_avg2(int t, int r) { return avg2(t, r); }
void or_top_pixels(const uint8_t *a, int x0, int y0, int stride, uint8_t out[8])
{
    memcpy(out, a + (y0 - 1) * stride + x0, 8);
}
void or_edge_pixels(const uint8_t *a, int x0, int y0, int stride, uint8_t out[9])
{
    /* e0..e3: left column bottom-up, e4: corner, e5..e8: top row */
    for (int k = 0; k < 4; k++) out[k] = a[(y0 + 3 - k) * stride + x0 - 1];
    out[4] = a[(y0 - 1) * stride + x0 - 1];
    for (int k = 0; k < 4; k++) out[5 + k] = a[(y0 - 1) * stride + x0 + k];
}

/* predict_vpred, prediction.rs:164 */
void or_pred_v(uint8_t *a, int size, int x0, int y0, int stride)
{
    for (int y = 0; y < size; y++) memcpy(a + (y0 + y) * stride + x0, a + (y0 - 1) * stride + x0, size);
}

/* predict_hpred, prediction.rs:174 */
void or_pred_h(uint8_t *a, int size, int x0, int y0, int stride)
{
    for (int y = 0; y < size; y++) memset(a + (y0 + y) * stride + x0, a[(y0 + y) * stride + x0 - 1], size);
}

/* predict_dcpred, prediction.rs:182-211 */
void or_pred_dc(uint8_t *a, int size, int stride, int above, int left)
{
    uint32_t sum = 0;
    int shf = size == 8 ? 2 : 3;
    if (left) {
        for (int y = 0; y < size; y++) sum += a[(y + 1) * stride];
        shf++;
    }
    if (above) {
        for (int x = 1; x <= size; x++) sum += a[x];
        shf++;
    }
    uint32_t dc = (!left && !above) ? 128 : ((sum + (1u << (shf - 1))) >> shf);
    for (int y = 0; y < size; y++) memset(a + 1 + stride * (y + 1), (int)(uint8_t)dc, size);
}

/* predict_tmpred, prediction.rs:293-324 */
void or_pred_tm(uint8_t *a, int size, int x0, int y0, int stride)
{
    int p = a[(y0 - 1) * stride + x0 - 1];
    const uint8_t *above = a + (y0 - 1) * stride + x0;
    for (int y = 0; y < size; y++) {
        int lmp = a[(y0 + y) * stride + x0 - 1] - p;
        for (int x = 0; x < size; x++) a[(y0 + y) * stride + x0 + x] = (uint8_t)or_clamp(lmp + above[x], 0, 255);
    }
}

/* I4Predictions::compute, prediction.rs:568-855 (all ten 4x4 predictors). */
void or_i4_preds(const uint8_t *src, int x0, int y0, int stride, uint8_t d[10][16])
{
    uint8_t T[8], E[9];
    or_top_pixels(src, x0, y0, stride, T);
    or_edge_pixels(src, x0, y0, stride, E);
    int a0 = T[0], a1 = T[1], a2 = T[2], a3 = T[3], a4 = T[4], a5 = T[5], a6 = T[6], a7 = T[7];
    int e0 = E[0], e1 = E[1], e2 = E[2], e3 = E[3], e4 = E[4], e5 = E[5], e6 = E[6], e7 = E[7], e8 = E[8];
    int p = e4, l0 = e3, l1 = e2, l2 = e1, l3 = e0;
    /* DC */
    {
        uint32_t v = 4 + a0 + a1 + a2 + a3 + l0 + l1 + l2 + l3;
        memset(d[0], (int)(uint8_t)(v >> 3), 16);
    }
    /* TM */
    {
        int L[4] = {l0, l1, l2, l3}, A[4] = {a0, a1, a2, a3};
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) d[1][y * 4 + x] = (uint8_t)or_clamp(L[y] - p + A[x], 0, 255);
    }
    /* VE */
    {
        uint8_t av[4] = {avg3(p, a0, a1), avg3(a0, a1, a2), avg3(a1, a2, a3), avg3(a2, a3, a4)};
        for (int y = 0; y < 4; y++) memcpy(d[2] + y * 4, av, 4);
    }
    /* HE */
    {
        uint8_t av[4] = {avg3(p, l0, l1), avg3(l0, l1, l2), avg3(l1, l2, l3), avg3(l2, l3, l3)};
        for (int y = 0; y < 4; y++) memset(d[3] + y * 4, av[y], 4);
    }
    /* LD */
    {
        uint8_t av[7] = {avg3(a0, a1, a2), avg3(a1, a2, a3), avg3(a2, a3, a4), avg3(a3, a4, a5),
                         avg3(a4, a5, a6), avg3(a5, a6, a7), avg3(a6, a7, a7)};
        for (int y = 0; y < 4; y++) memcpy(d[4] + y * 4, av + y, 4);
    }
    /* RD */
    {
        uint8_t av[7] = {avg3(e0, e1, e2), avg3(e1, e2, e3), avg3(e2, e3, e4), avg3(e3, e4, e5),
                         avg3(e4, e5, e6), avg3(e5, e6, e7), avg3(e6, e7, e8)};
        for (int y = 0; y < 4; y++) memcpy(d[5] + y * 4, av + 3 - y, 4);
    }
    /* VR */
    {
        uint8_t *q = d[6];
        q[12] = avg3(e1, e2, e3);
        q[8] = avg3(e2, e3, e4);
        q[13] = q[4] = avg3(e3, e4, e5);
        q[9] = q[0] = avg2(e4, e5);
        q[14] = q[5] = avg3(e4, e5, e6);
        q[10] = q[1] = avg2(e5, e6);
        q[15] = q[6] = avg3(e5, e6, e7);
        q[11] = q[2] = avg2(e6, e7);
        q[7] = avg3(e6, e7, e8);
        q[3] = avg2(e7, e8);
    }
    /* VL */
    {
        uint8_t *q = d[7];
        q[0] = avg2(a0, a1);
        q[4] = avg3(a0, a1, a2);
        q[8] = q[1] = avg2(a1, a2);
        q[5] = q[12] = avg3(a1, a2, a3);
        q[9] = q[2] = avg2(a2, a3);
        q[13] = q[6] = avg3(a2, a3, a4);
        q[10] = q[3] = avg2(a3, a4);
        q[14] = q[7] = avg3(a3, a4, a5);
        q[11] = avg3(a4, a5, a6);
        q[15] = avg3(a5, a6, a7);
    }
    /* HD */
    {
        uint8_t *q = d[8];
        q[12] = avg2(e0, e1);
        q[13] = avg3(e0, e1, e2);
        q[8] = q[14] = avg2(e1, e2);
        q[9] = q[15] = avg3(e1, e2, e3);
        q[10] = q[4] = avg2(e2, e3);
        q[11] = q[5] = avg3(e2, e3, e4);
        q[6] = q[0] = avg2(e3, e4);
        q[7] = q[1] = avg3(e3, e4, e5);
        q[2] = avg3(e4, e5, e6);
        q[3] = avg3(e5, e6, e7);
    }
    /* HU */
    {
        uint8_t *q = d[9];
        q[0] = avg2(l0, l1);
        q[1] = avg3(l0, l1, l2);
        q[2] = q[4] = avg2(l1, l2);
        q[3] = q[5] = avg3(l1, l2, l3);
        q[6] = q[8] = avg2(l2, l3);
        q[7] = q[9] = avg3(l2, l3, l3);
        q[10] = q[11] = q[12] = q[13] = q[14] = q[15] = (uint8_t)l3;
    }
}

/* The in-place predict_b* functions (prediction.rs:326-555) write exactly the
 * values I4Predictions::compute produces for the same border; restate them via
 * the table form and copy into the work buffer. */
void or_pred_b(uint8_t *a, int mode, int x0, int y0, int stride)
{
    uint8_t d[10][16];
    or_i4_preds(a, x0, y0, stride, d);
    for (int y = 0; y < 4; y++) memcpy(a + (y0 + y) * stride + x0, d[mode] + y * 4, 4);
}

/* ------------------------------------------------------------------------ */
/* Colour conversion (decoder/yuv.rs)                                         */
/* ------------------------------------------------------------------------ */

#define YUV_FIX 16
#define YUV_HALF (1 << (YUV_FIX - 1))

/* rgb_to_y yuv.rs:859 */
static inline uint8_t rgb_y(const uint8_t *p)
{
    int l = 16839 * p[0] + 33059 * p[1] + 6420 * p[2];
    return (uint8_t)((l + YUV_HALF + (16 << YUV_FIX)) >> YUV_FIX);
}
/* rgb_to_u_raw / rgb_to_v_raw yuv.rs:889-900 */
static inline int rgb_u_raw(const uint8_t *p) { return -9719 * p[0] - 19081 * p[1] + 28800 * p[2] + (128 << YUV_FIX); }
static inline int rgb_v_raw(const uint8_t *p) { return 28800 * p[0] - 24116 * p[1] - 4684 * p[2] + (128 << YUV_FIX); }
/* rgb_to_u_avg / rgb_to_v_avg yuv.rs:866-887 (truncating 'as u8', no clip) */
static inline uint8_t uv_avg(int s) { return (uint8_t)((s + (YUV_HALF << 2)) >> (YUV_FIX + 2)); }

/* convert_image_yuv::<BPP> yuv.rs:656-804, convert_image_y yuv.rs:806-857 (bpp 1/2). */
void or_rgb_to_yuv420(const uint8_t *img, int w, int h, int bpp, uint8_t *Y, uint8_t *U, uint8_t *V)
{
    int mbw = (w + 15) / 16, mbh = (h + 15) / 16;
    int lw = 16 * mbw, cw = 8 * mbw;
    if (bpp <= 2) {
        memset(U, 127, (size_t)cw * 8 * mbh);
        memset(V, 127, (size_t)cw * 8 * mbh);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) Y[y * lw + x] = img[((size_t)y * w + x) * bpp];
    } else {
        for (int rp = 0; rp < h / 2; rp++) {
            int r1 = 2 * rp, r2 = r1 + 1;
            for (int cp = 0; cp < w / 2; cp++) {
                int c1 = 2 * cp, c2 = c1 + 1;
                const uint8_t *p1 = img + ((size_t)r1 * w + c1) * bpp, *p2 = img + ((size_t)r1 * w + c2) * bpp;
                const uint8_t *p3 = img + ((size_t)r2 * w + c1) * bpp, *p4 = img + ((size_t)r2 * w + c2) * bpp;
                Y[r1 * lw + c1] = rgb_y(p1);
                Y[r1 * lw + c2] = rgb_y(p2);
                Y[r2 * lw + c1] = rgb_y(p3);
                Y[r2 * lw + c2] = rgb_y(p4);
                U[rp * cw + cp] = uv_avg(rgb_u_raw(p1) + rgb_u_raw(p2) + rgb_u_raw(p3) + rgb_u_raw(p4));
                V[rp * cw + cp] = uv_avg(rgb_v_raw(p1) + rgb_v_raw(p2) + rgb_v_raw(p3) + rgb_v_raw(p4));
            }
            if (w & 1) {
                int c = w - 1;
                const uint8_t *p1 = img + ((size_t)r1 * w + c) * bpp, *p3 = img + ((size_t)r2 * w + c) * bpp;
                Y[r1 * lw + c] = rgb_y(p1);
                Y[r2 * lw + c] = rgb_y(p3);
                U[rp * cw + w / 2] = uv_avg(2 * rgb_u_raw(p1) + 2 * rgb_u_raw(p3));
                V[rp * cw + w / 2] = uv_avg(2 * rgb_v_raw(p1) + 2 * rgb_v_raw(p3));
            }
        }
        if (h & 1) {
            int r = h - 1, rp = h / 2;
            for (int cp = 0; cp < w / 2; cp++) {
                int c1 = 2 * cp, c2 = c1 + 1;
                const uint8_t *p1 = img + ((size_t)r * w + c1) * bpp, *p2 = img + ((size_t)r * w + c2) * bpp;
                Y[r * lw + c1] = rgb_y(p1);
                Y[r * lw + c2] = rgb_y(p2);
                U[rp * cw + cp] = uv_avg(2 * rgb_u_raw(p1) + 2 * rgb_u_raw(p2));
                V[rp * cw + cp] = uv_avg(2 * rgb_v_raw(p1) + 2 * rgb_v_raw(p2));
            }
            if (w & 1) {
                const uint8_t *p = img + ((size_t)r * w + (w - 1)) * bpp;
                Y[r * lw + w - 1] = rgb_y(p);
                U[rp * cw + w / 2] = uv_avg(4 * rgb_u_raw(p));
                V[rp * cw + w / 2] = uv_avg(4 * rgb_v_raw(p));
            }
        }
    }
    /* MB padding by edge replication (yuv.rs:765-803 / :841-856) */
    for (int y = 0; y < h; y++) {
        uint8_t last = Y[y * lw + w - 1];
        for (int x = w; x < lw; x++) Y[y * lw + x] = last;
    }
    for (int y = h; y < 16 * mbh; y++) memcpy(Y + (size_t)y * lw, Y + (size_t)(h - 1) * lw, lw);
    if (bpp > 2) {
        int ch = (h + 1) / 2, acw = (w + 1) / 2;
        for (int y = 0; y < ch; y++) {
            uint8_t lu = U[y * cw + acw - 1], lv = V[y * cw + acw - 1];
            for (int x = acw; x < cw; x++) {
                U[y * cw + x] = lu;
                V[y * cw + x] = lv;
            }
        }
        for (int y = ch; y < 8 * mbh; y++) {
            memcpy(U + (size_t)y * cw, U + (size_t)(ch - 1) * cw, cw);
            memcpy(V + (size_t)y * cw, V + (size_t)(ch - 1) * cw, cw);
        }
    }
}

/* yuv_to_r/g/b, yuv.rs:33-78 */
static inline int mulhi8(int v, int c) { return (v * c) >> 8; }
static inline uint8_t clip6(int v) { return (uint8_t)or_clamp(v >> 6, 0, 255); }
static inline void set_px(uint8_t *o, int y, int u, int v)
{
    o[0] = clip6(mulhi8(y, 19077) + mulhi8(v, 26149) - 14234);
    o[1] = clip6(mulhi8(y, 19077) - mulhi8(u, 6419) - mulhi8(v, 13320) + 8708);
    o[2] = clip6(mulhi8(y, 19077) + mulhi8(u, 33050) - 17685);
}
static inline int fancy(int m, int s1, int s2, int t) { return (9 * m + 3 * s1 + 3 * s2 + t + 8) / 16; }

static void fancy_row2(uint8_t *o, const uint8_t *yr, int w, const uint8_t *u1, const uint8_t *u2,
                       const uint8_t *v1, const uint8_t *v2, int cwid, int bpp)
{
    set_px(o, yr[0], fancy(u1[0], u1[0], u2[0], u2[0]), fancy(v1[0], v1[0], v2[0], v2[0]));
    int x = 1, k = 0;
    for (; x + 1 < w && k + 1 < cwid; x += 2, k++) {
        set_px(o + x * bpp, yr[x], fancy(u1[k], u1[k + 1], u2[k], u2[k + 1]), fancy(v1[k], v1[k + 1], v2[k], v2[k + 1]));
        set_px(o + (x + 1) * bpp, yr[x + 1], fancy(u1[k + 1], u1[k], u2[k + 1], u2[k]),
               fancy(v1[k + 1], v1[k], v2[k + 1], v2[k]));
    }
    if (x < w) {
        int l = cwid - 1;
        set_px(o + x * bpp, yr[x], fancy(u1[l], u1[l], u2[l], u2[l]), fancy(v1[l], v1[l], v2[l], v2[l]));
    }
}

static void fancy_row1(uint8_t *o, const uint8_t *yr, int w, const uint8_t *u, const uint8_t *v, int cwid, int bpp)
{
    set_px(o, yr[0], u[0], v[0]);
    int x = 1, k = 0;
    for (; x + 1 < w && k + 1 < cwid; x += 2, k++) {
        set_px(o + x * bpp, yr[x], fancy(u[k], u[k + 1], u[k], u[k + 1]), fancy(v[k], v[k + 1], v[k], v[k + 1]));
        set_px(o + (x + 1) * bpp, yr[x + 1], fancy(u[k + 1], u[k], u[k + 1], u[k]), fancy(v[k + 1], v[k], v[k + 1], v[k]));
    }
    if (x < w) set_px(o + x * bpp, yr[x], u[cwid - 1], v[cwid - 1]);
}

/* fill_rgb_buffer_fancy, yuv.rs:82-160 (+ row helpers :264-395).  For BPP 4 the
 * caller fills alpha. */
void or_yuv_to_rgb_fancy(const uint8_t *Y, const uint8_t *U, const uint8_t *V, int w, int h,
                         int bw, int bpp, uint8_t *out)
{
    int cbw = bw / 2, cwid = (w + 1) / 2;
    fancy_row1(out, Y, w, U, V, cwid, bpp);
    int r = 1, cr = 0;
    for (; r + 2 <= h; r += 2, cr++) {
        const uint8_t *u1 = U + cr * cbw, *u2 = U + (cr + 1) * cbw;
        const uint8_t *v1 = V + cr * cbw, *v2 = V + (cr + 1) * cbw;
        fancy_row2(out + (size_t)r * w * bpp, Y + (size_t)r * bw, w, u1, u2, v1, v2, cwid, bpp);
        fancy_row2(out + (size_t)(r + 1) * w * bpp, Y + (size_t)(r + 1) * bw, w, u2, u1, v2, v1, cwid, bpp);
    }
    if (r < h) {
        int ch = (h + 1) / 2;
        fancy_row1(out + (size_t)r * w * bpp, Y + (size_t)r * bw, w, U + (ch - 1) * cbw, V + (ch - 1) * cbw, cwid, bpp);
    }
}

/* fill_rgb_buffer_simple + fill_rgba_row_simple_scalar, yuv.rs:402-515: every
 * chroma row serves two luma rows, every chroma sample two pixels; the odd
 * final pixel of a row takes the next chroma sample.  For BPP 4 the caller
 * fills alpha. */
void or_yuv_to_rgb_simple(const uint8_t *Y, const uint8_t *U, const uint8_t *V, int w, int h,
                          int bw, int bpp, uint8_t *out)
{
    int cbw = bw / 2;
    for (int r = 0; r < h; r++) {
        const uint8_t *yr = Y + (size_t)r * bw, *ur = U + (size_t)(r / 2) * cbw, *vr = V + (size_t)(r / 2) * cbw;
        uint8_t *o = out + (size_t)r * w * bpp;
        for (int x = 0; x < w; x++) set_px(o + (size_t)x * bpp, yr[x], ur[x / 2], vr[x / 2]);
    }
}

/* ------------------------------------------------------------------------ */
/* Loop filter (decoder/loop_filter.rs; order decoder/vp8.rs:1172-1345)      */
/* ------------------------------------------------------------------------ */

static inline int c8(int v) { return or_clamp(v, -128, 127); }
static inline int u2s(int v) { return v - 128; }
static inline uint8_t s2u(int v) { return (uint8_t)(c8(v) + 128); }

/* common_adjust_vertical loop_filter.rs:28 (generic stride form) */
static int common_adjust(int outer_taps, uint8_t *p, int s)
{
    int p1 = u2s(p[-2 * s]), p0 = u2s(p[-s]), q0 = u2s(p[0]), q1 = u2s(p[s]);
    int outer = outer_taps ? c8(p1 - q1) : 0;
    int a = c8(outer + 3 * (q0 - p0));
    int b = c8(a + 3) >> 3;
    a = c8(a + 4) >> 3;
    p[0] = s2u(q0 - a);
    p[-s] = s2u(p0 + b);
    return a;
}
static inline int simple_thresh(int lim, const uint8_t *p, int s)
{
    return or_abs(p[-s] - p[0]) * 2 + or_abs(p[-2 * s] - p[s]) / 2 <= lim;
}
static inline int should_filter(int il, int el, const uint8_t *p, int s)
{
    return simple_thresh(el, p, s) && or_abs(p[-4 * s] - p[-3 * s]) <= il && or_abs(p[-3 * s] - p[-2 * s]) <= il &&
           or_abs(p[-2 * s] - p[-s]) <= il && or_abs(p[3 * s] - p[2 * s]) <= il &&
           or_abs(p[2 * s] - p[s]) <= il && or_abs(p[s] - p[0]) <= il;
}
static inline int hev(int t, const uint8_t *p, int s) { return or_abs(p[-2 * s] - p[-s]) > t || or_abs(p[s] - p[0]) > t; }

/* simple_segment_* loop_filter.rs:144 */
static void f_simple(int el, uint8_t *p, int s)
{
    if (simple_thresh(el, p, s)) common_adjust(1, p, s);
}
/* subblock_filter_* loop_filter.rs:167 */
static void f_inner(int ht, int il, int el, uint8_t *p, int s)
{
    if (should_filter(il, el, p, s)) {
        int hv = hev(ht, p, s);
        int a = (common_adjust(hv, p, s) + 1) >> 1;
        if (!hv) {
            p[s] = s2u(u2s(p[s]) - a);
            p[-2 * s] = s2u(u2s(p[-2 * s]) + a);
        }
    }
}
/* macroblock_filter_* loop_filter.rs:212 */
static void f_mb(int ht, int il, int el, uint8_t *p, int s)
{
    if (should_filter(il, el, p, s)) {
        if (!hev(ht, p, s)) {
            int p2 = u2s(p[-3 * s]), p1 = u2s(p[-2 * s]), p0 = u2s(p[-s]);
            int q0 = u2s(p[0]), q1 = u2s(p[s]), q2 = u2s(p[2 * s]);
            int w = c8(c8(p1 - q1) + 3 * (q0 - p0));
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
            common_adjust(1, p, s);
        }
    }
}

/* calculate_filter_parameters, decoder/vp8.rs:1470-1523 */
void or_filter_params(const or_filter_hdr *h, const or_mb_flags *mb, int *level, int *ilimit, int *hevt)
{
    int fl = h->filter_level;
    *level = 0; *ilimit = 0; *hevt = 0;
    if (fl == 0) return;
    if (h->segments_enabled) {
        if (h->seg_delta_values) fl += h->seg_lf_level[mb->segment];
        else fl = h->seg_lf_level[mb->segment];
    }
    fl = or_clamp(fl, 0, 63);
    if (h->lf_adj_enabled) {
        fl += h->ref_delta0;
        if (mb->luma_mode == 4) fl += h->mode_delta0;
    }
    fl = or_clamp(fl, 0, 63);
    int il = fl;
    if (h->sharpness > 0) {
        il >>= (h->sharpness > 4) ? 2 : 1;
        if (il > 9 - h->sharpness) il = 9 - h->sharpness;
    }
    if (il == 0) il = 1;
    *level = fl;
    *ilimit = il;
    *hevt = fl >= 40 ? 2 : (fl >= 15 ? 1 : 0);
}

/* filter_row_in_cache decoder/vp8.rs:1172-1345, applied in place over whole
 * planes in raster MB order (the row cache with 8 extra rows is equivalent). */
void or_loop_filter_frame(uint8_t *Y, uint8_t *U, uint8_t *V, int mbw, int mbh,
                          const or_mb_flags *mbs, const or_filter_hdr *h)
{
    int ys = mbw * 16, cs = mbw * 8;
    for (int mby = 0; mby < mbh; mby++) {
        for (int mbx = 0; mbx < mbw; mbx++) {
            const or_mb_flags *mb = &mbs[mby * mbw + mbx];
            int L, I, H;
            or_filter_params(h, mb, &L, &I, &H);
            if (L == 0) continue;
            int mbe = (L + 2) * 2 + I, sube = L * 2 + I;
            int inner = mb->luma_mode == 4 || (!mb->skip && mb->non_zero_dct);
            uint8_t *yb = Y + (size_t)mby * 16 * ys + mbx * 16;
            uint8_t *ub = U + (size_t)mby * 8 * cs + mbx * 8;
            uint8_t *vb = V + (size_t)mby * 8 * cs + mbx * 8;
            if (mbx > 0) {
                if (h->filter_type) {
                    for (int r = 0; r < 16; r++) f_simple(mbe, yb + r * ys, 1);
                } else {
                    for (int r = 0; r < 16; r++) f_mb(H, I, mbe, yb + r * ys, 1);
                    for (int r = 0; r < 8; r++) f_mb(H, I, mbe, ub + r * cs, 1);
                    for (int r = 0; r < 8; r++) f_mb(H, I, mbe, vb + r * cs, 1);
                }
            }
            if (inner) {
                if (h->filter_type) {
                    for (int x = 4; x < 16; x += 4)
                        for (int r = 0; r < 16; r++) f_simple(sube, yb + r * ys + x, 1);
                } else {
                    for (int x = 4; x < 16; x += 4)
                        for (int r = 0; r < 16; r++) f_inner(H, I, sube, yb + r * ys + x, 1);
                    for (int r = 0; r < 8; r++) f_inner(H, I, sube, ub + r * cs + 4, 1);
                    for (int r = 0; r < 8; r++) f_inner(H, I, sube, vb + r * cs + 4, 1);
                }
            }
            if (mby > 0) {
                if (h->filter_type) {
                    for (int c = 0; c < 16; c++) f_simple(mbe, yb + c, ys);
                } else {
                    for (int c = 0; c < 16; c++) f_mb(H, I, mbe, yb + c, ys);
                    for (int c = 0; c < 8; c++) f_mb(H, I, mbe, ub + c, cs);
                    for (int c = 0; c < 8; c++) f_mb(H, I, mbe, vb + c, cs);
                }
            }
            if (inner) {
                if (h->filter_type) {
                    for (int y = 4; y < 16; y += 4)
                        for (int c = 0; c < 16; c++) f_simple(sube, yb + y * ys + c, ys);
                } else {
                    for (int y = 4; y < 16; y += 4)
                        for (int c = 0; c < 16; c++) f_inner(H, I, sube, yb + y * ys + c, ys);
                    for (int c = 0; c < 8; c++) f_inner(H, I, sube, ub + 4 * cs + c, cs);
                    for (int c = 0; c < 8; c++) f_inner(H, I, sube, vb + 4 * cs + c, cs);
                }
            }
        }
    }
}
