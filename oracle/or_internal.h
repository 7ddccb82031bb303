/* oracle/or_internal.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of zenwebp 0.2.0's VP8 lossy pipeline (the reference at
 * /root/reference).  Used only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker; never linked into the product library.
 * Every function cites the reference file:line it restates.
 */
#ifndef OR_INTERNAL_H
#define OR_INTERNAL_H

#include <stdint.h>
#include <stddef.h>
#include <string.h>

#define ZW_TABLE(T, N, D, ...) static const T N D = {__VA_ARGS__};
#include "or_tables.inc"
#undef ZW_TABLE

#define OR_BPS 32 /* prediction work-buffer stride (prediction.rs:10 LUMA_STRIDE) */
#define OR_LUMA_WS (OR_BPS * 17)
#define OR_CHROMA_WS (OR_BPS * 9)

static inline int or_clamp(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline int or_abs(int v) { return v < 0 ? -v : v; }

/* ---- transforms (common/transform.rs, transform_simd_intrinsics.rs) ---- */
void or_fdct(int32_t blk[16]);             /* dct4x4_scalar transform.rs:176 */
void or_fdct_sse2(int32_t blk[16]);        /* dct4x4_sse2 transform_simd_intrinsics.rs:157 */
void or_idct(int32_t blk[16]);             /* idct4x4_sse2 transform_simd_intrinsics.rs:478 */
void or_idct_scalar(int32_t blk[16]);      /* idct4x4_scalar transform.rs:35 */
void or_idct_dc(int32_t blk[16]);          /* idct4x4_dc transform.rs:13 */
void or_wht(int32_t blk[16]);              /* wht4x4 transform.rs:116 */
void or_iwht(int32_t blk[16]);             /* iwht4x4 transform.rs:82 */
void or_ftransform_analysis(const uint8_t *src, const uint8_t *pred, int ss, int ps, int16_t out[16]);
                                           /* forward_dct_4x4 analysis.rs:172 */

/* ---- prediction (common/prediction.rs) ---- */
void or_border_luma(uint8_t ws[OR_LUMA_WS], int mbx, int mby, int mbw, const uint8_t *top, const uint8_t *left);
void or_border_chroma(uint8_t ws[OR_CHROMA_WS], int mbx, int mby, const uint8_t *top, const uint8_t *left);
void or_add_residue(uint8_t *ws, const int32_t r[16], int y0, int x0, int stride);
void or_pred_v(uint8_t *a, int size, int x0, int y0, int stride);
void or_pred_h(uint8_t *a, int size, int x0, int y0, int stride);
void or_pred_dc(uint8_t *a, int size, int stride, int above, int left);
void or_pred_tm(uint8_t *a, int size, int x0, int y0, int stride);
void or_pred_b(uint8_t *a, int mode, int x0, int y0, int stride);   /* predict_b* */
void or_i4_preds(const uint8_t *src, int x0, int y0, int stride, uint8_t out[10][16]); /* I4Predictions::compute :568 */

/* ---- colour (decoder/yuv.rs) ---- */
void or_rgb_to_yuv420(const uint8_t *img, int w, int h, int bpp, uint8_t *y, uint8_t *u, uint8_t *v);
void or_yuv_to_rgb_simple(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int bw, int bpp,
                          uint8_t *out);
void or_yuv_to_rgb_fancy(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h,
                         int buffer_width, int bpp, uint8_t *out);

/* ---- loop filter (decoder/loop_filter.rs, decoder/vp8.rs:1172) ---- */
typedef struct {
    uint8_t luma_mode;     /* 0..4 (4 = B_PRED) */
    uint8_t segment;
    uint8_t skip;          /* coeffs_skipped */
    uint8_t non_zero_dct;
} or_mb_flags;

typedef struct {
    int filter_type;       /* 1 = simple */
    int filter_level;
    int sharpness;
    int segments_enabled;
    int seg_delta_values;  /* per-frame (all segments share) */
    int seg_lf_level[4];
    int lf_adj_enabled;
    int ref_delta0;
    int mode_delta0;
} or_filter_hdr;

void or_filter_params(const or_filter_hdr *h, const or_mb_flags *mb, int *level, int *ilimit, int *hev);
void or_loop_filter_frame(uint8_t *y, uint8_t *u, uint8_t *v, int mbw, int mbh,
                          const or_mb_flags *mbs, const or_filter_hdr *h);

#endif
