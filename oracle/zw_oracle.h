/* oracle/zw_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Public C API of the CPU restatement ("oracle") of zenwebp 0.2.0's VP8 lossy
 * path.  Loaded by tests/ (ctypes), __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg; never by the product library.
 *
 * Parity pinning: the decoder is pinned to libwebp (WebPDecodeYUV) and to the
 * reference's own golden PNGs (tests/reference/gallery1); transforms, bool coder
 * and trellis to the reference's in-crate known-answer tests.  The encoder's
 * mode decisions have no reference golden (the reference ships none): they are
 * a line-by-line restatement of encoder/vp8.rs + encoder/cost.rs, checked for
 * self-consistency (libwebp decodes our bitstream to our encoder's recon).
 */
#ifndef ZW_ORACLE_H
#define ZW_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OR_OK = 0,
    OR_EINVALID_DIMENSIONS = 1,
    OR_EINVALID_BUFFER_SIZE = 2,
    OR_EINVAL = 3,
    /* decoder errors (decoder/api.rs:79-110) */
    OR_EMAGIC = 10,
    OR_ECOLORSPACE = 11,
    OR_ELUMAMODE = 12,
    OR_EINTRAMODE = 13,
    OR_ECHROMAMODE = 14,
    OR_EBITSTREAM = 15,
    OR_EUNSUPPORTED = 16,
    OR_ENOTENOUGHDATA = 17,
};

typedef struct {
    uint8_t luma_mode;   /* 0 DC,1 V,2 H,3 TM,4 B */
    uint8_t bpred[16];
    uint8_t chroma_mode;
    uint8_t segment;
    uint8_t skip;
    uint8_t non_zero_dct; /* decoder only */
} or_mb_info;

/* Optional debug capture.  Any pointer may be NULL. */
typedef struct {
    uint8_t *src_y, *src_u, *src_v;       /* after RGB->YUV (MB padded) */
    uint8_t *recon_y, *recon_u, *recon_v; /* encoder pass-2 reconstruction */
    uint8_t *recon1_y;                    /* encoder pass-1 luma reconstruction */
    uint8_t *mb_alpha;                    /* analysis alphas, mbw*mbh */
    uint8_t *seg_map;                     /* mbw*mbh */
    or_mb_info *p1_info, *p2_info;        /* mbw*mbh each */
    int32_t *levels;                      /* pass 2: mbw*mbh*25*16 zigzag levels (0..15 Y, 16 Y2, 17..20 U, 21..24 V) */
    int32_t *i4_dump;                     /* pass 2 I4 MBs: mbw*mbh*16*34 (coeffs[16], pred[16], ctx0, mode) */
    uint32_t p1_stats[4][8][3][11];
    uint8_t final_probs[4][8][3][11];
    int seg_quant_index[4];
    int segments_enabled, filter_level, base_quant_index, skip_prob;
    int8_t p1_top_derr_last[1];
    int8_t *derr_in;                      /* pass 2: mbw*mbh*8 incoming error-diffusion terms (U top0, top1,
                                           * left0, left1, then V), the zw_transform_quant_mbs record order */
} or_enc_debug;

/* encode_frame_lossy (encoder/vp8.rs:3132): raw VP8 frame bytes (malloc'd). */
int or_encode(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, int quality,
              int method, uint8_t **out, size_t *out_len, or_enc_debug *dbg);
/* ... with nparts (1, 2, 4, 8) token partitions (vp8.rs:352-354, :1419-1421). */
int or_encode_parts(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, int quality,
                    int method, int nparts, uint8_t **out, size_t *out_len, or_enc_debug *dbg);
void or_free(void *p);

/* Vp8Decoder::decode_frame (decoder/vp8.rs:1526).  Planes are MB-aligned:
 * Y stride mbw*16 (mbh*16 rows), U/V stride mbw*8.  If unfiltered_y/u/v are
 * non-NULL they receive the pre-loop-filter reconstruction. */
typedef struct {
    int width, height, mbw, mbh;
    int filter_type, filter_level, sharpness;
    int segments_enabled, seg_delta_values, seg_lf_level[4], seg_quant_level[4];
    int lf_adj_enabled, ref_delta0, mode_delta0;
    int num_partitions;
} or_frame_hdr;

int or_decode_header(const uint8_t *data, size_t len, or_frame_hdr *hdr);
int or_decode(const uint8_t *data, size_t len, uint8_t *y, uint8_t *u, uint8_t *v,
              uint8_t *unfiltered_y, uint8_t *unfiltered_u, uint8_t *unfiltered_v,
              or_mb_info *mbinfo, or_frame_hdr *hdr_out);

/* Kernel-level oracles (for the device parity tests). */
void or_rgb_to_yuv420_c(const uint8_t *img, int w, int h, int bpp, uint8_t *y, uint8_t *u, uint8_t *v);
void or_fdct_c(int32_t *blk, int n);          /* n blocks, scalar dct4x4 */
void or_fdct_sse2_c(int32_t *blk, int n);     /* n blocks, SSE2 semantics */
void or_idct_c(int32_t *blk, int n);          /* n blocks, SSE2 i16 semantics */
void or_idct_scalar_c(int32_t *blk, int n);
void or_wht_c(int32_t *blk, int n);
void or_iwht_c(int32_t *blk, int n);
void or_loop_filter_c(uint8_t *y, uint8_t *u, uint8_t *v, int mbw, int mbh, const or_mb_info *mbs,
                      const or_frame_hdr *hdr);
void or_yuv_to_rgb_fancy_c(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int bpp, uint8_t *out);
/* encode_frame_lossless (encoder/api.rs:945-1173) and encode_alpha_lossless
 * (:1175-1222); *out is malloc'd (free with or_free). */
int or_encode_frame_lossless(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color,
                             int use_predictor, int implicit_dims, uint8_t **out, size_t *out_len);
int or_encode_alpha(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, uint8_t **out,
                    size_t *out_len);
/* <[(usize, u32)]>::sort_unstable_by_key(|&(_, k)| k) of Rust 1.92 (the
 * length-limit reassignment order of build_huffman_tree, api.rs:259-260);
 * sorts the (idx[i], key[i]) pairs in place. */
void or_rust_sort_unstable_by_key(uint32_t *idx, uint32_t *key, size_t n);
/* Streaming final transform over per-MB records (zw_transform_quant_mbs's
 * checker): levels [nframes*mbw*mbh][25][16] zigzag, recon MB-padded planes. */
void or_xform_mbs(int nframes, int mbw, int mbh, const uint8_t *y, const uint8_t *u, const uint8_t *v,
                  const uint8_t *recs, const int32_t *seg_qi, int16_t *levels, uint8_t *ry, uint8_t *ru, uint8_t *rv);
void or_yuv_to_rgb_simple_c(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int bpp, uint8_t *out);
void or_analyze(const uint8_t *Y, const uint8_t *U, const uint8_t *V, int width, int height,
                uint8_t *mb_alphas, uint32_t histo[256]);
int or_quality_to_quant_index(int quality);
int or_filter_level_for_quality(int quality);
int or_bool_encoder_kat(const int *ops, int nops, uint8_t *out, int out_cap);
int or_trellis_kat(const int32_t coeffs_in[16], int q_dc, int q_ac, int iq_dc, int iq_ac, uint32_t lambda,
                   int ctype, int first, int ctx0, int use_default_costs, int32_t out_levels[16],
                   int32_t out_coeffs[16]);
void or_quant_blocks_c(int n, const int32_t *coeffs, const uint8_t *ctx0, int ctype, int first, int use_trellis,
                       uint32_t lambda, int q_dc, int q_ac, int matrix_type, const uint8_t *probs, int32_t *levels,
                       int32_t *dequant);
uint32_t or_fixed_cost_i16(int mode);
uint32_t or_fixed_cost_uv(int mode);
size_t or_debug_struct_size(void);
/* known-answer-test entry points (fast_math.rs, cost.rs, prediction.rs, bit_reader.rs) */
float or_fm_roundf(float x);
double or_fm_round(double x);
double or_fm_cbrt(double x);
double or_fm_pow(double x, double n);
uint64_t or_rd_score(uint32_t sse, uint32_t rate, uint32_t lambda);
int or_t_transform(const uint8_t *in, int stride, const uint16_t w[16]);
void or_seg_lambdas(uint32_t q, uint32_t out[8]);
void or_add_residue_kat(uint8_t pblock[16], const int32_t r[16]);
int or_bool_read_kat(const uint8_t *data, size_t len, const int *ops, int nops, int *out);
void or_i4_preds_edge_c(const uint8_t e[13], uint8_t out[160]);

#ifdef __cplusplus
}
#endif
#endif
