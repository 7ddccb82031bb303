/* zwebp.h -- C ABI of the MI355X-native VP8 lossy block-transform pipeline.
 *
 * Drop-in boundary for zenwebp 0.2.0's lossy path (reference crate at
 * imazen/image-webp).  The reference has no FFI of its own; each entry point
 * below replaces one internal seam or public Rust API and cites it:
 *
 *   zw_encode_frame_lossy   encode_frame_lossy        src/encoder/vp8.rs:3132-3153
 *   zw_encode_webp          WebPEncoder::encode       src/encoder/api.rs:1291-1398
 *                           (EncoderParams::lossy(q, m); RGBA / LA inputs get VP8X + ALPH)
 *   zw_encode_webp_ex       WebPEncoder::{set_params, set_icc_profile, set_exif_metadata,
 *                           set_xmp_metadata, encode}  src/encoder/api.rs:1244-1398
 *   zw_encode_frame_lossless  encode_frame_lossless  src/encoder/api.rs:945-1173
 *   zw_encode_alpha         encode_alpha_lossless     src/encoder/api.rs:1175-1222
 *   zw_encode_batch         many independent encode_frame_lossy calls (new: batch)
 *   zw_vp8_decode_frame     Vp8Decoder::decode_frame  src/decoder/vp8.rs:1526
 *   zw_vp8_decode_rgb       decode_frame + Frame::fill_rgb/fill_rgba  src/decoder/vp8.rs:200-258
 *   zw_webp_parse           WebPDecoder::new (read_data)  src/decoder/api.rs:334-510
 *   zw_webp_decode          decode_rgb / decode_rgba   src/decoder/api.rs:938-993
 *   zw_webp_decode_into     decode_rgb_into / decode_rgba_into  src/decoder/api.rs:1004-1128
 *   zw_yuv_to_rgb           fill_rgb_buffer_fancy/_simple  src/decoder/yuv.rs:82 / :402
 *   zw_rgb_to_yuv420        convert_image_yuv/_y      src/decoder/yuv.rs:656 / :806
 *   zw_loop_filter_frame    filter_row_in_cache       src/decoder/vp8.rs:1172-1345
 *
 * Conventions: plain pointers + sizes, no ownership transfer except zw_bytes /
 * zw_frame buffers (free with zw_bytes_free / zw_frame_free).  A zw_ctx owns one
 * HIP device's streams and device buffers; it is not thread-safe (one ctx per
 * host thread), matching the reference's single-threaded encoder/decoder.
 * Every compute entry point runs on the GPU; there is no CPU fallback: without
 * a usable device zw_ctx_create fails with ZW_EDEVICE.
 */
#ifndef ZWEBP_H
#define ZWEBP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes.  Encoder: EncodingError (api.rs:35-48) plus the reference's panics
 * (quality > 100 vp8.rs:2401, data length mismatch vp8.rs:1307).  Decoder:
 * DecodingError variants used by the VP8 path (decoder/api.rs:79-110). */
enum {
    ZW_OK = 0,
    ZW_EINVALID_DIMENSIONS = 1,
    ZW_EINVALID_BUFFER_SIZE = 2,
    ZW_EINVAL = 3,
    ZW_EDEVICE = 4,
    ZW_EUNSUPPORTED = 5,
    ZW_ENOMEM = 6,
    ZW_EVP8_MAGIC = 10,
    ZW_ECOLORSPACE = 11,
    ZW_ELUMA_MODE = 12,
    ZW_EINTRA_MODE = 13,
    ZW_ECHROMA_MODE = 14,
    ZW_EBITSTREAM = 15,
    ZW_EUNSUPPORTED_FEATURE = 16,
    ZW_ENOT_ENOUGH_INIT_DATA = 17,
    /* container (WebPDecoder::new / read_image, decoder/api.rs:334-700) */
    ZW_ECHUNK_HEADER = 18,       /* ChunkHeaderInvalid */
    ZW_EWEBP_SIGNATURE = 19,     /* WebpSignatureInvalid */
    ZW_ECHUNK_MISSING = 20,      /* ChunkMissing */
    ZW_EINCONSISTENT_SIZES = 21, /* InconsistentImageSizes */
    ZW_EIMAGE_TOO_LARGE = 22     /* ImageTooLarge */
};

/* UpsamplingMethod (decoder/api.rs:268-279), same order; Bilinear is the default. */
enum { ZW_UPSAMPLE_BILINEAR = 0, ZW_UPSAMPLE_SIMPLE = 1 };

/* ColorType (api.rs:83-92), same order. */
enum { ZW_COLOR_L8 = 0, ZW_COLOR_LA8 = 1, ZW_COLOR_RGB8 = 2, ZW_COLOR_RGBA8 = 3 };

typedef struct zw_ctx zw_ctx;

typedef struct {
    uint8_t *data;
    size_t len;
} zw_bytes;

/* Decoded VP8 frame (decoder/vp8.rs Frame :153-183): MB-aligned planes. */
typedef struct {
    uint16_t width, height;
    uint32_t y_stride, uv_stride; /* mbw*16, mbw*8 */
    uint32_t mb_rows;             /* planes hold mb_rows*16 (Y) / *8 (U,V) rows */
    uint8_t *y, *u, *v;
    uint8_t filter_type, filter_level, sharpness_level, pad;
} zw_frame;

/* What WebPDecoder::new learns from the container (decoder/api.rs:334-510). */
typedef struct {
    uint32_t width, height; /* canvas */
    int has_alpha, is_lossy, is_lossless, is_animated;
    uint64_t vp8_offset, vp8_len; /* the "VP8 " chunk payload inside the file */
} zw_webp_info;

typedef struct {
    const uint8_t *data; /* host pointer, w*h*bpp bytes */
    size_t len;
    uint32_t width, height;
    int color;
} zw_image;

int zw_ctx_create(int device, zw_ctx **out);
/* The last zw_ctx_destroy of the process also frees the decoded-frame buffers
 * zw_frame_free / zw_bytes_free handed back to the reuse pool (which keeps up to
 * ZW_DEC_POOL_MB, default 4096, MB of them while any context is alive). */
void zw_ctx_destroy(zw_ctx *ctx);
/* Frees the context's grow-only device scratch and pinned host staging (the
 * single-call and batch decode / filter entry points keep them between calls);
 * the next call reallocates what it needs. */
void zw_ctx_release_buffers(zw_ctx *ctx);
const char *zw_strerror(int code);
void zw_bytes_free(zw_bytes *b);
void zw_frame_free(zw_frame *f);

/* EncoderParams (encoder/api.rs:415-458).  Default: lossless, quality 95,
 * method 4, predictor transform on. */
typedef struct {
    int use_lossy;
    uint8_t lossy_quality, method;
    int use_predictor_transform;
} zw_encoder_params;

/* WebPEncoder metadata (set_icc_profile / set_exif_metadata / set_xmp_metadata,
 * encoder/api.rs:1262-1287); empty = absent. */
typedef struct {
    const uint8_t *icc;
    size_t icc_len;
    const uint8_t *exif;
    size_t exif_len;
    const uint8_t *xmp;
    size_t xmp_len;
} zw_metadata;

/* encode_frame_lossy: raw VP8 frame bytes ("VP8 " chunk payload).  Thread-safe;
 * concurrent calls on one device (any contexts) are batched: while at most
 * ZW_SEAM_SOLO (default 16) calls are in flight each encodes on its own (its
 * context's cached one-frame pipeline); calls beyond that queue, and up to two
 * of them at a time encode the queue's frames of their shape (size, colour,
 * quality, method, partitions) as one batch of up to 64 (a power of two) and
 * hand every caller its own bitstream -- byte-identical to a call of its own.
 * The batches run on internal contexts that the last zw_ctx_destroy frees
 * (zw_ctx_release_buffers frees their idle pipelines).  ZW_SEAM=0: no batching. */
int zw_encode_frame_lossy(zw_ctx *ctx, const uint8_t *data, size_t len, uint32_t width, uint32_t height,
                          int color, uint8_t quality, uint8_t method, zw_bytes *out);

/* The same with token_partitions (1, 2, 4 or 8) residual partitions: MB row y's
 * tokens go to partition y % n (the row-to-partition map of the reference
 * encoder, vp8.rs:352-354 / :1419-1421, which fixes one partition, vp8.rs:273).
 * The partition-size LAYOUT deliberately follows RFC 6386 9.5 and the reference
 * DECODER (decoder/vp8.rs:421-450): all n-1 sizes right after the first
 * partition, then the partitions.  It does NOT follow the reference encoder's
 * write_partitions (vp8.rs:381-386), which would put each size directly before
 * its partition; that writer is unreachable there (one partition) and its
 * layout is not one decoders read.  Byte parity for n > 1 is therefore not
 * pinned by any reference fixture; the checks are the oracle's identical
 * bytes plus libwebp / device decodes to the same pixels.  1 gives
 * encode_frame_lossy's bytes.  A single frame's partitions are entropy-coded
 * on parallel host threads.  ZW_EINVAL for any other count. */
int zw_encode_frame_lossy_ex(zw_ctx *ctx, const uint8_t *data, size_t len, uint32_t width, uint32_t height,
                             int color, uint8_t quality, uint8_t method, int token_partitions, zw_bytes *out);

/* WebPEncoder::encode with EncoderParams::lossy(quality, method): RIFF container
 * ("VP8 " simple form; VP8X + ALPH + "VP8 " for LA8 / RGBA8 inputs). */
int zw_encode_webp(zw_ctx *ctx, const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color,
                   uint8_t quality, uint8_t method, zw_bytes *out);
/* WebPEncoder::encode with any EncoderParams and metadata (params / meta may be
 * NULL: defaults / none).  Lossless encodes need no device (ctx may be NULL). */
int zw_encode_webp_ex(zw_ctx *ctx, const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color,
                      const zw_encoder_params *params, const zw_metadata *meta, zw_bytes *out);
/* encode_frame_lossless (VP8L bitstream incl. its 5-byte header, the "VP8L"
 * chunk payload).  Host entropy coder (like the VP8 bool coder): no device. */
int zw_encode_frame_lossless(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color,
                             int use_predictor_transform, zw_bytes *out);
/* encode_alpha_lossless: the ALPH chunk payload of an LA8 / RGBA8 image.  Host. */
int zw_encode_alpha(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, zw_bytes *out);

/* n independent frames of identical size/color; outs[i] receives frame i. */
int zw_encode_batch(zw_ctx *ctx, int n, const zw_image *imgs, uint8_t quality, uint8_t method, zw_bytes *outs);
/* ... with token_partitions (1, 2, 4, 8) per frame, as zw_encode_frame_lossy_ex. */
int zw_encode_batch_ex(zw_ctx *ctx, int n, const zw_image *imgs, uint8_t quality, uint8_t method,
                       int token_partitions, zw_bytes *outs);
/* n independent WebPEncoder::encode calls with EncoderParams::lossy(quality,
 * method) (api.rs:1291-1398; new: batch): outs[i] is frame i's RIFF container,
 * with VP8X + ALPH for LA8 / RGBA8.  The ALPH chunks are encoded on the host
 * threads that emit the VP8 tokens, while the device runs later frames. */
int zw_encode_webp_batch(zw_ctx *ctx, int n, const zw_image *imgs, uint8_t quality, uint8_t method, zw_bytes *outs);

/* Vp8Decoder::decode_frame */
int zw_vp8_decode_frame(zw_ctx *ctx, const uint8_t *vp8, size_t len, zw_frame *out);
/* n independent decode_frame calls (new: batch).  Frames may differ in size:
 * each run of consecutive frames of one size decodes as a batch of its own, in
 * order; the first failing frame's error is returned (no outputs are kept). */
int zw_vp8_decode_batch(zw_ctx *ctx, int n, const uint8_t *const *data, const size_t *lens, zw_frame *outs);
/* decode_frame + Frame::fill_rgb (bpp 3) / fill_rgba (bpp 4, alpha 255 as
 * decode_rgba) (decoder/vp8.rs:200-258, yuv.rs:82 / :402) on the device: the
 * packed w*h*bpp image is returned in out (free with zw_bytes_free).
 * upsampling: ZW_UPSAMPLE_BILINEAR (fancy) or ZW_UPSAMPLE_SIMPLE. */
int zw_vp8_decode_rgb(zw_ctx *ctx, const uint8_t *vp8, size_t len, int bpp, int upsampling, zw_bytes *out,
                      uint32_t *width, uint32_t *height);
/* n frames (new: batch; runs of one size as zw_vp8_decode_batch); widths /
 * heights may be NULL. */
int zw_vp8_decode_rgb_batch(zw_ctx *ctx, int n, const uint8_t *const *data, const size_t *lens, int bpp,
                            int upsampling, zw_bytes *outs, uint32_t *widths, uint32_t *heights);
/* The same into the caller's buffers (decode_rgba_into / decode_rgb_into,
 * decoder/api.rs:1004-1128, batched): outs[i] holds out_lens[i] >= stride_bytes
 * * height bytes, rows stride_bytes >= width * bpp apart; ZW_EINVAL otherwise
 * (the reference's InvalidParameter). */
int zw_vp8_decode_rgb_batch_into(zw_ctx *ctx, int n, const uint8_t *const *data, const size_t *lens, int bpp,
                                 int upsampling, uint8_t *const *outs, const size_t *out_lens, uint32_t stride_bytes,
                                 uint32_t *widths, uint32_t *heights);
/* WebPDecoder::new (container parse, no decoding; lossy subset: ALPH, VP8L and
 * animation return ZW_EUNSUPPORTED with info filled as far as parsed). */
int zw_webp_parse(const uint8_t *data, size_t len, zw_webp_info *info);
/* decode_rgb (bpp 3) / decode_rgba (bpp 4) (decoder/api.rs:938-993) of a lossy
 * WebP file; WebPDecoder::set_lossy_upsampling via `upsampling`. */
int zw_webp_decode(zw_ctx *ctx, const uint8_t *data, size_t len, int bpp, int upsampling, zw_bytes *out,
                   uint32_t *width, uint32_t *height);
/* decode_rgba_into (bpp 4) / decode_rgb_into (bpp 3) (decoder/api.rs:1004-1128)
 * of a lossy WebP file into out (out_len >= stride_bytes * height bytes). */
int zw_webp_decode_into(zw_ctx *ctx, const uint8_t *data, size_t len, int bpp, int upsampling, uint8_t *out,
                        size_t out_len, uint32_t stride_bytes, uint32_t *width, uint32_t *height);
/* Device time (HIP events on the context stream) of the last decode batch:
 * ms[0] = k_dec_recon (dequant + iWHT/iDCT + prediction), ms[1] = k_loopfilter. */
int zw_decode_kernel_times(zw_ctx *ctx, float *ms);
/* Host stages of the last decode batch on ctx, wall ms summed over its chunks
 * (chunks overlap: parse of chunk c runs beside the download of chunk c-1):
 * ms[0] header/mode/token parse (bool decoder, all host threads), ms[1] planes
 * or images device->host, ms[2] download + fan-out into the output buffers
 * (a chunk's download runs in parts, each fanned out while the next lands). */
int zw_decode_stage_times(zw_ctx *ctx, float *ms);
/* Device time of the last decode batch's token parse (k_dec_tok1 + k_dec_tok2:
 * one frame per lane, then one MB per lane; 0 when the host parsed every
 * frame's tokens).  The device parses the
 * token partitions (read_coefficients, decoder/vp8.rs:872-1058) of a batch's
 * later frames while the host parses the earlier chunks; headers and modes stay
 * on the host.  ZW_DEC_TOKENS=host|device|mixed forces the host, the device or a
 * split (ZW_DEC_TOKENS_HOST = the host's share); frames with several token
 * partitions always parse on the host. */
int zw_decode_token_ms(zw_ctx *ctx, float *ms);
/* The same by stage (ms): ms[0] stage 1 (k_dec_tok1: each frame's decision
 * chain on one lane, a snapshot per MB), ms[1] the count pass (k_dec_tok2 over
 * every MB from its snapshot) + record offsets + the host's wait for the total,
 * ms[2] the record pass (k_dec_tok2 writing the packed records). */
int zw_decode_token_stages(zw_ctx *ctx, float *ms);
/* Test hook, host only (no device work): steps the device token parse's
 * state machines (k_dec_tok1's decision chain, then k_dec_tok2's per-MB replay
 * from each MB's snapshot) over one VP8 frame on the CPU and compares the
 * packed MB records with the host parser's.  Returns the host parse's code;
 * *match = 1 (records equal, or both failed), 0 (they differ), -1 (a frame the
 * device parse never takes: several partitions, one MB column, or a header /
 * mode error). */
int zw_dbg_tokl_frame(const uint8_t *vp8, size_t len, int *match);
/* Test hook: the encode seam's process-wide counters -- out[0] batches led,
 * out[1] frames in them, out[2] the largest batch; reset != 0 clears them. */
int zw_dbg_seam_stats(uint64_t *out, int reset);
/* ... and of its k_yuv2rgb launch (0 when the batch returned planes). */
int zw_decode_rgb_kernel_ms(zw_ctx *ctx, float *ms);

/* Kernel-level entry points (host buffers in/out) for parity testing. */
int zw_rgb_to_yuv420(zw_ctx *ctx, const uint8_t *img, uint32_t width, uint32_t height, int bpp, uint8_t *y,
                     uint8_t *u, uint8_t *v);
/* fill_rgb_buffer_fancy (upsampling 0) / fill_rgb_buffer_simple (1) of one
 * image's planes (rows of y_stride / uv_stride bytes, ceil(h/2) chroma rows)
 * into out: w*h*bpp bytes, packed; bpp 4 writes alpha 255. */
int zw_yuv_to_rgb(zw_ctx *ctx, const uint8_t *y, const uint8_t *u, const uint8_t *v, uint32_t width,
                  uint32_t height, uint32_t y_stride, uint32_t uv_stride, int bpp, int upsampling, uint8_t *out);
/* Quantisation of n 4x4 coefficient blocks (natural order in, zigzag levels and
 * natural-order dequantised values out): VP8Matrix::quantize_coeff
 * (encoder/cost.rs:457) or trellis_quantize_block (cost.rs:788-1006) with level
 * costs from `probs` (NULL = default COEFF_PROBS).  ctype: 0 I16-AC, 1 Y2,
 * 2 UV, 3 I4; matrix_type 0 Y1 (sharpened), 1 Y2, 2 UV; ctx0[i] in 0..2. */
int zw_quant_blocks(zw_ctx *ctx, int n, const int32_t *coeffs, const uint8_t *ctx0, int ctype, int first,
                    int use_trellis, uint32_t lambda, int q_dc, int q_ac, int matrix_type, const uint8_t *probs,
                    int32_t *levels, int32_t *dequant);
/* Streaming DCT+quant pass ("transform + quant + recon" of transform_luma_block
 * / transform_chroma_blocks, encoder/vp8.rs:2647-2780 and :3039-3121, with the
 * prediction materialised): for n 4x4 blocks, block-major u8 source and
 * prediction (16 B each, raster order in the block) ->
 *   levels[n][16] int16, zigzag: quantize_coeff(dct4x4(src - pred)) (cost.rs:457;
 *                 positions < first are 0, first = 1 for I16 AC blocks)
 *   recon[n][16]  u8: clamp(pred + idct4x4(dequantised levels)).
 * matrix_type 0 Y1, 1 Y2, 2 UV selects the rounding biases (cost.rs:402-406). */
int zw_transform_quant_blocks(zw_ctx *ctx, size_t n, const uint8_t *src, const uint8_t *pred, int q_dc, int q_ac,
                              int matrix_type, int first, int16_t *levels, uint8_t *recon);
/* Same on device pointers, enqueued on `stream` (a hipStream_t; NULL = the
 * context's stream), asynchronous. */
int zw_transform_quant_blocks_device(zw_ctx *ctx, void *stream, size_t n, const void *d_src, const void *d_pred,
                                     int q_dc, int q_ac, int matrix_type, int first, void *d_levels, void *d_recon);
/* Streaming DCT+quant pass over per-MB records (SURVEY 8(d)'s HBM-roofline
 * pass): the encoder's final transform with the trellis off, per MB,
 *   luma I16  transform_luma_block      (encoder/vp8.rs:2647-2780): prediction,
 *             dct4x4 x16, wht4x4 -> Y2 quantize/dequantize -> iwht4x4, Y1 AC
 *             quantize_coeff/dequantize, idct4x4, add_residue;
 *   luma I4   transform_luma_blocks_4x4 (:2785-2916), sub-blocks in order;
 *   chroma    transform_chroma_blocks   (:3039-3121) with
 *             apply_chroma_error_diffusion (:572-647).
 * Each MB is independent: the borders create_border_luma/chroma would build
 * (common/prediction.rs:15-130) and the incoming error-diffusion terms come
 * from its 96-byte record, raster order per frame:
 *   [0] luma mode (0 DC, 1 V, 2 H, 3 TM, 4 B)   [1] chroma mode (0..3)
 *   [2] segment (0..3)   [3] bit 0: MB row > 0, bit 1: MB column > 0 (the
 *       DC predictors' edge availability, prediction.rs:182-211)
 *   [4..11] I4 sub-modes, 4 bits each (sub-block i: byte 4 + i/2, low nibble for even i)
 *   [12..15] U error diffusion in: top[0], top[1], left[0], left[1] (int8)
 *   [16..19] the same for V
 *   [20] luma corner  [21] U corner  [22] V corner  [23] 0
 *   [24..43] luma top 16 + top-right 4   [44..59] luma left 16   [60..63] 0
 *   [64..71] U top 8   [72..79] U left 8   [80..87] V top 8   [88..95] V left 8
 * Planes y/u/v and ry/ru/rv are MB-padded (stride mbw*16 / mbw*8), frame-major.
 * levels: [nframes*mbw*mbh][25][16] int16, zigzag, blocks 0..15 Y, 16 Y2 (zero
 * for I4 MBs), 17..20 U, 21..24 V (the ZwMbOut order).  seg_qi: [nframes][4]
 * quantizer index (0..127) of each segment (Segment::init_matrices,
 * types.rs:806). */
#define ZW_XMB_RECORD_BYTES 96
int zw_transform_quant_mbs(zw_ctx *ctx, int nframes, uint32_t mbw, uint32_t mbh, const uint8_t *y, const uint8_t *u,
                           const uint8_t *v, const uint8_t *recs, const int32_t *seg_qi, int16_t *levels, uint8_t *ry,
                           uint8_t *ru, uint8_t *rv);
/* Device form: the quantiser table of nframes frames (zw_xmb_seg_table, host
 * memory of zw_xmb_seg_table_bytes(nframes) bytes, copied by the caller to the
 * device as d_segs), device pointers, enqueued on `stream` (NULL = the
 * context's stream), asynchronous. */
size_t zw_xmb_seg_table_bytes(int nframes);
int zw_xmb_seg_table(int nframes, const int32_t *seg_qi, void *out);
int zw_transform_quant_mbs_device(zw_ctx *ctx, void *stream, int nframes, uint32_t mbw, uint32_t mbh, const void *d_y,
                                  const void *d_u, const void *d_v, const void *d_recs, const void *d_segs,
                                  void *d_levels, void *d_ry, void *d_ru, void *d_rv);
/* The same pass fused with the colour conversion it follows in the encoder
 * (convert_image_yuv::<3/4>, encoder/yuv.rs:656-804, with the MB padding of
 * :765-803): nframes frames of RGB (bpp 3) or RGBA (bpp 4) pixels, width x
 * height, frame after frame (the device form: frame f at d_img + f *
 * img_stride).  Outputs equal zw_transform_quant_mbs on the planes
 * zw_rgb_to_yuv420 makes of the same frames; the planes themselves are never
 * written (BASELINE config 2: RGBA in, DCT/quant/IDCT, reconstructed YUV out). */
int zw_transform_quant_mbs_rgb(zw_ctx *ctx, int nframes, uint32_t width, uint32_t height, int bpp, const uint8_t *img,
                               const uint8_t *recs, const int32_t *seg_qi, int16_t *levels, uint8_t *ry, uint8_t *ru,
                               uint8_t *rv);
int zw_transform_quant_mbs_rgb_device(zw_ctx *ctx, void *stream, int nframes, uint32_t width, uint32_t height, int bpp,
                                      const void *d_img, size_t img_stride, const void *d_recs, const void *d_segs,
                                      void *d_levels, void *d_ry, void *d_ru, void *d_rv);
/* In-place loop filter of MB-aligned planes; per-MB flags (luma_mode 0..4,
 * segment, skip, non_zero_dct) as 4 bytes per MB, raster order. */
int zw_loop_filter_frame(zw_ctx *ctx, uint8_t *y, uint8_t *u, uint8_t *v, uint32_t mbw, uint32_t mbh,
                         const uint8_t *mb_flags, int filter_type, int filter_level, int sharpness,
                         int segments_enabled, int seg_delta_values, const int8_t seg_lf_level[4],
                         int lf_adj_enabled, int ref_delta0, int mode_delta0);

/* ---- Device-resident batch pipeline (benchmarks, multi-frame serving) ----
 * A pipeline owns HBM buffers for n frames of one size.  Inputs may be written
 * directly to the device RGBA buffer (zw_pipe_input_device_ptr, e.g. from a
 * PyTorch tensor) so that timing excludes PCIe. */
typedef struct zw_pipe zw_pipe;
int zw_pipe_create(zw_ctx *ctx, int nframes, uint32_t width, uint32_t height, int color, uint8_t quality,
                   uint8_t method, zw_pipe **out);
void zw_pipe_destroy(zw_pipe *p);
void *zw_pipe_input_device_ptr(zw_pipe *p);
int zw_pipe_upload(zw_pipe *p, int frame, const uint8_t *data, size_t len);
/* Container output: zw_pipe_output then returns WebPEncoder::encode's RIFF
 * container (EncoderParams::lossy) instead of the bare VP8 frame.  For LA8 /
 * RGBA8 the ALPH chunk is encoded from host_frames[i] (width*height*bpp bytes,
 * valid while the pipe encodes); host_frames may be NULL for L8 / RGB8.
 * enable = 0 switches back to bare frames. */
int zw_pipe_set_container(zw_pipe *p, int enable, const uint8_t *const *host_frames);
/* Token partitions (1, 2, 4, 8) of every frame the pipe emits (default 1);
 * see zw_encode_frame_lossy_ex.  ZW_EINVAL for any other count. */
int zw_pipe_set_token_partitions(zw_pipe *p, int nparts);
/* Runs the full encode of all frames; bitstreams retrievable afterwards. */
int zw_pipe_encode(zw_pipe *p);
/* Encodes the uploaded batch n times back to back, streaming-style: batch k+1's
 * pass-1 kernels are queued before batch k's host token emission, so the GPU
 * and the host entropy stage overlap across batches.  Outputs afterwards are
 * those of the last batch (identical to zw_pipe_encode's). */
int zw_pipe_encode_repeat(zw_pipe *p, int n);
/* PCIe-inclusive streaming encode of nb batches from host memory: frames[b*n + i]
 * (img bytes each, any host memory) is frame i of batch b.  Each lane's uploader
 * thread copies batch b+1 into a second device input buffer while batch b's
 * passes run, so the host->device copies overlap the kernels.  The outputs
 * (zw_pipe_output) are the last batch's.  Not with container output (ZW_EINVAL).
 * Replaces the caller-side loop WebPEncoder::encode(&[u8]) per frame
 * (encoder/api.rs:1291) for a stream of host frames.  RGBA frames cross
 * PCIe as RGB: the uploader drops the alpha bytes (which the VP8 payload
 * does not read) while staging each frame in pinned memory.  With
 * ZW_UPLOAD_PACK=0 they cross as RGBA, and page-locked frames (hipHostMalloc
 * / hipHostRegister) are then read by the DMA engines directly.
 * After ZW_EDEVICE (a copy that did not complete in time) a DMA engine may
 * still read the caller's frames: keep them allocated for the process's
 * lifetime, and destroy the context (its device buffers are then leaked, not
 * reused). */
int zw_pipe_encode_host(zw_pipe *p, int nb, const uint8_t *const *frames);
/* Device-only passes (rgb2yuv, analysis, segments, pass 1, stats, pass 2) without
 * token emission, for kernel timing.  Returns 0 or an error. */
int zw_pipe_run_device(zw_pipe *p);
int zw_pipe_output(zw_pipe *p, int frame, zw_bytes *out);
/* Debug/parity taps (host copies).  zw_pipe_run_pass1 runs only the analysis
 * and pass-1 kernels, optionally writing the pass-1 reconstruction into the
 * recon planes (read with which=1). */
int zw_pipe_run_pass1(zw_pipe *p, int write_recon);
int zw_pipe_read_planes(zw_pipe *p, int frame, int which /*0 src,1 recon*/, uint8_t *y, uint8_t *u, uint8_t *v);
int zw_pipe_read_mbinfo(zw_pipe *p, int frame, int pass, uint8_t *modes /*nmb*20*/, int16_t *levels /*nmb*400*/);
int zw_pipe_read_alpha(zw_pipe *p, int frame, uint8_t *alpha);
/* Pass-2 I4 dump for parity debugging: per MB 16 sub-blocks x 34 int32
 * (fDCT coefficients[16], prediction[16], ctx0, sub-mode).  Enable before encoding. */
int zw_pipe_enable_debug(zw_pipe *p);
int zw_pipe_read_debug(zw_pipe *p, int frame, int32_t *out);
/* Quantizer index of each of the frame's 4 segments in the last encode
 * (Segment::quant_index, types.rs:761). */
int zw_pipe_read_segments(zw_pipe *p, int frame, int32_t *seg_qi);
/* Token probabilities (4*8*3*11) and skip probability used by pass 2. */
int zw_pipe_read_probs(zw_pipe *p, int frame, uint8_t *probs, int *skip_prob);
/* The pipe splits its frames into lanes (env ZW_PIPE_LANES; default 2 from two launches of frames up, else 1), each with
 * a kernel stream and a copy stream, and each lane into chunks (env
 * ZW_PIPE_CHUNK, default one frame per CU per launch): the host entropy work on
 * one chunk overlaps the kernels of the next.  Chunks of at most 12 MB rows per CU
 * run the row-parallel encode kernels (one wave per MB row; env ZW_ENC_ROWS=0/1
 * forces either shape).  zw_pipe_kernel_times: ms[0..3] = mean per-launch device time of
 * rgb2yuv, analysis+segments, pass 1, pass 2 (each launch covers one lane's
 * frames); ms[4..7] = host ms of fetch1, stats, fetch2, emit (wall, max over lanes);
 * ms[8] = the emission workers' thread CPU ms per batch, summed over lanes (n >= 9). */
int zw_pipe_lanes(zw_pipe *p);
/* frames covered by one encode-kernel launch (a lane's chunk) */
int zw_pipe_launch_frames(zw_pipe *p);
int zw_pipe_kernel_times(zw_pipe *p, float *ms, int n);
/* Host worker threads the library uses per process for entropy coding and
 * decode parsing: ZW_HOST_THREADS, else the process's affinity mask divided by
 * LOCAL_WORLD_SIZE, capped by OMP_NUM_THREADS when set. */
int zw_host_threads(void);

#ifdef __cplusplus
}
#endif
#endif
