// zw_common.h -- layouts shared by the HIP kernels (zw_kernels.hip) and the host
// runtime (zw_host.cpp).  Plain POD structs, no HIP types.
//
// HBM layout of one frame batch (all frames the same size):
//   rgba    : [nframes][h][w][bpp]                   input, uint8
//   Y       : [nframes][mbh*16][mbw*16]              MB-padded luma
//   U, V    : [nframes][mbh*8][mbw*8]                MB-padded chroma
//   alpha   : [nframes][mbh*mbw]                     analysis susceptibility
//   params  : [nframes] ZwFrameParams                segments, probs, method
//   lcost   : [nframes] ZwLevelCosts                 pass-2 token cost tables
//   mbout   : [nframes][mbh*mbw] ZwMbOut             modes, skip, zigzag levels
//   recon   : Y/U/V-shaped reconstruction (pass 2)   for parity checks
#pragma once
#include <stdint.h>

#define ZW_MAX_W 16383
#define ZW_BPS 32  // prediction work-buffer stride (prediction.rs:10 LUMA_STRIDE)

// One quantizer matrix (VP8Matrix, encoder/cost.rs:401): positions 1..15 share
// the AC values, so only DC/AC are stored; sharpen is per position (Y1 only).
struct ZwMatrix {
    uint32_t q[2], iq[2], bias[2], zthresh[2];
};

// Segment (common/types.rs:761, init_matrices :806).
struct ZwSegment {
    ZwMatrix y1, y2, uv;
    uint16_t sharpen[16];
    uint32_t lt_i4, lt_i16, lt_uv;         // trellis lambdas
    uint32_t l_i16, l_i4, l_uv, l_mode;    // RD lambdas
    uint32_t tlambda;
    int32_t quant_index, quantizer_level;  // index and delta vs base
};

struct ZwFrameParams {
    int32_t width, height, mbw, mbh;
    int32_t method, do_trellis, seg_enabled, seg_update_map;
    int32_t base_qi, filter_level, skip_prob, pad0;
    uint8_t seg_probs[4];
    uint8_t seg_map_lut[256];              // alpha -> segment id (k-means map)
    ZwSegment seg[4];
    uint8_t probs[4][8][3][11];            // token probabilities in effect
};

// Pass-1 token statistics of one frame from k_stats (zw_stats_kernels.hip):
// ProbaStats counters [type][band][ctx][node] exactly as the reference holds
// them, and the MB counts for the skip probability.
struct ZwStatsOut {
    uint32_t s[4 * 8 * 3 * 11];
    uint32_t nonzero_mbs, total_mbs;
};

// LevelCosts (encoder/cost.rs:1452-1545) for one frame.
struct ZwLevelCosts {
    uint16_t lc[4][8][3][68];
    uint16_t eob[4][8][3];
    uint16_t init[4][8][3];
};

// Per-macroblock result of an encode pass.
// levels: zigzag-ordered quantized levels as the emission codes them:
//   blocks 0..15 Y (raster), 16 Y2 (I16 only), 17..20 U, 21..24 V.
struct ZwMbOut {
    uint8_t luma_mode;    // 0 DC 1 V 2 H 3 TM 4 B
    uint8_t chroma_mode;
    uint8_t skip;         // check_all_coeffs_zero (vp8.rs:962)
    uint8_t segment;
    uint8_t bpred[16];
    int16_t levels[25][16];
};

// Decoder-side per-MB record (host bool decoder -> device recon,
// decoder/vp8.rs:681-734 modes, :1060-1168 residual tokens).  Levels stay
// quantised; the device dequantises, runs the iWHT and picks full / DC-only
// iDCT per block from nz_mask and the DC value.
// Packed decode record (what crosses PCIe): 16-byte aligned, per MB
//   [0] luma_mode | chroma_mode << 3 | skip << 5   [1] segment   [2..3] pad
//   [4..7] nz_mask   [8..15] bpred, 4 bits each
//   [16..65] start[25] (u16): block b's levels (b = Y 0..15, U 0..3, V 0..3)
//            are entries start[b] .. start[b+1]-1 of the level array (its
//            zigzag prefix up to the last nonzero); start[24] = the total.
//            Y2's levels (I16 MBs) come first, entries 0 .. start[0]-1, in the
//            order the token partition holds them   [66..79] pad (0)
//   [80..] int16 levels, zigzag order; pad to 16 (0).
// k_dec_recon / k_dec_recon_rows read it straight from the upload (one MB
// ahead, staged in LDS); a level is start[b] + zigzag position < start[b+1].
// k_pack_scan's per-chunk counter words: [0] running offset, [1] frames done,
// [2] the chunk's total bytes (read by the host), [3] pad.  The last frame's
// workgroup publishes the total and clears [0] and [1] for the next launch.
#define ZW_PACK_CTR_WORDS 4
#define ZW_DREC_HDR 80
#define ZW_DREC_MAX (ZW_DREC_HDR + 25 * 16 * 2)  // 880 B = 55 lines

// Device token parse (k_dec_tokl, zw_dec_tokens.hip).  The host parses the
// frame header and the first partition's per-MB modes into ZW_TOK_MODE bytes
// per MB (the record header's bytes 0..15: byte 0 luma mode | chroma mode << 3
// | skip << 5, byte 1 segment, bytes 8..15 the I4 sub-modes; the rest 0); the
// device parses the token partition into the records above.  Probabilities
// per frame: tokl::PROBS (1056) bytes, [type][band][ctx][node] as parsed.
struct ZwTokFrame {
    uint64_t off;  // the token partition's byte offset in the uploaded blob (16-aligned)
    uint32_t len;  // its length (the blob holds it zero-padded to 16, plus 16 zero bytes at the end)
    uint32_t pad;
};
#define ZW_TOK_MODE 16

// Loop-filter parameters per segment x {i16, i4} (calculate_filter_parameters,
// decoder/vp8.rs:1470): level, interior limit, hev threshold.
struct ZwFilterParams {
    int32_t filter_type;   // 1 = simple
    int32_t mbw, mbh, pad;
    uint8_t level[4][2], ilimit[4][2], hev[4][2], pad2[8];
};
