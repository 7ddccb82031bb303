/* oracle/or_dec.c -- TEST INFRASTRUCTURE ONLY (see or_internal.h).
 *
 * Restatement of zenwebp 0.2.0's VP8 keyframe decoder:
 *   decoder/bit_reader.rs (VP8HeaderBitReader / PartitionReader, libwebp style)
 *   decoder/vp8.rs        (header parse :553-670, MB header :681-734, residuals
 *                          :872-1168, intra prediction :736-870, loop filter
 *                          :1172-1345 via or_loop_filter_frame)
 */
#include <stdlib.h>
#include "or_internal.h"
#include "zw_oracle.h"

/* ---- bit reader (bit_reader.rs:254-640) ---- */
typedef struct {
    const uint8_t *d;
    size_t len, pos;
    uint64_t value;
    uint32_t range; /* range - 1 */
    int bits;
    int eof;
} br_t;

static void br_load(br_t *b)
{
    size_t rem = b->len - b->pos;
    if (rem >= 7) {
        uint64_t bits = 0;
        if (rem >= 8) {
            for (int i = 0; i < 8; i++) bits = (bits << 8) | b->d[b->pos + i];
            bits >>= 8;
        } else {
            for (int i = 0; i < 7; i++) bits = (bits << 8) | b->d[b->pos + i];
        }
        b->value = bits | (b->value << 56);
        b->bits += 56;
        b->pos += 7;
    } else if (b->pos < b->len) {
        b->bits += 8;
        b->value = (uint64_t)b->d[b->pos] | (b->value << 8);
        b->pos++;
    } else if (!b->eof) {
        b->value <<= 8;
        b->bits += 8;
        b->eof = 1;
    } else {
        b->bits = 0;
    }
}
static void br_init(br_t *b, const uint8_t *d, size_t len)
{
    b->d = d; b->len = len; b->pos = 0;
    b->value = 0; b->range = 254; b->bits = -8; b->eof = 0;
    br_load(b);
}
static int br_bit(br_t *b, int prob)
{
    uint32_t range = b->range;
    if (b->bits < 0) br_load(b);
    int pos = b->bits;
    uint32_t split = (range * (uint32_t)prob) >> 8;
    uint32_t value = (uint32_t)(b->value >> pos);
    int bit = value > split;
    if (bit) {
        range -= split;
        b->value -= ((uint64_t)split + 1) << pos;
    } else {
        range = split + 1;
    }
    int lz = range ? __builtin_clz(range) : 32;
    int shift = 7 ^ (31 ^ lz);
    range <<= shift;
    b->bits -= shift;
    b->range = range - 1;
    return bit;
}
static int br_lit(br_t *b, int n)
{
    int v = 0;
    for (int i = 0; i < n; i++) v = (v << 1) | br_bit(b, 128);
    return v;
}
static int br_signed(br_t *b, int n)
{
    if (!br_bit(b, 128)) return 0;
    int m = br_lit(b, n);
    return br_bit(b, 128) ? -m : m;
}
/* read_with_tree: trees given as (tree[], probs[]) like the encoder */
static int br_tree(br_t *b, const int8_t *tree, const uint8_t *probs)
{
    int i = 0;
    for (;;) {
        int t = tree[i + br_bit(b, probs[i >> 1])];
        if (t <= 0) return -t;
        i = t;
    }
}

static const int8_t SEG_TREE[6] = {2, 4, -0, -1, -2, -3};
static const int8_t YMODE_TREE[8] = {-4, 2, 4, 6, -0, -1, -2, -3};
static const int8_t BMODE_TREE[18] = {-0, 2, -1, 4, -2, 6, 8, 12, -3, 10, -5, -6, -4, 14, -7, 16, -8, -9};
static const int8_t UVMODE_TREE[6] = {-0, 2, -1, 4, -2, -3};

typedef struct {
    int16_t ydc, yac, y2dc, y2ac, uvdc, uvac;
    int8_t quant_level, lf_level;
    int delta_values;
} dseg_t;

typedef struct {
    br_t b;
    br_t part[8];
    int nparts;
    or_frame_hdr h;
    dseg_t seg[4];
    int seg_update_map;
    uint8_t seg_probs[3];
    uint8_t probs[4][8][3][11];
    int skip_prob;
} dec_t;

static int dq_dc(int i) { return DC_QUANT[or_clamp(i, 0, 127)]; }
static int dq_ac(int i) { return AC_QUANT[or_clamp(i, 0, 127)]; }

/* read_frame_header decoder/vp8.rs:553-670 */
static int parse_header(dec_t *D, const uint8_t *data, size_t len)
{
    memset(D, 0, sizeof *D);
    if (len < 3) return OR_EBITSTREAM;
    uint32_t tag = data[0] | (data[1] << 8) | (data[2] << 16);
    if (tag & 1) return OR_EUNSUPPORTED;
    uint32_t fps = tag >> 5;
    if (len < 6) return OR_EBITSTREAM;
    if (data[3] != 0x9d || data[4] != 0x01 || data[5] != 0x2a) return OR_EMAGIC;
    if (len < 10) return OR_EBITSTREAM;
    int w = (data[6] | (data[7] << 8)) & 0x3fff, h = (data[8] | (data[9] << 8)) & 0x3fff;
    D->h.width = w;
    D->h.height = h;
    D->h.mbw = (w + 15) / 16;
    D->h.mbh = (h + 15) / 16;
    size_t off = 10;
    if (len - off < fps) return OR_EBITSTREAM;
    if (fps == 0) return OR_ENOTENOUGHDATA;
    br_t *b = &D->b;
    br_init(b, data + off, fps);
    off += fps;
    int cs = br_lit(b, 1);
    (void)br_lit(b, 1);
    if (cs != 0) return OR_ECOLORSPACE;
    D->h.segments_enabled = br_bit(b, 128);
    D->seg_probs[0] = D->seg_probs[1] = D->seg_probs[2] = 255;
    if (D->h.segments_enabled) {
        D->seg_update_map = br_bit(b, 128);
        int upd = br_bit(b, 128);
        if (upd) {
            int mode = br_bit(b, 128);
            for (int i = 0; i < 4; i++) D->seg[i].delta_values = !mode;
            for (int i = 0; i < 4; i++) D->seg[i].quant_level = (int8_t)br_signed(b, 7);
            for (int i = 0; i < 4; i++) D->seg[i].lf_level = (int8_t)br_signed(b, 6);
        }
        if (D->seg_update_map)
            for (int i = 0; i < 3; i++) D->seg_probs[i] = br_bit(b, 128) ? (uint8_t)br_lit(b, 8) : 255;
        if (b->eof) return OR_EBITSTREAM;
    }
    D->h.filter_type = br_bit(b, 128);
    D->h.filter_level = br_lit(b, 6);
    D->h.sharpness = br_lit(b, 3);
    D->h.lf_adj_enabled = br_bit(b, 128);
    if (D->h.lf_adj_enabled) {
        if (br_bit(b, 128)) {
            int rd[4], md[4];
            for (int i = 0; i < 4; i++) rd[i] = br_signed(b, 6);
            for (int i = 0; i < 4; i++) md[i] = br_signed(b, 6);
            D->h.ref_delta0 = rd[0];
            D->h.mode_delta0 = md[0];
        }
        if (b->eof) return OR_EBITSTREAM;
    }
    D->nparts = 1 << br_lit(b, 2);
    D->h.num_partitions = D->nparts;
    if (b->eof) return OR_EBITSTREAM;
    /* init_partitions :421-450 */
    size_t sz_off = off;
    if (D->nparts > 1) {
        if (len - off < (size_t)(3 * D->nparts - 3)) return OR_EBITSTREAM;
        off += 3 * D->nparts - 3;
    }
    for (int p = 0; p < D->nparts; p++) {
        size_t psz;
        if (p < D->nparts - 1) {
            const uint8_t *s = data + sz_off + 3 * p;
            psz = s[0] | (s[1] << 8) | (s[2] << 16);
            if (len - off < psz) return OR_EBITSTREAM;
        } else {
            psz = len - off;
        }
        br_init(&D->part[p], data + off, psz);
        off += psz;
    }
    /* read_quantization_indices :452-504 */
    int yac = br_lit(b, 7);
    int ydc_d = br_signed(b, 4), y2dc_d = br_signed(b, 4), y2ac_d = br_signed(b, 4);
    int uvdc_d = br_signed(b, 4), uvac_d = br_signed(b, 4);
    int n = D->h.segments_enabled ? 4 : 1;
    for (int i = 0; i < n; i++) {
        int base = D->h.segments_enabled ? (D->seg[i].delta_values ? D->seg[i].quant_level + yac : D->seg[i].quant_level) : yac;
        dseg_t *s = &D->seg[i];
        s->ydc = (int16_t)dq_dc(base + ydc_d);
        s->yac = (int16_t)dq_ac(base);
        s->y2dc = (int16_t)(dq_dc(base + y2dc_d) * 2);
        s->y2ac = (int16_t)(dq_ac(base + y2ac_d) * 155 / 100);
        s->uvdc = (int16_t)dq_dc(base + uvdc_d);
        s->uvac = (int16_t)dq_ac(base + uvac_d);
        if (s->y2ac < 8) s->y2ac = 8;
        if (s->uvdc > 132) s->uvdc = 132;
    }
    if (b->eof) return OR_EBITSTREAM;
    (void)br_lit(b, 1);
    memcpy(D->probs, COEFF_PROBS, sizeof D->probs);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++)
            for (int k = 0; k < 3; k++)
                for (int t = 0; t < 11; t++)
                    if (br_bit(b, COEFF_UPDATE_PROBS[i][j][k][t])) D->probs[i][j][k][t] = (uint8_t)br_lit(b, 8);
    if (b->eof) return OR_EBITSTREAM;
    D->skip_prob = br_lit(b, 1) ? br_lit(b, 8) : -1;
    if (b->eof) return OR_EBITSTREAM;
    D->h.seg_delta_values = D->seg[0].delta_values;
    for (int i = 0; i < 4; i++) {
        D->h.seg_lf_level[i] = D->seg[i].lf_level;
        D->h.seg_quant_level[i] = D->seg[i].quant_level;
    }
    return OR_OK;
}

int or_decode_header(const uint8_t *data, size_t len, or_frame_hdr *hdr)
{
    dec_t *D = (dec_t *)malloc(sizeof(dec_t));
    int r = parse_header(D, data, len);
    if (hdr) *hdr = D->h;
    free(D);
    return r;
}

/* read_coefficients(_to_block) :872-1058.  Returns -1 on EOF error, else nz flag. */
static int read_coeffs(br_t *r, const uint8_t P[8][3][11], int32_t *blk, int first, int ctx, int dcq, int acq)
{
    int n = first;
    const uint8_t *p = P[COEFF_BANDS[n]][ctx];
    while (n < 16) {
        if (!br_bit(r, p[0])) break;
        while (!br_bit(r, p[1])) {
            n++;
            if (n >= 16) return r->eof ? -1 : 1;
            p = P[COEFF_BANDS[n]][0];
        }
        int v, nctx;
        if (!br_bit(r, p[2])) {
            v = 1;
            nctx = 1;
        } else {
            if (!br_bit(r, p[3])) {
                if (!br_bit(r, p[4])) v = 2;
                else v = 3 + br_bit(r, p[5]);
            } else {
                if (!br_bit(r, p[6])) {
                    if (!br_bit(r, p[7])) v = 5 + br_bit(r, 159);
                    else {
                        v = 7 + 2 * br_bit(r, 165);
                        v += br_bit(r, 145);
                    }
                } else {
                    int b1 = br_bit(r, p[8]);
                    int b0 = br_bit(r, p[9 + b1]);
                    int cat = 2 * b1 + b0;
                    const uint8_t *cp = PROB_DCT_CAT[2 + cat];
                    int extra = 0;
                    for (int k = 0; k < 12 && cp[k]; k++) extra = extra + extra + br_bit(r, cp[k]);
                    v = 3 + (8 << cat) + extra;
                }
            }
            nctx = 2;
        }
        int sv = br_bit(r, 128) ? -v : v;
        int zz = ZIGZAG[n];
        blk[zz] = sv * (zz > 0 ? acq : dcq);
        n++;
        if (n < 16) p = P[COEFF_BANDS[n]][nctx];
    }
    if (r->eof) return -1;
    return n > first;
}

static void set_border_chroma(uint8_t *left, uint8_t *top, const uint8_t *ws, int mbx)
{
    left[0] = ws[8];
    for (int i = 0; i < 8; i++) left[1 + i] = ws[(i + 1) * OR_BPS + 8];
    for (int i = 0; i < 8; i++) top[mbx * 8 + i] = ws[8 * OR_BPS + 1 + i];
}

int or_decode(const uint8_t *data, size_t len, uint8_t *Y, uint8_t *U, uint8_t *V, uint8_t *uY, uint8_t *uU,
              uint8_t *uV, or_mb_info *mbinfo, or_frame_hdr *hdr_out)
{
    dec_t *D = (dec_t *)malloc(sizeof(dec_t));
    int r = parse_header(D, data, len);
    if (hdr_out) *hdr_out = D->h;
    if (r != OR_OK) { free(D); return r; }
    int mbw = D->h.mbw, mbh = D->h.mbh, ys = mbw * 16, cs = mbw * 8;
    uint8_t *top_y = (uint8_t *)malloc((size_t)ys + 64), *top_u = (uint8_t *)malloc((size_t)cs + 64);
    uint8_t *top_v = (uint8_t *)malloc((size_t)cs + 64);
    memset(top_y, 127, (size_t)ys + 64);
    memset(top_u, 127, (size_t)cs + 64);
    memset(top_v, 127, (size_t)cs + 64);
    uint8_t left_y[17], left_u[9], left_v[9];
    uint8_t (*top_cx)[9] = (uint8_t(*)[9])calloc((size_t)mbw, 9);
    uint8_t (*top_bp)[4] = (uint8_t(*)[4])calloc((size_t)mbw, 4);
    or_mb_flags *flags = (or_mb_flags *)calloc((size_t)mbw * mbh, sizeof(or_mb_flags));
    int err = OR_OK;
    for (int mby = 0; mby < mbh && err == OR_OK; mby++) {
        br_t *pr = &D->part[mby % D->nparts];
        uint8_t left_cx[9] = {0}, left_bp[4] = {0};
        memset(left_y, 129, 17);
        memset(left_u, 129, 9);
        memset(left_v, 129, 9);
        for (int mbx = 0; mbx < mbw; mbx++) {
            br_t *b = &D->b;
            int segid = 0;
            if (D->h.segments_enabled && D->seg_update_map) segid = br_tree(b, SEG_TREE, D->seg_probs);
            int skip = D->skip_prob >= 0 ? br_bit(b, D->skip_prob) : 0;
            int lm = br_tree(b, YMODE_TREE, KEYFRAME_YMODE_PROBS);
            uint8_t bp[16] = {0};
            if (lm == 4) {
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) {
                        int m = br_tree(b, BMODE_TREE, KEYFRAME_BPRED_MODE_PROBS[top_bp[mbx][x]][left_bp[y]]);
                        bp[x + y * 4] = (uint8_t)m;
                        top_bp[mbx][x] = (uint8_t)m;
                        left_bp[y] = (uint8_t)m;
                    }
            } else {
                static const int intra_of[4] = {0, 2, 3, 1};
                for (int i = 0; i < 4; i++) {
                    bp[12 + i] = (uint8_t)intra_of[lm];
                    left_bp[i] = (uint8_t)intra_of[lm];
                }
            }
            int cm = br_tree(b, UVMODE_TREE, KEYFRAME_UV_MODE_PROBS);
            memcpy(top_bp[mbx], bp + 12, 4);
            if (b->eof) { err = OR_EBITSTREAM; break; }

            int32_t cb[24 * 16];
            memset(cb, 0, sizeof cb);
            int nzdct = 0;
            const dseg_t *s = &D->seg[segid];
            if (!skip) {
                int first = 1;
                if (lm != 4) {
                    int32_t y2[16] = {0};
                    int cx = top_cx[mbx][0] + left_cx[0];
                    int nz = read_coeffs(pr, (const uint8_t(*)[3][11])D->probs[1], y2, 0, cx, s->y2dc, s->y2ac);
                    if (nz < 0) { err = OR_EBITSTREAM; break; }
                    left_cx[0] = top_cx[mbx][0] = (uint8_t)nz;
                    or_iwht(y2);
                    for (int k = 0; k < 16; k++) cb[16 * k] = y2[k];
                } else first = 0;
                int plane = lm != 4 ? 0 : 3;
                for (int y = 0; y < 4 && err == OR_OK; y++) {
                    int left = left_cx[y + 1];
                    for (int x = 0; x < 4; x++) {
                        int i = x + y * 4;
                        int cx = top_cx[mbx][x + 1] + left;
                        int nz = read_coeffs(pr, (const uint8_t(*)[3][11])D->probs[plane], cb + i * 16, first, cx, s->ydc, s->yac);
                        if (nz < 0) { err = OR_EBITSTREAM; break; }
                        if (cb[i * 16] != 0 || nz) {
                            nzdct = 1;
                            if (nz) or_idct(cb + i * 16);
                            else or_idct_dc(cb + i * 16);
                        }
                        left = nz;
                        top_cx[mbx][x + 1] = (uint8_t)nz;
                    }
                    left_cx[y + 1] = (uint8_t)left;
                }
                for (int jj = 0; jj < 2 && err == OR_OK; jj++) {
                    int j = jj ? 7 : 5;
                    for (int y = 0; y < 2 && err == OR_OK; y++) {
                        int left = left_cx[y + j];
                        for (int x = 0; x < 2; x++) {
                            int i = x + y * 2 + (j == 5 ? 16 : 20);
                            int cx = top_cx[mbx][x + j] + left;
                            int nz = read_coeffs(pr, (const uint8_t(*)[3][11])D->probs[2], cb + i * 16, 0, cx, s->uvdc, s->uvac);
                            if (nz < 0) { err = OR_EBITSTREAM; break; }
                            if (cb[i * 16] != 0 || nz) {
                                nzdct = 1;
                                if (nz) or_idct(cb + i * 16);
                                else or_idct_dc(cb + i * 16);
                            }
                            left = nz;
                            top_cx[mbx][x + j] = (uint8_t)nz;
                        }
                        left_cx[y + j] = (uint8_t)left;
                    }
                }
                if (err != OR_OK) break;
            } else {
                if (lm != 4) left_cx[0] = top_cx[mbx][0] = 0;
                for (int i = 1; i < 9; i++) left_cx[i] = top_cx[mbx][i] = 0;
            }
            /* intra_predict_luma :736-806 */
            uint8_t ws[OR_LUMA_WS];
            or_border_luma(ws, mbx, mby, mbw, top_y, left_y);
            if (lm == 4) {
                for (int sby = 0; sby < 4; sby++)
                    for (int sbx = 0; sbx < 4; sbx++) {
                        int i = sbx + sby * 4;
                        or_pred_b(ws, bp[i], sbx * 4 + 1, sby * 4 + 1, OR_BPS);
                        or_add_residue(ws, cb + i * 16, sby * 4 + 1, sbx * 4 + 1, OR_BPS);
                    }
            } else {
                switch (lm) {
                case 1: or_pred_v(ws, 16, 1, 1, OR_BPS); break;
                case 2: or_pred_h(ws, 16, 1, 1, OR_BPS); break;
                case 3: or_pred_tm(ws, 16, 1, 1, OR_BPS); break;
                default: or_pred_dc(ws, 16, OR_BPS, mby != 0, mbx != 0); break;
                }
                for (int i = 0; i < 16; i++) or_add_residue(ws, cb + i * 16, 1 + (i / 4) * 4, 1 + (i % 4) * 4, OR_BPS);
            }
            left_y[0] = ws[16];
            for (int i = 0; i < 16; i++) left_y[1 + i] = ws[(i + 1) * OR_BPS + 16];
            memcpy(top_y + mbx * 16, ws + 16 * OR_BPS + 1, 16);
            for (int y = 0; y < 16; y++) memcpy(Y + (size_t)(mby * 16 + y) * ys + mbx * 16, ws + (1 + y) * OR_BPS + 1, 16);
            /* intra_predict_chroma :809-870 */
            uint8_t uw[OR_CHROMA_WS], vw[OR_CHROMA_WS];
            or_border_chroma(uw, mbx, mby, top_u, left_u);
            or_border_chroma(vw, mbx, mby, top_v, left_v);
            switch (cm) {
            case 1: or_pred_v(uw, 8, 1, 1, OR_BPS); or_pred_v(vw, 8, 1, 1, OR_BPS); break;
            case 2: or_pred_h(uw, 8, 1, 1, OR_BPS); or_pred_h(vw, 8, 1, 1, OR_BPS); break;
            case 3: or_pred_tm(uw, 8, 1, 1, OR_BPS); or_pred_tm(vw, 8, 1, 1, OR_BPS); break;
            default:
                or_pred_dc(uw, 8, OR_BPS, mby != 0, mbx != 0);
                or_pred_dc(vw, 8, OR_BPS, mby != 0, mbx != 0);
                break;
            }
            for (int i = 0; i < 4; i++) {
                int y0 = 1 + (i / 2) * 4, x0 = 1 + (i % 2) * 4;
                or_add_residue(uw, cb + (16 + i) * 16, y0, x0, OR_BPS);
                or_add_residue(vw, cb + (20 + i) * 16, y0, x0, OR_BPS);
            }
            set_border_chroma(left_u, top_u, uw, mbx);
            set_border_chroma(left_v, top_v, vw, mbx);
            for (int y = 0; y < 8; y++) {
                memcpy(U + (size_t)(mby * 8 + y) * cs + mbx * 8, uw + (1 + y) * OR_BPS + 1, 8);
                memcpy(V + (size_t)(mby * 8 + y) * cs + mbx * 8, vw + (1 + y) * OR_BPS + 1, 8);
            }
            or_mb_flags *f = &flags[mby * mbw + mbx];
            f->luma_mode = (uint8_t)lm;
            f->segment = (uint8_t)segid;
            f->skip = (uint8_t)skip;
            f->non_zero_dct = (uint8_t)nzdct;
            if (mbinfo) {
                or_mb_info *o = &mbinfo[mby * mbw + mbx];
                o->luma_mode = (uint8_t)lm;
                memcpy(o->bpred, bp, 16);
                o->chroma_mode = (uint8_t)cm;
                o->segment = (uint8_t)segid;
                o->skip = (uint8_t)skip;
                o->non_zero_dct = (uint8_t)nzdct;
            }
        }
    }
    if (err == OR_OK) {
        if (uY) memcpy(uY, Y, (size_t)ys * mbh * 16);
        if (uU) memcpy(uU, U, (size_t)cs * mbh * 8);
        if (uV) memcpy(uV, V, (size_t)cs * mbh * 8);
        or_filter_hdr fh;
        memset(&fh, 0, sizeof fh);
        fh.filter_type = D->h.filter_type;
        fh.filter_level = D->h.filter_level;
        fh.sharpness = D->h.sharpness;
        fh.segments_enabled = D->h.segments_enabled;
        fh.seg_delta_values = D->h.seg_delta_values;
        for (int i = 0; i < 4; i++) fh.seg_lf_level[i] = D->seg[i].lf_level;
        fh.lf_adj_enabled = D->h.lf_adj_enabled;
        fh.ref_delta0 = D->h.ref_delta0;
        fh.mode_delta0 = D->h.mode_delta0;
        or_loop_filter_frame(Y, U, V, mbw, mbh, flags, &fh);
    }
    free(top_y); free(top_u); free(top_v); free(top_cx); free(top_bp); free(flags);
    free(D);
    return err;
}

/* ---- kernel-level wrappers for tests ---- */
void or_free(void *p) { free(p); }
void or_rgb_to_yuv420_c(const uint8_t *img, int w, int h, int bpp, uint8_t *y, uint8_t *u, uint8_t *v)
{
    or_rgb_to_yuv420(img, w, h, bpp, y, u, v);
}
void or_fdct_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_fdct(b + 16 * i); }
void or_fdct_sse2_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_fdct_sse2(b + 16 * i); }
void or_idct_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_idct(b + 16 * i); }
void or_idct_scalar_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_idct_scalar(b + 16 * i); }
void or_wht_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_wht(b + 16 * i); }
void or_iwht_c(int32_t *b, int n) { for (int i = 0; i < n; i++) or_iwht(b + 16 * i); }
void or_loop_filter_c(uint8_t *y, uint8_t *u, uint8_t *v, int mbw, int mbh, const or_mb_info *mbs,
                      const or_frame_hdr *h)
{
    or_mb_flags *f = (or_mb_flags *)calloc((size_t)mbw * mbh, sizeof(or_mb_flags));
    for (int i = 0; i < mbw * mbh; i++) {
        f[i].luma_mode = mbs[i].luma_mode;
        f[i].segment = mbs[i].segment;
        f[i].skip = mbs[i].skip;
        f[i].non_zero_dct = mbs[i].non_zero_dct;
    }
    or_filter_hdr fh;
    memset(&fh, 0, sizeof fh);
    fh.filter_type = h->filter_type;
    fh.filter_level = h->filter_level;
    fh.sharpness = h->sharpness;
    fh.segments_enabled = h->segments_enabled;
    fh.seg_delta_values = h->seg_delta_values;
    for (int i = 0; i < 4; i++) fh.seg_lf_level[i] = h->seg_lf_level[i];
    fh.lf_adj_enabled = h->lf_adj_enabled;
    fh.ref_delta0 = h->ref_delta0;
    fh.mode_delta0 = h->mode_delta0;
    or_loop_filter_frame(y, u, v, mbw, mbh, f, &fh);
    free(f);
}
void or_yuv_to_rgb_fancy_c(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int bpp, uint8_t *out)
{
    int mbw = (w + 15) / 16;
    or_yuv_to_rgb_fancy(y, u, v, w, h, mbw * 16, bpp, out);
    if (bpp == 4)
        for (size_t i = 0; i < (size_t)w * h; i++) out[i * 4 + 3] = 255;
}
void or_yuv_to_rgb_simple_c(const uint8_t *y, const uint8_t *u, const uint8_t *v, int w, int h, int bpp, uint8_t *out)
{
    int mbw = (w + 15) / 16;
    or_yuv_to_rgb_simple(y, u, v, w, h, mbw * 16, bpp, out);
    if (bpp == 4)
        for (size_t i = 0; i < (size_t)w * h; i++) out[i * 4 + 3] = 255;
}
size_t or_debug_struct_size(void) { return sizeof(or_enc_debug); }
/* all ten I4 predictions for a 13-pixel edge (L3,L2,L1,L0,P,A0..A7) */
void or_i4_preds_edge_c(const uint8_t e[13], uint8_t out[160])
{
    uint8_t ws[8 * OR_BPS];
    memset(ws, 0, sizeof ws);
    int x0 = 1, y0 = 1;
    ws[(y0 - 1) * OR_BPS + x0 - 1] = e[4];
    for (int i = 0; i < 8; i++) ws[(y0 - 1) * OR_BPS + x0 + i] = e[5 + i];
    for (int i = 0; i < 4; i++) ws[(y0 + i) * OR_BPS + x0 - 1] = e[3 - i];
    or_i4_preds(ws, x0, y0, OR_BPS, (uint8_t(*)[16])out);
}

/* Known-answer-test entry point for the bool decoder (bit_reader.rs /
 * arithmetic.rs tests): ops[i] > 0 reads a bool with that probability,
 * ops[i] < 0 a literal of -ops[i] bits; out[i] receives the value.  Returns the
 * reader's eof flag after the reads. */
int or_bool_read_kat(const uint8_t *data, size_t len, const int *ops, int nops, int *out)
{
    br_t b;
    br_init(&b, data, len);
    for (int i = 0; i < nops; i++) out[i] = ops[i] > 0 ? br_bit(&b, ops[i]) : br_lit(&b, -ops[i]);
    return b.eof;
}
