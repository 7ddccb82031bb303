/* oracle/or_enc.c -- TEST INFRASTRUCTURE ONLY (see or_internal.h).
 *
 * Restatement of zenwebp 0.2.0's lossy VP8 encoder:
 *   encoder/vp8.rs      (Vp8Encoder: two-pass encode, RD mode search, transforms,
 *                        error diffusion, skip detection, token emission, headers)
 *   encoder/cost.rs     (VP8Matrix, trellis, LevelCosts, residual cost, ProbaStats)
 *   encoder/analysis.rs (segment analysis, k-means, segment quant)
 *   encoder/fast_math.rs(f64 cbrt/pow used for quantizer selection)
 *   encoder/arithmetic.rs (boolean encoder)
 * Compiled with -ffp-contract=off so the f64 quantizer mapping rounds exactly
 * as the Rust code does.
 */
#include <stdlib.h>
#include <math.h>
#include "or_internal.h"
#include "zw_oracle.h"

/* ======================================================================== */
/* fast_math.rs                                                             */
/* ======================================================================== */

static double fm_round(double x) { return (double)(int64_t)(x + 0.5); } /* fast_math.rs:15 */

static double fm_cbrt(double x) /* fast_math.rs:22-42 */
{
    if (x == 0.0) return 0.0;
    uint64_t bits;
    memcpy(&bits, &x, 8);
    uint64_t ab = bits / 3 + (uint64_t)(1023ull * 2 / 3) * (1ull << 52);
    double y;
    memcpy(&y, &ab, 8);
    for (int i = 0; i < 4; i++) {
        double y2 = y * y;
        y = (2.0 * y + x / y2) / 3.0;
    }
    return y;
}

static double fm_log2(double x) /* fast_math.rs:66-90 */
{
    uint64_t bits;
    memcpy(&bits, &x, 8);
    int64_t e = (int64_t)((bits >> 52) & 0x7FF) - 1023;
    uint64_t mb = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m;
    memcpy(&m, &mb, 8);
    double y = (m - 1.0) / (m + 1.0);
    double y2 = y * y;
    const double C0 = 2.8853900817779268, C1 = 0.9617966939259756, C2 = 0.5770780163555854,
                 C3 = 0.4121985831111324, C4 = 0.3205988987531030;
    double poly = C0 + y2 * (C1 + y2 * (C2 + y2 * (C3 + y2 * C4)));
    return (double)e + y * poly;
}

static double fm_exp2(double x) /* fast_math.rs:93-120 */
{
    if (x < -1022.0) x = -1022.0;
    if (x > 1023.0) x = 1023.0;
    int64_t xi = x >= 0.0 ? (int64_t)x : (int64_t)x - 1;
    double xf = x - (double)xi;
    const double LN2 = 0.6931471805599453;
    const double C1 = LN2, C2 = LN2 * LN2 / 2.0, C3 = LN2 * LN2 * LN2 / 6.0,
                 C4 = LN2 * LN2 * LN2 * LN2 / 24.0, C5 = LN2 * LN2 * LN2 * LN2 * LN2 / 120.0;
    double poly = 1.0 + xf * (C1 + xf * (C2 + xf * (C3 + xf * (C4 + xf * C5))));
    uint64_t eb = (uint64_t)(xi + 1023) << 52;
    double scale;
    memcpy(&scale, &eb, 8);
    return poly * scale;
}

static double fm_pow(double x, double n) /* fast_math.rs:48-62 */
{
    if (x <= 0.0) return 0.0;
    if (x == 1.0 || n == 0.0) return 1.0;
    if (n == 1.0) return x;
    return fm_exp2(n * fm_log2(x));
}

/* quality_to_compression / quality_to_quant_index, encoder/vp8.rs:37-55 */
int or_quality_to_quant_index(int quality)
{
    double c = (double)quality / 100.0;
    double lin = c < 0.75 ? c * (2.0 / 3.0) : 2.0 * c - 1.0;
    double comp = fm_cbrt(lin);
    double r = fm_round(127.0 * (1.0 - comp));
    int q = (int)r;
    return or_clamp(q, 0, 127);
}

/* compute_segment_quant, analysis.rs:1145-1174 */
static int compute_segment_quant(int base, int alpha, int sns)
{
    double amp = 0.9 * (double)sns / 100.0 / 128.0;
    double expn = 1.0 - amp * (double)alpha;
    if (expn <= 0.0) return base;
    double cb = 1.0 - ((double)base / 127.0);
    double c = fm_pow(cb, expn);
    double qd = 127.0 * (1.0 - c);
    int q = (int)qd; /* 'as i32' truncation (values are in range) */
    return or_clamp(q, 0, 127);
}

/* ======================================================================== */
/* cost.rs: matrices, quantization, filter level                             */
/* ======================================================================== */

#define QFIX 17
static inline uint32_t qbias(uint32_t b) { return ((b << QFIX) + 128) >> 8; }
static inline int32_t quantdiv(uint32_t c, uint32_t iq, uint32_t bias)
{
    return (int32_t)(((uint64_t)c * iq + bias) >> QFIX);
}

typedef struct {
    uint16_t q[16];
    uint32_t iq[16], bias[16], zthresh[16];
    uint16_t sharpen[16];
} mtx_t;

/* VP8Matrix::new, cost.rs:401-446 ; type 0 = Y1, 1 = Y2, 2 = UV */
static void mtx_init(mtx_t *m, int qdc, int qac, int type)
{
    static const int bias_dc[3] = {96, 96, 110}, bias_ac[3] = {110, 108, 115};
    memset(m, 0, sizeof *m);
    m->q[0] = (uint16_t)qdc;
    m->q[1] = (uint16_t)qac;
    for (int i = 0; i < 2; i++) {
        uint32_t b = i ? bias_ac[type] : bias_dc[type];
        m->iq[i] = (uint32_t)((1ull << QFIX) / m->q[i]);
        m->bias[i] = qbias(b);
        m->zthresh[i] = ((1u << QFIX) - 1 - m->bias[i]) / m->iq[i];
    }
    for (int i = 2; i < 16; i++) {
        m->q[i] = m->q[1];
        m->iq[i] = m->iq[1];
        m->bias[i] = m->bias[1];
        m->zthresh[i] = m->zthresh[1];
    }
    if (type == 0)
        for (int i = 0; i < 16; i++) m->sharpen[i] = (uint16_t)(((uint32_t)VP8_FREQ_SHARPENING[i] * m->q[i]) >> 11);
}

/* VP8Matrix::quantize_coeff cost.rs:457 */
static inline int32_t quant(const mtx_t *m, int32_t c, int pos)
{
    int neg = c < 0;
    uint32_t a = (uint32_t)(neg ? -c : c);
    int32_t l = quantdiv(a, m->iq[pos], m->bias[pos]);
    return neg ? -l : l;
}
static inline int32_t dequant(const mtx_t *m, int32_t l, int pos) { return l * (int32_t)m->q[pos]; }

/* compute_filter_level cost.rs:271-294 */
static int compute_filter_level(int qi, int sharp, int strength)
{
    uint32_t level0 = 5u * strength;
    int qstep = (uint8_t)(VP8_AC_TABLE[qi] >> 2);
    int pos = qstep < 63 ? qstep : 63;
    uint32_t base = LEVELS_FROM_DELTA[sharp < 7 ? sharp : 7][pos];
    uint32_t f = base * level0 / 256;
    if (f < 2) return 0;
    if (f > 63) return 63;
    return (int)f;
}

/* ======================================================================== */
/* Segment (types.rs:761-854)                                                */
/* ======================================================================== */

typedef struct {
    int16_t ydc, yac, y2dc, y2ac, uvdc, uvac;
    int8_t quantizer_level;
    uint8_t quant_index;
    mtx_t y1, y2, uv;
    uint32_t lt_i4, lt_i16, lt_uv, l_i16, l_i4, l_uv, l_mode, tlambda;
} seg_t;

static uint32_t umax1(uint32_t v) { return v ? v : 1; }

/* Segment::init_matrices types.rs:806-854 */
static void seg_init(seg_t *s)
{
    mtx_init(&s->y1, (uint16_t)s->ydc, (uint16_t)s->yac, 0);
    mtx_init(&s->y2, (uint16_t)s->y2dc, (uint16_t)s->y2ac, 1);
    mtx_init(&s->uv, (uint16_t)s->uvdc, (uint16_t)s->uvac, 2);
    uint32_t qi4 = ((uint32_t)s->ydc + 15u * (uint32_t)s->yac + 8) >> 4;
    uint32_t qi16 = ((uint32_t)s->y2dc + 15u * (uint32_t)s->y2ac + 8) >> 4;
    uint32_t quv = ((uint32_t)s->uvdc + 15u * (uint32_t)s->uvac + 8) >> 4;
    s->lt_i4 = umax1((7 * qi4 * qi4) >> 3);
    s->lt_i16 = umax1((qi16 * qi16) >> 2);
    s->lt_uv = umax1((quv * quv) << 1);
    s->l_i4 = umax1((3 * qi4 * qi4) >> 7);
    s->l_i16 = umax1(3 * qi16 * qi16);
    s->l_uv = umax1((3 * quv * quv) >> 6);
    s->l_mode = umax1((qi4 * qi4) >> 7);
    s->tlambda = (50 * qi4) >> 5;
}

static void seg_from_index(seg_t *s, int qi, int delta)
{
    memset(s, 0, sizeof *s);
    s->ydc = DC_QUANT[qi];
    s->yac = AC_QUANT[qi];
    s->y2dc = (int16_t)(DC_QUANT[qi] * 2);
    int y2ac = (int)AC_QUANT[qi] * 155 / 100;
    s->y2ac = (int16_t)(y2ac < 8 ? 8 : y2ac);
    s->uvdc = DC_QUANT[qi];
    s->uvac = AC_QUANT[qi];
    s->quantizer_level = (int8_t)delta;
    s->quant_index = (uint8_t)qi;
    seg_init(s);
}

/* ======================================================================== */
/* LevelCosts / residual cost (cost.rs:1452-1980)                            */
/* ======================================================================== */

#define MAX_LEVEL 2047
#define MAX_VLEVEL 67

typedef struct {
    uint16_t lc[4][8][3][MAX_VLEVEL + 1];
    uint16_t eob[4][8][3];
    uint16_t init[4][8][3];
} lcost_t;

static inline uint16_t bitcost(int bit, uint8_t p) { return bit ? VP8_ENTROPY_COST[255 - p] : VP8_ENTROPY_COST[p]; }

/* variable_level_cost cost.rs:1422 */
static uint16_t var_level_cost(int level, const uint8_t *p)
{
    if (level == 0) return 0;
    int idx = (level < MAX_VLEVEL ? level : MAX_VLEVEL) - 1;
    int pat = VP8_LEVEL_CODES[idx][0], bits = VP8_LEVEL_CODES[idx][1];
    uint16_t cost = 0;
    for (int i = 2; pat; i++) {
        if (pat & 1) cost = (uint16_t)(cost + bitcost(bits & 1, p[i]));
        bits >>= 1;
        pat >>= 1;
    }
    return cost;
}

/* LevelCosts::calculate cost.rs:1500-1545 */
static void lcost_calc(lcost_t *L, const uint8_t probs[4][8][3][11])
{
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++) {
                const uint8_t *p = probs[t][b][c];
                uint16_t cost0 = c > 0 ? bitcost(1, p[0]) : 0;
                uint16_t base = (uint16_t)(bitcost(1, p[1]) + cost0);
                L->lc[t][b][c][0] = (uint16_t)(bitcost(0, p[1]) + cost0);
                for (int v = 1; v <= MAX_VLEVEL; v++) L->lc[t][b][c][v] = (uint16_t)(base + var_level_cost(v, p));
                L->eob[t][b][c] = bitcost(0, p[0]);
                L->init[t][b][c] = bitcost(1, p[0]);
            }
}

/* get_residual_cost (SSE2 and scalar agree) cost.rs:1670-1733 */
static uint32_t residual_cost(int ctx0, const int32_t *coeffs, int ctype, int first, const lcost_t *L,
                              const uint8_t probs[4][8][3][11])
{
    int last = -1;
    for (int i = 15; i >= 0; i--)
        if (coeffs[i] != 0) { last = i; break; }
    int n = first;
    uint8_t p0 = probs[ctype][VP8_ENC_BANDS[n]][ctx0][0];
    int ctx = ctx0;
    uint32_t cost = ctx0 == 0 ? bitcost(1, p0) : 0;
    if (last < 0) return bitcost(0, p0);
    while (n < last) {
        uint32_t v = (uint32_t)or_abs(coeffs[n]);
        cost += VP8_LEVEL_FIXED_COSTS[v < MAX_LEVEL ? v : MAX_LEVEL] +
                L->lc[ctype][VP8_ENC_BANDS[n]][ctx][v < MAX_VLEVEL ? v : MAX_VLEVEL];
        ctx = v >= 2 ? 2 : (int)v;
        n++;
    }
    {
        uint32_t v = (uint32_t)or_abs(coeffs[n]);
        cost += VP8_LEVEL_FIXED_COSTS[v < MAX_LEVEL ? v : MAX_LEVEL] +
                L->lc[ctype][VP8_ENC_BANDS[n]][ctx][v < MAX_VLEVEL ? v : MAX_VLEVEL];
        if (n < 15) {
            int nctx = v == 1 ? 1 : 2;
            cost += bitcost(0, probs[ctype][VP8_ENC_BANDS[n + 1]][nctx][0]);
        }
    }
    return cost;
}

/* ======================================================================== */
/* Trellis (cost.rs:788-1006)                                                */
/* ======================================================================== */

#define MAX_COST (INT64_MAX / 2)

static inline int64_t rd_trellis(uint32_t lambda, int64_t rate, int64_t dist) { return rate * (int64_t)lambda + 256 * dist; }

/* returns has_nz; coeffs (natural) become dequantized values, out (zigzag) levels */
static int trellis(int32_t coeffs[16], int32_t out[16], const mtx_t *m, uint32_t lambda, int first,
                   const lcost_t *L, int ctype, int ctx0)
{
    typedef struct { int8_t prev; uint8_t sign; int16_t level; } node_t;
    typedef struct { int64_t score; const uint16_t *costs; } ss_t;
    node_t nodes[16][2];
    ss_t ss[2][2];
    memset(nodes, 0, sizeof nodes);
    int cur = 0, prev = 1;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++) { ss[a][b].score = MAX_COST; ss[a][b].costs = NULL; }

    int thresh = (int)((int64_t)m->q[1] * m->q[1] / 4);
    int last = first - 1;
    for (int n = 15; n >= first; n--) {
        int j = ZIGZAG[n];
        int err = coeffs[j] * coeffs[j];
        if (err > thresh) { last = n; break; }
    }
    if (last < 15) last++;

    int best_path[3] = {-1, -1, -1};
    int64_t skip_cost = L->eob[ctype][VP8_ENC_BANDS[first]][ctx0];
    int64_t best_score = rd_trellis(lambda, skip_cost, 0);
    const uint16_t *init_costs = L->lc[ctype][VP8_ENC_BANDS[first]][ctx0];
    int64_t init_rate = ctx0 == 0 ? L->init[ctype][VP8_ENC_BANDS[first]][ctx0] : 0;
    int64_t init_score = rd_trellis(lambda, init_rate, 0);
    for (int d = 0; d < 2; d++) { ss[cur][d].score = init_score; ss[cur][d].costs = init_costs; }

    for (int n = first; n <= last; n++) {
        int j = ZIGZAG[n];
        int q = m->q[j];
        uint32_t iq = m->iq[j];
        uint32_t nb = qbias(0);
        int sign = coeffs[j] < 0;
        int abs_c = sign ? -coeffs[j] : coeffs[j];
        int cws = abs_c + m->sharpen[j];
        int level0 = quantdiv((uint32_t)cws, iq, nb);
        if (level0 > MAX_LEVEL) level0 = MAX_LEVEL;
        int thresh_level = quantdiv((uint32_t)cws, iq, qbias(0x80));
        if (thresh_level > MAX_LEVEL) thresh_level = MAX_LEVEL;
        int t = cur; cur = prev; prev = t;
        for (int d = 0; d < 2; d++) {
            int level = level0 + d;
            int ctx = level < 2 ? level : 2;
            const uint16_t *next_costs = (n + 1 < 16) ? L->lc[ctype][VP8_ENC_BANDS[n + 1]][ctx] : NULL;
            ss[cur][d].score = MAX_COST;
            ss[cur][d].costs = next_costs;
            if (level < 0 || level > thresh_level) continue;
            int new_err = cws - level * q;
            int64_t orig_sq = (int64_t)(cws * cws);
            int64_t new_sq = (int64_t)(new_err * new_err);
            int64_t w = VP8_WEIGHT_TRELLIS[j];
            int64_t dd = w * (new_sq - orig_sq);
            int64_t base = rd_trellis(lambda, 0, dd);
            int64_t sc[2];
            for (int p = 0; p < 2; p++) {
                int64_t cost;
                if (ss[prev][p].costs) {
                    int lv = level;
                    cost = (int64_t)VP8_LEVEL_FIXED_COSTS[lv] + ss[prev][p].costs[lv < MAX_VLEVEL ? lv : MAX_VLEVEL] +
                           (lv > 0 ? 256 : 0);
                } else {
                    cost = VP8_LEVEL_FIXED_COSTS[level];
                }
                sc[p] = ss[prev][p].score + cost * (int64_t)lambda;
            }
            int64_t best_cur;
            int bp;
            if (sc[1] < sc[0]) { best_cur = sc[1] + base; bp = 1; }
            else { best_cur = sc[0] + base; bp = 0; }
            nodes[n][d].sign = (uint8_t)sign;
            nodes[n][d].level = (int16_t)level;
            nodes[n][d].prev = (int8_t)bp;
            ss[cur][d].score = best_cur;
            if (level != 0 && best_cur < best_score) {
                int64_t eob = n < 15 ? L->eob[ctype][VP8_ENC_BANDS[(n + 1) < 15 ? n + 1 : 15]][ctx] : 0;
                int64_t term = best_cur + rd_trellis(lambda, eob, 0);
                if (term < best_score) {
                    best_score = term;
                    best_path[0] = n;
                    best_path[1] = d;
                    best_path[2] = bp;
                }
            }
        }
    }
    if (first == 1) {
        for (int i = 1; i < 16; i++) { out[i] = 0; coeffs[i] = 0; }
    } else {
        for (int i = 0; i < 16; i++) { out[i] = 0; coeffs[i] = 0; }
    }
    if (best_path[0] == -1) return 0;
    int has_nz = 0;
    int bd = best_path[1];
    int n = best_path[0];
    nodes[n][bd].prev = (int8_t)best_path[2];
    for (;;) {
        node_t *nd = &nodes[n][bd];
        int j = ZIGZAG[n];
        int level = nd->sign ? -nd->level : nd->level;
        out[n] = level;
        has_nz |= level != 0;
        coeffs[j] = level * (int32_t)m->q[j];
        if (n == first) break;
        bd = nd->prev;
        n--;
    }
    return has_nz;
}

/* ======================================================================== */
/* Bool encoder (encoder/arithmetic.rs)                                      */
/* ======================================================================== */

typedef struct {
    uint8_t *buf;
    size_t len, cap;
    uint32_t bottom, range;
    int bit_num;
} benc_t;

static void be_init(benc_t *e)
{
    e->buf = NULL; e->len = 0; e->cap = 0;
    e->bottom = 0; e->range = 255; e->bit_num = 24;
}
static void be_push(benc_t *e, uint8_t b)
{
    if (e->len == e->cap) {
        e->cap = e->cap ? e->cap * 2 : 1024;
        e->buf = (uint8_t *)realloc(e->buf, e->cap);
    }
    e->buf[e->len++] = b;
}
static void be_add_one(benc_t *e) /* arithmetic.rs:47-60 */
{
    size_t i = e->len;
    while (i > 0) {
        i--;
        if (e->buf[i] < 255) { e->buf[i]++; return; }
        e->buf[i] = 0;
    }
    be_push(e, 0);
    memmove(e->buf + 1, e->buf, e->len - 1);
    e->buf[0] = 1;
}
static void be_bool(benc_t *e, int bit, int prob) /* arithmetic.rs:67-95 */
{
    uint32_t split = 1 + (((e->range - 1) * (uint32_t)prob) >> 8);
    if (bit) { e->bottom += split; e->range -= split; }
    else e->range = split;
    while (e->range < 128) {
        e->range <<= 1;
        if (e->bottom & (1u << 31)) be_add_one(e);
        e->bottom <<= 1;
        e->bit_num--;
        if (e->bit_num == 0) {
            be_push(e, (uint8_t)(e->bottom >> 24));
            e->bottom &= (1u << 24) - 1;
            e->bit_num = 8;
        }
    }
}
static void be_flag(benc_t *e, int f) { be_bool(e, f, 128); }
static void be_lit(benc_t *e, int nbits, int v)
{
    for (int b = nbits - 1; b >= 0; b--) be_bool(e, ((1 << b) & v) > 0, 128);
}
/* write_with_tree_start_index arithmetic.rs:120-174 */
static void be_tree(benc_t *e, const int8_t *tree, int tlen, const uint8_t *probs, int value, int start)
{
    int cur = -1;
    for (int i = 0; i < tlen; i++)
        if (tree[i] == -value) { cur = i; break; }
    int enc[16], pr[16], cnt = 0;
    for (;;) {
        if (cur == start) { enc[cnt] = 0; pr[cnt] = probs[cur / 2]; cnt++; break; }
        if (cur == start + 1) { enc[cnt] = 1; pr[cnt] = probs[cur / 2]; cnt++; break; }
        int ev;
        if (cur % 2 == 0) ev = 0;
        else { cur -= 1; ev = 1; }
        enc[cnt] = ev; pr[cnt] = probs[cur / 2]; cnt++;
        int pi = -1;
        for (int i = 0; i < tlen; i++)
            if (tree[i] == cur) { pi = i; break; }
        cur = pi;
    }
    for (int i = cnt - 1; i >= 0; i--) be_bool(e, enc[i], pr[i]);
}
static void be_flush(benc_t *e) /* flush_and_get_buffer arithmetic.rs:176-195 */
{
    int c = e->bit_num;
    uint32_t v = e->bottom;
    if (e->bottom & (1u << (32 - e->bit_num))) be_add_one(e);
    v <<= (c & 7);
    c = (c >> 3) - 1;
    while (c >= 0) { v <<= 8; c--; }
    c = 3;
    while (c >= 0) { be_push(e, (uint8_t)(v >> 24)); v <<= 8; c--; }
}

/* Trees (types.rs:191-332, :699) */
static const int8_t SEGMENT_ID_TREE[6] = {2, 4, -0, -1, -2, -3};
static const int8_t YMODE_TREE[8] = {-4, 2, 4, 6, -0, -1, -2, -3};
static const int8_t BMODE_TREE[18] = {-0, 2, -1, 4, -2, 6, 8, 12, -3, 10, -5, -6, -4, 14, -7, 16, -8, -9};
static const int8_t UVMODE_TREE[6] = {-0, 2, -1, 4, -2, -3};
static const int8_t TOKEN_TREE[22] = {-11, 2, -0, 4, -1, 6, 8, 12, -2, 10, -3, -4, 14, 16, -5, -6, 18, 20, -7, -8, -9, -10};

/* ======================================================================== */
/* Analysis (analysis.rs)                                                    */
/* ======================================================================== */

static const int DSP_SCAN[24] = {0, 4, 8, 12, 0 + 4 * 32, 4 + 4 * 32, 8 + 4 * 32, 12 + 4 * 32,
                                 0 + 8 * 32, 4 + 8 * 32, 8 + 8 * 32, 12 + 8 * 32, 0 + 12 * 32, 4 + 12 * 32,
                                 8 + 12 * 32, 12 + 12 * 32, 0, 4, 0 + 4 * 32, 4 + 4 * 32, 8, 12,
                                 8 + 4 * 32, 12 + 4 * 32};

static int histo_alpha(const uint8_t *src, int sb, const uint8_t *pred, int pb, int b0, int b1)
{
    uint32_t dist[32] = {0};
    for (int j = b0; j < b1; j++) {
        int16_t o[16];
        or_ftransform_analysis(src + sb + DSP_SCAN[j], pred + pb + DSP_SCAN[j], 32, 32, o);
        for (int k = 0; k < 16; k++) {
            int v = or_abs(o[k]) >> 3;
            dist[v < 31 ? v : 31]++;
        }
    }
    uint32_t maxv = 0;
    int lnz = 1;
    for (int k = 0; k < 32; k++)
        if (dist[k] > 0) {
            if (dist[k] > maxv) maxv = dist[k];
            lnz = k;
        }
    return maxv > 1 ? (int)(510u * (uint32_t)lnz / maxv) : 0; /* get_alpha analysis.rs:160 */
}

static void fill_blk(uint8_t *d, int v, int size)
{
    for (int y = 0; y < size; y++) memset(d + y * 32, v, size);
}

/* analyze_image analysis.rs:964-1003 (AnalysisIterator import :622, modes :811/:861) */
void or_analyze(const uint8_t *Y, const uint8_t *U, const uint8_t *V, int width, int height,
                uint8_t *mb_alphas, uint32_t histo[256])
{
    int mbw = (width + 15) / 16, mbh = (height + 15) / 16;
    int ys = mbw * 16, cs = mbw * 8;
    uint8_t yin[32 * 16], yp[32 * 16 + 32 * 16 + 8 * 32 + 64];
    uint8_t y_left[17], u_left[9], v_left[9];
    uint8_t *y_top = (uint8_t *)malloc((size_t)mbw * 16 + 4);
    uint8_t *uv_top = (uint8_t *)malloc((size_t)mbw * 16);
    memset(y_top, 127, (size_t)mbw * 16 + 4);
    memset(uv_top, 127, (size_t)mbw * 16);
    memset(histo, 0, 256 * sizeof(uint32_t));
    memset(yp, 0, sizeof yp);
    int idx = 0;
    for (int y = 0; y < mbh; y++) {
        for (int x = 0; x < mbw; x++) {
            int yo = y * 16 * ys + x * 16, uo = y * 8 * cs + x * 8;
            int w = width - x * 16 < 16 ? width - x * 16 : 16;
            int h = height - y * 16 < 16 ? height - y * 16 : 16;
            int uw = (w + 1) / 2, uh = (h + 1) / 2;
            /* import_block */
            memset(yin, 0, sizeof yin);
            for (int r = 0; r < h; r++) {
                for (int c = 0; c < w; c++) yin[r * 32 + c] = Y[yo + r * ys + c];
                for (int c = w; c < 16; c++) yin[r * 32 + c] = yin[r * 32 + w - 1];
            }
            for (int r = h; r < 16; r++) memcpy(yin + r * 32, yin + (h - 1) * 32, 16);
            for (int pl = 0; pl < 2; pl++) {
                const uint8_t *P = pl ? V : U;
                uint8_t *d = yin + 16 + 8 * pl;
                for (int r = 0; r < uh; r++) {
                    for (int c = 0; c < uw; c++) d[r * 32 + c] = P[uo + r * cs + c];
                    for (int c = uw; c < 8; c++) d[r * 32 + c] = d[r * 32 + uw - 1];
                }
                for (int r = uh; r < 8; r++) memcpy(d + r * 32, d + (uh - 1) * 32, 8);
            }
            /* boundary samples */
            if (x == 0) {
                uint8_t corner = y > 0 ? 129 : 127;
                y_left[0] = u_left[0] = v_left[0] = corner;
                memset(y_left + 1, 129, 16);
                memset(u_left + 1, 129, 8);
                memset(v_left + 1, 129, 8);
            } else {
                if (y == 0) {
                    y_left[0] = u_left[0] = v_left[0] = 127;
                } else {
                    y_left[0] = Y[yo - 1 - ys];
                    u_left[0] = U[uo - 1 - cs];
                    v_left[0] = V[uo - 1 - cs];
                }
                for (int i = 0; i < h; i++) y_left[1 + i] = Y[yo - 1 + i * ys];
                for (int i = h; i < 16; i++) y_left[1 + i] = y_left[1 + (h > 0 ? h - 1 : 0)];
                for (int i = 0; i < uh; i++) {
                    u_left[1 + i] = U[uo - 1 + i * cs];
                    v_left[1 + i] = V[uo - 1 + i * cs];
                }
                for (int i = uh; i < 8; i++) {
                    u_left[1 + i] = u_left[1 + uh - 1];
                    v_left[1 + i] = v_left[1 + uh - 1];
                }
            }
            if (y == 0) {
                memset(y_top + x * 16, 127, 16);
                memset(uv_top + x * 16, 127, 16);
            } else {
                for (int i = 0; i < w; i++) y_top[x * 16 + i] = Y[yo - ys + i];
                for (int i = w; i < 16; i++) y_top[x * 16 + i] = y_top[x * 16 + w - 1];
                for (int i = 0; i < uw; i++) {
                    uv_top[x * 16 + i] = U[uo - cs + i];
                    uv_top[x * 16 + 8 + i] = V[uo - cs + i];
                }
                for (int i = uw; i < 8; i++) {
                    uv_top[x * 16 + i] = uv_top[x * 16 + uw - 1];
                    uv_top[x * 16 + 8 + i] = uv_top[x * 16 + 8 + uw - 1];
                }
            }
            int has_l = x > 0, has_t = y > 0;
            /* luma predictions: DC at 0, TM at 16 (make_luma16_preds :366) */
            {
                const uint8_t *top = y_top + x * 16;
                int dc;
                if (has_t && has_l) {
                    uint32_t s = 0;
                    for (int i = 0; i < 16; i++) s += top[i] + y_left[1 + i];
                    dc = (int)((s + 16) >> 5);
                } else if (has_t) {
                    uint32_t s = 0;
                    for (int i = 0; i < 16; i++) s += top[i];
                    s += s;
                    dc = (int)((s + 16) >> 5);
                } else if (has_l) {
                    uint32_t s = 0;
                    for (int i = 0; i < 16; i++) s += y_left[1 + i];
                    s += s;
                    dc = (int)((s + 16) >> 5);
                } else dc = 0x80;
                fill_blk(yp, dc, 16);
                uint8_t *tm = yp + 16;
                if (has_l && has_t) {
                    int tl = y_left[0];
                    for (int r = 0; r < 16; r++)
                        for (int c = 0; c < 16; c++) tm[r * 32 + c] = (uint8_t)or_clamp(y_left[1 + r] + top[c] - tl, 0, 255);
                } else if (has_l) {
                    for (int r = 0; r < 16; r++) memset(tm + r * 32, y_left[1 + r], 16);
                } else if (has_t) {
                    for (int r = 0; r < 16; r++) memcpy(tm + r * 32, top, 16);
                } else fill_blk(tm, 129, 16);
            }
            int best_alpha = -1;
            for (int mode = 0; mode < 2; mode++) {
                int a = histo_alpha(yin, 0, yp, mode ? 16 : 0, 0, 16);
                if (a > best_alpha) best_alpha = a;
            }
            /* chroma predictions at C8DC8 = 2*16*32, C8TM8 = +16 (make_chroma8_preds :458) */
            {
                uint8_t *base = yp + 2 * 16 * 32;
                for (int pl = 0; pl < 2; pl++) {
                    const uint8_t *left = pl ? v_left : u_left;
                    const uint8_t *top = uv_top + x * 16 + 8 * pl;
                    int dc;
                    if (has_t && has_l) {
                        uint32_t s = 0;
                        for (int i = 0; i < 8; i++) s += top[i] + left[1 + i];
                        dc = (int)((s + 8) >> 4);
                    } else if (has_t) {
                        uint32_t s = 0;
                        for (int i = 0; i < 8; i++) s += top[i];
                        s += s;
                        dc = (int)((s + 8) >> 4);
                    } else if (has_l) {
                        uint32_t s = 0;
                        for (int i = 0; i < 8; i++) s += left[1 + i];
                        s += s;
                        dc = (int)((s + 8) >> 4);
                    } else dc = 0x80;
                    fill_blk(base + 8 * pl, dc, 8);
                    uint8_t *tm = base + 16 + 8 * pl;
                    if (has_l && has_t) {
                        int tl = left[0];
                        for (int r = 0; r < 8; r++)
                            for (int c = 0; c < 8; c++) tm[r * 32 + c] = (uint8_t)or_clamp(left[1 + r] + top[c] - tl, 0, 255);
                    } else if (has_l) {
                        for (int r = 0; r < 8; r++) memset(tm + r * 32, left[1 + r], 8);
                    } else if (has_t) {
                        for (int r = 0; r < 8; r++) memcpy(tm + r * 32, top, 8);
                    } else fill_blk(tm, 129, 8);
                }
            }
            int best_uv = -1;
            for (int mode = 0; mode < 2; mode++) {
                int a = histo_alpha(yin, 16, yp, 2 * 16 * 32 + (mode ? 16 : 0), 16, 24);
                if (a > best_uv) best_uv = a;
            }
            int alpha = (3 * best_alpha + best_uv + 2) >> 2;
            alpha = or_clamp(255 - alpha, 0, 255); /* final_alpha_value :248 */
            mb_alphas[idx++] = (uint8_t)alpha;
            histo[alpha]++;
        }
    }
    free(y_top);
    free(uv_top);
}

/* assign_segments_kmeans analysis.rs:1029-1133 */
static void kmeans(const uint32_t alphas[256], uint8_t centers[4], uint8_t map[256], int *wavg)
{
    const int ns = 4;
    memset(centers, 0, 4);
    memset(map, 0, 256);
    int min_a = 0, max_a = 255;
    for (int n = 0; n < 256; n++)
        if (alphas[n] > 0) { min_a = n; break; }
    for (int n = 255; n >= min_a; n--)
        if (alphas[n] > 0) { max_a = n; break; }
    int range = max_a > min_a ? max_a - min_a : 0;
    for (int k = 0; k < ns; k++) centers[k] = (uint8_t)(min_a + ((1 + 2 * k) * range) / (2 * ns));
    uint32_t accum[4], dacc[4];
    int64_t wa = 0;
    uint32_t tw = 0;
    for (int it = 0; it < 6; it++) {
        for (int i = 0; i < ns; i++) accum[i] = dacc[i] = 0;
        int cc = 0;
        for (int a = min_a; a <= max_a; a++) {
            if (alphas[a] > 0) {
                while (cc + 1 < ns) {
                    int dcur = or_abs(a - centers[cc]), dnext = or_abs(a - centers[cc + 1]);
                    if (dnext < dcur) cc++;
                    else break;
                }
                map[a] = (uint8_t)cc;
                dacc[cc] += (uint32_t)a * alphas[a];
                accum[cc] += alphas[a];
            }
        }
        int displaced = 0;
        wa = 0;
        tw = 0;
        for (int n = 0; n < ns; n++) {
            if (accum[n] > 0) {
                uint8_t nc = (uint8_t)((dacc[n] + accum[n] / 2) / accum[n]);
                displaced += or_abs(centers[n] - nc);
                centers[n] = nc;
                wa += (int64_t)nc * (int32_t)accum[n];
                tw += accum[n];
            }
        }
        if (displaced < 5) break;
    }
    if (tw > 0) *wavg = (int)(((int32_t)wa + (int32_t)tw / 2) / (int32_t)tw);
    else *wavg = 128;
}

/* ======================================================================== */
/* Encoder state (vp8.rs:174-277)                                            */
/* ======================================================================== */

typedef struct { uint8_t y2, y[4], u[2], v[2]; } cplx_t;

typedef struct {
    int luma_mode;       /* 0..3 I16, 4 = B */
    uint8_t bpred[16];
    int chroma_mode;
    int segment_id;      /* -1 = None */
    int skipped;
} mbinfo_t;

typedef struct {
    int width, height, mbw, mbh, method;
    uint8_t *Y, *U, *V;
    int ys, cs;
    seg_t seg[4];
    int seg_enabled, seg_update_map;
    uint8_t seg_probs[3];
    uint8_t *seg_map;
    int filter_level, sharpness;
    int qi;
    int skip_prob; /* -1 = None */
    uint8_t probs[4][8][3][11];
    int have_updated;
    uint8_t updated[4][8][3][11];
    uint32_t stats[4][8][3][11];
    lcost_t lc;
    int do_trellis;
    cplx_t *top_c, left_c;
    uint8_t *top_bpred, left_bpred[4];
    uint8_t left_y[17], left_u[9], left_v[9];
    uint8_t *top_y, *top_u, *top_v;
    int8_t (*top_derr)[2][2];
    int8_t left_derr[2][2];
    benc_t hdr, parts[8], *part; /* token partitions; part = the current row's (mby % nparts) */
    int nparts;
    or_enc_debug *dbg;
    int pass;
} enc_t;

static const seg_t *seg_for(const enc_t *e, int mbx, int mby)
{
    int id = (e->seg_enabled && e->seg_map) ? e->seg_map[mby * e->mbw + mbx] : 0;
    return &e->seg[id];
}

/* ---- distortion helpers (vp8.rs:66-127, cost.rs:59-160) ---- */
static uint32_t sse_ws(const uint8_t *src, int ss, const uint8_t *ws, int size)
{
    uint32_t s = 0;
    for (int y = 0; y < size; y++)
        for (int x = 0; x < size; x++) {
            int d = src[y * ss + x] - ws[(y + 1) * OR_BPS + 1 + x];
            s += (uint32_t)(d * d);
        }
    return s;
}
static int t_xform(const uint8_t *in, int stride, const uint16_t *w) /* t_transform cost.rs:59 */
{
    int tmp[16];
    for (int i = 0; i < 4; i++) {
        const uint8_t *r = in + i * stride;
        int a0 = r[0] + r[2], a1 = r[1] + r[3], a2 = r[1] - r[3], a3 = r[0] - r[2];
        tmp[i * 4] = a0 + a1;
        tmp[i * 4 + 1] = a3 + a2;
        tmp[i * 4 + 2] = a3 - a2;
        tmp[i * 4 + 3] = a0 - a1;
    }
    int sum = 0;
    for (int i = 0; i < 4; i++) {
        int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
        int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
        int b0 = a0 + a1, b1 = a3 + a2, b2 = a3 - a2, b3 = a0 - a1;
        sum += w[i] * or_abs(b0) + w[4 + i] * or_abs(b1) + w[8 + i] * or_abs(b2) + w[12 + i] * or_abs(b3);
    }
    return sum;
}
static int tdisto16(const uint8_t *a, const uint8_t *b, int stride) /* tdisto_16x16 cost.rs:137 */
{
    int d = 0;
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) {
            int off = y * 4 * stride + x * 4;
            d += or_abs(t_xform(b + off, stride, VP8_WEIGHT_Y) - t_xform(a + off, stride, VP8_WEIGHT_Y)) >> 5;
        }
    return d;
}
static int is_flat_src16(const uint8_t *s, int stride)
{
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++)
            if (s[y * stride + x] != s[0]) return 0;
    return 1;
}
static int is_flat_coeffs(const int32_t *lv, int nblk, int thresh) /* cost.rs:199 */
{
    int score = 0;
    for (int b = 0; b < nblk; b++)
        for (int i = 1; i < 16; i++)
            if ((int16_t)lv[b * 16 + i] != 0) {
                if (++score > thresh) return 0;
            }
    return 1;
}

/* residual + fDCT of a 4x4 block (ftransform2 / dct4x4 dispatch, equal to scalar for |res|<=255) */
static void fdct_res(const uint8_t *src, int ss, const uint8_t *pred, int ps, int32_t out[16])
{
    for (int y = 0; y < 4; y++)
        for (int x = 0; x < 4; x++) out[y * 4 + x] = src[y * ss + x] - pred[y * ps + x];
    or_fdct_sse2(out);
}

/* get_predicted_luma_block_16x16 vp8.rs:2512 */
static void pred_luma16(const enc_t *e, int mode, int mbx, int mby, uint8_t ws[OR_LUMA_WS])
{
    or_border_luma(ws, mbx, mby, e->mbw, e->top_y, e->left_y);
    switch (mode) {
    case 1: or_pred_v(ws, 16, 1, 1, OR_BPS); break;
    case 2: or_pred_h(ws, 16, 1, 1, OR_BPS); break;
    case 3: or_pred_tm(ws, 16, 1, 1, OR_BPS); break;
    default: or_pred_dc(ws, 16, OR_BPS, mby != 0, mbx != 0); break;
    }
}
/* get_predicted_chroma_block vp8.rs:2940 */
static void pred_chroma(int mode, int mbx, int mby, const uint8_t *top, const uint8_t *left, uint8_t ws[OR_CHROMA_WS])
{
    or_border_chroma(ws, mbx, mby, top, left);
    switch (mode) {
    case 1: or_pred_v(ws, 8, 1, 1, OR_BPS); break;
    case 2: or_pred_h(ws, 8, 1, 1, OR_BPS); break;
    case 3: or_pred_tm(ws, 8, 1, 1, OR_BPS); break;
    default: or_pred_dc(ws, 8, OR_BPS, mby != 0, mbx != 0); break;
    }
}
static void luma_blocks16(const enc_t *e, const uint8_t *ws, int mbx, int mby, int32_t out[256])
{
    for (int by = 0; by < 4; by++)
        for (int bx = 0; bx < 4; bx++)
            fdct_res(e->Y + (mby * 16 + by * 4) * e->ys + mbx * 16 + bx * 4, e->ys,
                     ws + (by * 4 + 1) * OR_BPS + bx * 4 + 1, OR_BPS, out + (by * 4 + bx) * 16);
}
static void chroma_blocks(const enc_t *e, const uint8_t *ws, const uint8_t *plane, int mbx, int mby, int32_t out[64])
{
    for (int by = 0; by < 2; by++)
        for (int bx = 0; bx < 2; bx++)
            fdct_res(plane + (mby * 8 + by * 4) * e->cs + mbx * 8 + bx * 4, e->cs,
                     ws + (by * 4 + 1) * OR_BPS + bx * 4 + 1, OR_BPS, out + (by * 2 + bx) * 16);
}

/* ---- pick_best_intra16 vp8.rs:1504-1687 ---- */
static int pick_i16(const enc_t *e, int mbx, int mby, uint64_t *score_out)
{
    const seg_t *s = seg_for(e, mbx, mby);
    const uint8_t *src = e->Y + mby * 16 * e->ys + mbx * 16;
    int flat = is_flat_src16(src, e->ys);
    int best_mode = 0;
    int64_t best_rd = INT64_MAX;
    uint32_t best_cc = 0, best_sse = 0;
    uint16_t best_mc = 0;
    int32_t best_sd = 0;
    for (int mode = 0; mode < 4; mode++) {
        if (mode == 1 && mby == 0) continue;
        if (mode == 2 && mbx == 0) continue;
        if (mode == 3 && (mbx == 0 || mby == 0)) continue;
        uint8_t ws[OR_LUMA_WS];
        pred_luma16(e, mode, mbx, mby, ws);
        int32_t lb[256];
        luma_blocks16(e, ws, mbx, mby, lb);
        int32_t y2[16], y2q[16], y1q[256];
        for (int i = 0; i < 16; i++) y2[i] = lb[i * 16];
        or_wht(y2);
        for (int i = 0; i < 16; i++) y2q[i] = quant(&s->y2, y2[i], i);
        for (int b = 0; b < 16; b++) {
            y1q[b * 16] = 0;
            for (int i = 1; i < 16; i++) y1q[b * 16 + i] = quant(&s->y1, lb[b * 16 + i], i);
        }
        uint32_t cc = residual_cost(0, y2q, 1, 0, &e->lc, (const uint8_t(*)[8][3][11])e->probs);
        for (int b = 0; b < 16; b++) cc += residual_cost(0, y1q + b * 16, 0, 1, &e->lc, (const uint8_t(*)[8][3][11])e->probs);
        int32_t y2d[16];
        for (int i = 0; i < 16; i++) y2d[i] = dequant(&s->y2, y2q[i], i);
        or_iwht(y2d);
        uint8_t rec[OR_LUMA_WS];
        memcpy(rec, ws, OR_LUMA_WS);
        for (int b = 0; b < 16; b++) {
            int32_t blk[16];
            blk[0] = y2d[b];
            for (int i = 1; i < 16; i++) blk[i] = dequant(&s->y1, y1q[b * 16 + i], i);
            or_idct(blk);
            or_add_residue(rec, blk, 1 + (b / 4) * 4, 1 + (b % 4) * 4, OR_BPS);
        }
        uint32_t sse = sse_ws(src, e->ys, rec, 16);
        int32_t sd = 0;
        if (s->tlambda > 0) {
            uint8_t sb[256], rb[256];
            for (int y = 0; y < 16; y++)
                for (int x = 0; x < 16; x++) {
                    sb[y * 16 + x] = src[y * e->ys + x];
                    rb[y * 16 + x] = rec[(y + 1) * OR_BPS + x + 1];
                }
            int td = tdisto16(sb, rb, 16);
            sd = ((int32_t)s->tlambda * td + 128) >> 8;
        }
        uint32_t dfin = sse;
        int32_t sdfin = sd;
        if (flat && is_flat_coeffs(y1q, 16, 0)) { dfin = sse * 2; sdfin = sd * 2; }
        uint16_t mc = FIXED_COSTS_I16[mode];
        int64_t rd = ((int64_t)mc + cc) * (int64_t)s->l_i16 + 256 * ((int64_t)dfin + sdfin);
        if (rd < best_rd) {
            best_rd = rd; best_mode = mode; best_cc = cc; best_mc = mc; best_sse = dfin; best_sd = sdfin;
        }
    }
    int64_t fin = ((int64_t)best_mc + best_cc) * (int64_t)s->l_mode + 256 * ((int64_t)best_sse + best_sd);
    *score_out = fin < 0 ? 0 : (uint64_t)fin;
    return best_mode;
}

static inline uint64_t rd_score(uint32_t sse, uint16_t rate, uint32_t lambda)
{
    return (uint64_t)sse * 256 + (uint64_t)rate * lambda;
}

/* ---- pick_best_intra4 vp8.rs:1790-2040; returns 1 when I4 wins ---- */
static int pick_i4(const enc_t *e, int mbx, int mby, uint64_t i16_score, uint8_t modes[16])
{
    uint8_t ws[OR_LUMA_WS];
    or_border_luma(ws, mbx, mby, e->mbw, e->top_y, e->left_y);
    const seg_t *s = seg_for(e, mbx, mby);
    uint64_t running = 211ull * s->l_mode;
    uint32_t total_mode_cost = 0;
    const uint32_t max_hdr = 256 * 16 * 16 / 4;
    int top_nz[4] = {0}, left_nz[4] = {0};
    int bidx[16] = {0};
    int maxm = e->method <= 3 ? 3 : (e->method == 4 ? 4 : 10);
    for (int sby = 0; sby < 4; sby++)
        for (int sbx = 0; sbx < 4; sbx++) {
            int i = sby * 4 + sbx, y0 = sby * 4 + 1, x0 = sbx * 4 + 1;
            int tctx = sby == 0 ? 0 : bidx[(sby - 1) * 4 + sbx];
            int lctx = sbx == 0 ? 0 : bidx[sby * 4 + sbx - 1];
            int nzt = sby == 0 ? 0 : top_nz[sbx];
            int nzl = sbx == 0 ? 0 : left_nz[sby];
            uint8_t pr[10][16];
            or_i4_preds(ws, x0, y0, OR_BPS, pr);
            uint8_t sb[16];
            const uint8_t *src = e->Y + (mby * 16 + sby * 4) * e->ys + mbx * 16 + sbx * 4;
            for (int y = 0; y < 4; y++) memcpy(sb + y * 4, src + y * e->ys, 4);
            uint32_t msse[10];
            int order[10];
            for (int m = 0; m < 10; m++) {
                uint32_t t = 0;
                for (int k = 0; k < 16; k++) {
                    int d = sb[k] - pr[m][k];
                    t += (uint32_t)(d * d);
                }
                msse[m] = t;
                order[m] = m;
            }
            /* sort_unstable_by_key on 10 entries: insertion sort (stable), quirk A12 */
            for (int a = 1; a < 10; a++) {
                int v = order[a], b = a;
                while (b > 0 && msse[order[b - 1]] > msse[v]) { order[b] = order[b - 1]; b--; }
                order[b] = v;
            }
            uint64_t bscore = UINT64_MAX;
            int bmode = 0, bnz = 0;
            int32_t bq[16] = {0};
            uint32_t bsse = 0, brate = 0;
            for (int k = 0; k < maxm; k++) {
                int m = order[k];
                int32_t res[16], q[16];
                for (int t = 0; t < 16; t++) res[t] = sb[t] - pr[m][t];
                or_fdct_sse2(res);
                for (int t = 0; t < 16; t++) q[t] = quant(&s->y1, res[t], t);
                int ctx = nzt + nzl;
                uint32_t cc = residual_cost(ctx, q, 3, 0, &e->lc, (const uint8_t(*)[8][3][11])e->probs);
                int hnz = 0;
                for (int t = 0; t < 16; t++) hnz |= q[t] != 0;
                int32_t dq[16];
                for (int t = 0; t < 16; t++) dq[t] = dequant(&s->y1, q[t], t);
                or_idct(dq);
                uint32_t sse = 0;
                for (int t = 0; t < 16; t++) {
                    int r = or_clamp(pr[m][t] + dq[t], 0, 255);
                    int d = sb[t] - r;
                    sse += (uint32_t)(d * d);
                }
                uint16_t mc = VP8_FIXED_COSTS_I4[tctx][lctx][m];
                uint32_t rate = (uint32_t)mc + cc;
                uint64_t sc = rd_score(sse, (uint16_t)rate, s->l_i4);
                if (sc < bscore) {
                    bscore = sc; bmode = m; bnz = hnz; memcpy(bq, q, sizeof q); bsse = sse; brate = rate;
                }
            }
            modes[i] = (uint8_t)bmode;
            bidx[i] = bmode;
            top_nz[sbx] = bnz;
            left_nz[sby] = bnz;
            total_mode_cost += VP8_FIXED_COSTS_I4[tctx][lctx][bmode];
            running += rd_score(bsse, (uint16_t)brate, s->l_mode);
            if (running >= i16_score) return 0;
            if (total_mode_cost > max_hdr) return 0;
            or_pred_b(ws, bmode, x0, y0, OR_BPS);
            int32_t dq[16];
            for (int t = 0; t < 16; t++) dq[t] = dequant(&s->y1, bq[t], t);
            or_idct(dq);
            or_add_residue(ws, dq, y0, x0, OR_BPS);
        }
    return 1;
}

/* ---- pick_best_uv vp8.rs:2050-2200 ---- */
static int pick_uv(const enc_t *e, int mbx, int mby)
{
    const seg_t *s = seg_for(e, mbx, mby);
    int best = 0;
    int64_t best_rd = INT64_MAX;
    for (int mode = 0; mode < 4; mode++) {
        if (mode == 1 && mby == 0) continue;
        if (mode == 2 && mbx == 0) continue;
        if (mode == 3 && (mbx == 0 || mby == 0)) continue;
        uint8_t pu[OR_CHROMA_WS], pv[OR_CHROMA_WS];
        pred_chroma(mode, mbx, mby, e->top_u, e->left_u, pu);
        pred_chroma(mode, mbx, mby, e->top_v, e->left_v, pv);
        int32_t ub[64], vb[64], q[128];
        chroma_blocks(e, pu, e->U, mbx, mby, ub);
        chroma_blocks(e, pv, e->V, mbx, mby, vb);
        for (int b = 0; b < 4; b++)
            for (int i = 0; i < 16; i++) {
                q[b * 16 + i] = quant(&s->uv, ub[b * 16 + i], i);
                q[(4 + b) * 16 + i] = quant(&s->uv, vb[b * 16 + i], i);
            }
        uint32_t cc = 0;
        for (int b = 0; b < 8; b++) cc += residual_cost(0, q + b * 16, 2, 0, &e->lc, (const uint8_t(*)[8][3][11])e->probs);
        uint8_t ru[OR_CHROMA_WS], rv[OR_CHROMA_WS];
        memcpy(ru, pu, sizeof ru);
        memcpy(rv, pv, sizeof rv);
        for (int b = 0; b < 4; b++) {
            int32_t bu[16], bv[16];
            for (int i = 0; i < 16; i++) {
                bu[i] = dequant(&s->uv, q[b * 16 + i], i);
                bv[i] = dequant(&s->uv, q[(4 + b) * 16 + i], i);
            }
            or_idct(bu);
            or_idct(bv);
            or_add_residue(ru, bu, 1 + (b / 2) * 4, 1 + (b % 2) * 4, OR_BPS);
            or_add_residue(rv, bv, 1 + (b / 2) * 4, 1 + (b % 2) * 4, OR_BPS);
        }
        uint32_t sse = sse_ws(e->U + mby * 8 * e->cs + mbx * 8, e->cs, ru, 8) +
                       sse_ws(e->V + mby * 8 * e->cs + mbx * 8, e->cs, rv, 8);
        uint32_t pen = 0;
        if (mode > 0 && is_flat_coeffs(q, 8, 2)) pen = 140 * 8;
        int64_t rd = ((int64_t)FIXED_COSTS_UV[mode] + cc + pen) * (int64_t)s->l_uv + 256 * (int64_t)sse;
        if (rd < best_rd) { best_rd = rd; best = mode; }
    }
    return best;
}

/* ---- choose_macroblock_info vp8.rs:2202-2245 ---- */
static void choose_mb(const enc_t *e, int mbx, int mby, mbinfo_t *mi)
{
    uint64_t i16s;
    int lm = pick_i16(e, mbx, mby, &i16s);
    mi->luma_mode = lm;
    memset(mi->bpred, 0, 16);
    if (e->method > 1) {
        const seg_t *s = seg_for(e, mbx, mby);
        uint64_t thr = 211ull * s->l_mode;
        int try4 = e->method >= 5 || i16s > thr || lm != 0;
        if (try4) {
            uint8_t modes[16];
            if (pick_i4(e, mbx, mby, i16s, modes)) {
                mi->luma_mode = 4;
                memcpy(mi->bpred, modes, 16);
            }
        }
    }
    mi->chroma_mode = pick_uv(e, mbx, mby);
    mi->segment_id = (e->seg_enabled && e->seg_map) ? e->seg_map[mby * e->mbw + mbx] : -1;
    mi->skipped = 0;
}

static void store_recon(const enc_t *e, const uint8_t *ws, int size, int stride_ws, uint8_t *plane, int ps, int x0, int y0)
{
    (void)e;
    for (int y = 0; y < size; y++) memcpy(plane + (size_t)(y0 + y) * ps + x0, ws + (y + 1) * stride_ws + 1, size);
}

/* ---- transform_luma_block vp8.rs:2647-2780 / transform_luma_blocks_4x4 :2785-2916 ---- */
static void transform_luma(enc_t *e, int mbx, int mby, const mbinfo_t *mi, int32_t lb[256])
{
    const seg_t *s = &e->seg[mi->segment_id < 0 ? 0 : mi->segment_id];
    uint8_t ws[OR_LUMA_WS];
    int top_nz[4], left_nz[4];
    for (int i = 0; i < 4; i++) {
        top_nz[i] = e->top_c[mbx].y[i] != 0;
        left_nz[i] = e->left_c.y[i] != 0;
    }
    if (mi->luma_mode != 4) {
        pred_luma16(e, mi->luma_mode, mbx, mby, ws);
        luma_blocks16(e, ws, mbx, mby, lb);
        int32_t c0[16];
        for (int i = 0; i < 16; i++) c0[i] = lb[i * 16];
        or_wht(c0);
        for (int i = 0; i < 16; i++) c0[i] = quant(&s->y2, c0[i], i);
        int32_t y2d[16];
        for (int i = 0; i < 16; i++) y2d[i] = dequant(&s->y2, c0[i], i);
        or_iwht(y2d);
        int32_t deq[256];
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int i = y * 4 + x;
                int32_t blk[16];
                memcpy(blk, lb + i * 16, sizeof blk);
                if (e->do_trellis) {
                    int ctx0 = left_nz[y] + top_nz[x];
                    if (ctx0 > 2) ctx0 = 2;
                    int32_t zz[16] = {0};
                    int nz = trellis(blk, zz, &s->y1, s->lt_i16, 1, &e->lc, 0, ctx0);
                    top_nz[x] = nz;
                    left_nz[y] = nz;
                } else {
                    int nz = 0;
                    blk[0] = 0;
                    for (int k = 1; k < 16; k++) {
                        int l = quant(&s->y1, blk[k], k);
                        nz |= l != 0;
                        blk[k] = dequant(&s->y1, l, k);
                    }
                    top_nz[x] = nz;
                    left_nz[y] = nz;
                }
                blk[0] = y2d[i];
                or_idct(blk);
                memcpy(deq + i * 16, blk, sizeof blk);
            }
        for (int i = 0; i < 16; i++) or_add_residue(ws, deq + i * 16, 1 + (i / 4) * 4, 1 + (i % 4) * 4, OR_BPS);
    } else {
        or_border_luma(ws, mbx, mby, e->mbw, e->top_y, e->left_y);
        for (int sby = 0; sby < 4; sby++)
            for (int sbx = 0; sbx < 4; sbx++) {
                int i = sby * 4 + sbx, y0 = sby * 4 + 1, x0 = sbx * 4 + 1;
                or_pred_b(ws, mi->bpred[i], x0, y0, OR_BPS);
                int32_t cur[16];
                const uint8_t *src = e->Y + (mby * 16 + sby * 4) * e->ys + mbx * 16 + sbx * 4;
                fdct_res(src, e->ys, ws + y0 * OR_BPS + x0, OR_BPS, cur);
                memcpy(lb + i * 16, cur, sizeof cur);
                if (e->dbg && e->dbg->i4_dump && e->pass == 2) {
                    int32_t *d = e->dbg->i4_dump + ((size_t)(mby * e->mbw + mbx) * 16 + i) * 34;
                    memcpy(d, cur, 16 * sizeof(int32_t));
                    for (int k = 0; k < 16; k++) d[16 + k] = ws[(y0 + k / 4) * OR_BPS + x0 + k % 4];
                    int c0 = left_nz[sby] + top_nz[sbx];
                    d[32] = c0 > 2 ? 2 : c0;
                    d[33] = mi->bpred[i];
                }
                int nz;
                if (e->do_trellis) {
                    int ctx0 = left_nz[sby] + top_nz[sbx];
                    if (ctx0 > 2) ctx0 = 2;
                    int32_t zz[16] = {0};
                    nz = trellis(cur, zz, &s->y1, s->lt_i4, 0, &e->lc, 3, ctx0);
                } else {
                    nz = 0;
                    for (int k = 0; k < 16; k++) {
                        int l = quant(&s->y1, cur[k], k);
                        nz |= l != 0;
                        cur[k] = dequant(&s->y1, l, k);
                    }
                }
                top_nz[sbx] = nz;
                left_nz[sby] = nz;
                or_idct(cur);
                or_add_residue(ws, cur, y0, x0, OR_BPS);
            }
    }
    for (int y = 0; y < 17; y++) e->left_y[y] = ws[y * OR_BPS + 16];
    for (int x = 0; x < 16; x++) e->top_y[mbx * 16 + x] = ws[16 * OR_BPS + x + 1];
    if (e->dbg && e->pass == 2 && e->dbg->recon_y) store_recon(e, ws, 16, OR_BPS, e->dbg->recon_y, e->ys, mbx * 16, mby * 16);
    if (e->dbg && e->pass == 1 && e->dbg->recon1_y) store_recon(e, ws, 16, OR_BPS, e->dbg->recon1_y, e->ys, mbx * 16, mby * 16);
}

/* apply_chroma_error_diffusion vp8.rs:572-647 */
static int8_t diffuse(int32_t *dc, int8_t te, int8_t le, const mtx_t *m)
{
    int q = m->q[0];
    uint32_t iq = m->iq[0], bias = m->bias[0];
    int adj = (7 * te + 8 * le) >> 3;
    *dc += adj;
    int sign = *dc < 0;
    uint32_t a = (uint32_t)(sign ? -*dc : *dc);
    uint32_t zt = ((1u << 17) - 1 - bias) / iq;
    int level = a > zt ? (int)((a * iq + bias) >> 17) : 0;
    int err = (int)a - level * q;
    int se = sign ? -err : err;
    return (int8_t)or_clamp(se >> 1, -127, 127);
}
static void error_diffusion(enc_t *e, int32_t ub[64], int32_t vb[64], int mbx, const mtx_t *m)
{
    for (int ch = 0; ch < 2; ch++) {
        int32_t *b = ch ? vb : ub;
        int8_t *top = e->top_derr[mbx][ch], *left = e->left_derr[ch];
        int8_t e0 = diffuse(&b[0], top[0], left[0], m);
        int8_t e1 = diffuse(&b[16], top[1], e0, m);
        int8_t e2 = diffuse(&b[32], e0, left[1], m);
        int8_t e3 = diffuse(&b[48], e1, e2, m);
        left[0] = e1;
        left[1] = (int8_t)((3 * e3) >> 2);
        top[0] = e2;
        top[1] = (int8_t)(e3 - left[1]);
    }
}

/* transform_chroma_blocks vp8.rs:3039-3121 */
static void transform_chroma(enc_t *e, int mbx, int mby, int mode, int32_t ub[64], int32_t vb[64])
{
    const seg_t *s = seg_for(e, mbx, mby);
    uint8_t pu[OR_CHROMA_WS], pv[OR_CHROMA_WS];
    pred_chroma(mode, mbx, mby, e->top_u, e->left_u, pu);
    pred_chroma(mode, mbx, mby, e->top_v, e->left_v, pv);
    chroma_blocks(e, pu, e->U, mbx, mby, ub);
    chroma_blocks(e, pv, e->V, mbx, mby, vb);
    if (e->dbg && e->dbg->derr_in && e->pass == 2) {
        int8_t *d = e->dbg->derr_in + (size_t)(mby * e->mbw + mbx) * 8;
        for (int ch = 0; ch < 2; ch++) {
            d[4 * ch + 0] = e->top_derr[mbx][ch][0];
            d[4 * ch + 1] = e->top_derr[mbx][ch][1];
            d[4 * ch + 2] = e->left_derr[ch][0];
            d[4 * ch + 3] = e->left_derr[ch][1];
        }
    }
    error_diffusion(e, ub, vb, mbx, &s->uv);
    for (int b = 0; b < 4; b++) {
        int32_t du[16], dv[16];
        for (int i = 0; i < 16; i++) {
            du[i] = dequant(&s->uv, quant(&s->uv, ub[b * 16 + i], i), i);
            dv[i] = dequant(&s->uv, quant(&s->uv, vb[b * 16 + i], i), i);
        }
        or_idct(du);
        or_idct(dv);
        or_add_residue(pu, du, 1 + (b / 2) * 4, 1 + (b % 2) * 4, OR_BPS);
        or_add_residue(pv, dv, 1 + (b / 2) * 4, 1 + (b % 2) * 4, OR_BPS);
    }
    for (int y = 0; y < 9; y++) {
        e->left_u[y] = pu[y * OR_BPS + 8];
        e->left_v[y] = pv[y * OR_BPS + 8];
    }
    for (int x = 0; x < 8; x++) {
        e->top_u[mbx * 8 + x] = pu[8 * OR_BPS + x + 1];
        e->top_v[mbx * 8 + x] = pv[8 * OR_BPS + x + 1];
    }
    if (e->dbg && e->pass == 2 && e->dbg->recon_u) {
        store_recon(e, pu, 8, OR_BPS, e->dbg->recon_u, e->cs, mbx * 8, mby * 8);
        store_recon(e, pv, 8, OR_BPS, e->dbg->recon_v, e->cs, mbx * 8, mby * 8);
    }
}

/* check_all_coeffs_zero vp8.rs:962-1023 */
static int all_zero(const enc_t *e, const mbinfo_t *mi, const int32_t *lb, const int32_t *ub, const int32_t *vb)
{
    const seg_t *s = &e->seg[mi->segment_id < 0 ? 0 : mi->segment_id];
    if (mi->luma_mode != 4) {
        int32_t c0[16];
        for (int i = 0; i < 16; i++) c0[i] = lb[i * 16];
        or_wht(c0);
        for (int i = 0; i < 16; i++)
            if (quant(&s->y2, c0[i], i) != 0) return 0;
        for (int b = 0; b < 16; b++)
            for (int i = 1; i < 16; i++)
                if (quant(&s->y1, lb[b * 16 + i], i) != 0) return 0;
    } else {
        for (int b = 0; b < 16; b++)
            for (int i = 0; i < 16; i++)
                if (quant(&s->y1, lb[b * 16 + i], i) != 0) return 0;
    }
    for (int b = 0; b < 4; b++)
        for (int i = 0; i < 16; i++)
            if (quant(&s->uv, ub[b * 16 + i], i) != 0 || quant(&s->uv, vb[b * 16 + i], i) != 0) return 0;
    return 1;
}

/* ProbaStats::record cost.rs:1200 */
static inline void rec_stat(uint32_t *s, int bit)
{
    if (*s >= 0xfffe0000u) *s = ((*s + 1) >> 1) & 0x7fff7fffu;
    *s += 0x00010000u + (bit ? 1 : 0);
}

/* record_coeffs cost.rs:1297-1397 */
static void record_coeffs(enc_t *e, const int32_t *c, int t, int first, int ctx)
{
    int last = -1;
    for (int i = 15; i >= 0; i--)
        if (c[i] != 0) { last = i; break; }
    int eob = last >= 0 ? last + 1 : 0;
    int n = first;
    if (eob <= first) {
        rec_stat(&e->stats[t][VP8_ENC_BANDS[first]][ctx][0], 0);
        return;
    }
    int skip_eob = 0;
    while (n < eob) {
        int band = VP8_ENC_BANDS[n];
        uint32_t v = (uint32_t)or_abs(c[n]);
        n++;
        uint32_t *S = e->stats[t][band][ctx];
        if (!skip_eob) rec_stat(&S[0], 1);
        if (v == 0) {
            rec_stat(&S[1], 0);
            skip_eob = 1;
            ctx = 0;
            continue;
        }
        rec_stat(&S[1], 1);
        if (v == 1) {
            rec_stat(&S[2], 0);
            ctx = 1;
        } else {
            rec_stat(&S[2], 1);
            if (v > MAX_VLEVEL) v = MAX_VLEVEL;
            if (v <= 4) {
                rec_stat(&S[3], 0);
                if (v == 2) rec_stat(&S[4], 0);
                else {
                    rec_stat(&S[4], 1);
                    rec_stat(&S[5], v == 4);
                }
            } else if (v <= 10) {
                rec_stat(&S[3], 1);
                rec_stat(&S[6], 0);
                rec_stat(&S[7], v > 6);
            } else {
                rec_stat(&S[3], 1);
                rec_stat(&S[6], 1);
                if (v < 3 + (8 << 2)) {
                    rec_stat(&S[8], 0);
                    rec_stat(&S[9], v >= 3 + (8 << 1));
                } else {
                    rec_stat(&S[8], 1);
                    rec_stat(&S[10], v >= 3 + (8 << 3));
                }
            }
            ctx = 2;
        }
    }
    if (n < 16) rec_stat(&e->stats[t][VP8_ENC_BANDS[n]][ctx][0], 0);
}

static void cplx_clear(cplx_t *c, int y2)
{
    memset(c->y, 0, 4);
    memset(c->u, 0, 2);
    memset(c->v, 0, 2);
    if (y2) c->y2 = 0;
}

/* record_residual_stats vp8.rs:1027-1200 */
static void record_residual_stats(enc_t *e, const mbinfo_t *mi, int mbx, const int32_t *lb, const int32_t *ub,
                                  const int32_t *vb)
{
    const seg_t *s = &e->seg[mi->segment_id < 0 ? 0 : mi->segment_id];
    int is_i4 = mi->luma_mode == 4;
    if (!is_i4) {
        int32_t c0[16], zz[16];
        for (int i = 0; i < 16; i++) c0[i] = lb[i * 16];
        or_wht(c0);
        for (int i = 0; i < 16; i++) zz[i] = quant(&s->y2, c0[ZIGZAG[i]], ZIGZAG[i]);
        int cx = e->left_c.y2 + e->top_c[mbx].y2;
        record_coeffs(e, zz, 1, 0, cx < 2 ? cx : 2);
        int hc = 0;
        for (int i = 0; i < 16; i++) hc |= zz[i] != 0;
        e->left_c.y2 = e->top_c[mbx].y2 = (uint8_t)hc;
    }
    int tt = is_i4 ? 3 : 0, first = is_i4 ? 0 : 1;
    uint32_t tl = is_i4 ? s->lt_i4 : s->lt_i16;
    for (int y = 0; y < 4; y++) {
        int left = e->left_c.y[y];
        for (int x = 0; x < 4; x++) {
            int32_t zz[16] = {0};
            int ctx0 = left + e->top_c[mbx].y[x];
            if (ctx0 > 2) ctx0 = 2;
            if (e->do_trellis) {
                int32_t cc[16];
                memcpy(cc, lb + (y * 4 + x) * 16, sizeof cc);
                trellis(cc, zz, &s->y1, tl, first, &e->lc, tt, ctx0);
            } else {
                for (int i = first; i < 16; i++) zz[i] = quant(&s->y1, lb[(y * 4 + x) * 16 + ZIGZAG[i]], ZIGZAG[i]);
            }
            record_coeffs(e, zz, tt, first, ctx0);
            int hc = 0;
            for (int i = first; i < 16; i++) hc |= zz[i] != 0;
            left = hc;
            e->top_c[mbx].y[x] = (uint8_t)hc;
        }
        e->left_c.y[y] = (uint8_t)left;
    }
    for (int pl = 0; pl < 2; pl++) {
        const int32_t *cb = pl ? vb : ub;
        uint8_t *lc = pl ? e->left_c.v : e->left_c.u;
        uint8_t *tc = pl ? e->top_c[mbx].v : e->top_c[mbx].u;
        for (int y = 0; y < 2; y++) {
            int left = lc[y];
            for (int x = 0; x < 2; x++) {
                int32_t zz[16];
                for (int i = 0; i < 16; i++) zz[i] = quant(&s->uv, cb[(y * 2 + x) * 16 + ZIGZAG[i]], ZIGZAG[i]);
                int cx = left + tc[x];
                record_coeffs(e, zz, 2, 0, cx < 2 ? cx : 2);
                int hc = 0;
                for (int i = 0; i < 16; i++) hc |= zz[i] != 0;
                left = hc;
                tc[x] = (uint8_t)hc;
            }
            lc[y] = (uint8_t)left;
        }
    }
}

/* encode_coefficients vp8.rs:798-958 ; returns has_coeffs; zz_out gets levels */
static int encode_coeffs(enc_t *e, const int32_t *blk, int plane, int ctx, const mtx_t *m, int use_trellis,
                         uint32_t tl, int32_t *zz_out)
{
    int first = plane == 0 ? 1 : 0;
    const uint8_t(*P)[3][11] = (const uint8_t(*)[3][11])e->probs[plane];
    int32_t zz[16] = {0};
    if (use_trellis) {
        int32_t cc[16];
        memcpy(cc, blk, sizeof cc);
        trellis(cc, zz, m, tl, first, &e->lc, plane, ctx);
    } else {
        for (int i = first; i < 16; i++) zz[i] = quant(m, blk[ZIGZAG[i]], ZIGZAG[i]);
    }
    if (zz_out) memcpy(zz_out, zz, sizeof zz);
    int eobi = 0;
    for (int i = 15; i >= 0; i--)
        if (zz[i] != 0) { eobi = i + 1; break; }
    int skip_eob = 0;
    for (int idx = first; idx < eobi; idx++) {
        int coeff = zz[idx];
        const uint8_t *pr = P[COEFF_BANDS[idx]][ctx];
        int start = skip_eob ? 2 : 0;
        int a = or_abs(coeff);
        int token;
        if (a == 0) {
            be_tree(e->part, TOKEN_TREE, 22, pr, 0, start);
            skip_eob = 1;
            token = 0;
        } else if (a <= 4) {
            be_tree(e->part, TOKEN_TREE, 22, pr, a, start);
            skip_eob = 0;
            token = a;
        } else {
            int cat = a <= 6 ? 5 : a <= 10 ? 6 : a <= 18 ? 7 : a <= 34 ? 8 : a <= 66 ? 9 : 10;
            be_tree(e->part, TOKEN_TREE, 22, pr, cat, start);
            const uint8_t *cp = PROB_DCT_CAT[cat - 5];
            int extra = a - DCT_CAT_BASE[cat - 5];
            int mask = cat == 10 ? 1 << 10 : 1 << (cat - 5);
            for (int k = 0; k < 12 && cp[k]; k++) {
                be_bool(e->part, (extra & mask) > 0, cp[k]);
                mask >>= 1;
            }
            skip_eob = 0;
            token = cat;
        }
        if (token != 0) be_flag(e->part, !(coeff > 0));
        ctx = token == 0 ? 0 : (token == 1 ? 1 : 2);
    }
    if (eobi < 16) {
        int bi = first > eobi ? first : eobi;
        be_tree(e->part, TOKEN_TREE, 22, P[COEFF_BANDS[bi]][ctx], 11, 0);
    }
    return eobi > 0;
}

/* encode_residual_data vp8.rs:650-795 */
static void encode_residual(enc_t *e, const mbinfo_t *mi, int mbx, const int32_t *lb, const int32_t *ub,
                            const int32_t *vb, int32_t *lv /* 25*16 or NULL */)
{
    const seg_t *s = &e->seg[mi->segment_id < 0 ? 0 : mi->segment_id];
    int is_i4 = mi->luma_mode == 4;
    int plane = is_i4 ? 3 : 1;
    uint32_t tl = is_i4 ? s->lt_i4 : s->lt_i16;
    if (plane == 1) {
        int32_t c0[16];
        for (int i = 0; i < 16; i++) c0[i] = lb[i * 16];
        or_wht(c0);
        int cx = e->left_c.y2 + e->top_c[mbx].y2;
        int hc = encode_coeffs(e, c0, 1, cx, &s->y2, 0, 0, lv ? lv + 16 * 16 : NULL);
        e->left_c.y2 = e->top_c[mbx].y2 = (uint8_t)hc;
        plane = 0;
    }
    for (int y = 0; y < 4; y++) {
        int left = e->left_c.y[y];
        for (int x = 0; x < 4; x++) {
            int cx = left + e->top_c[mbx].y[x];
            int hc = encode_coeffs(e, lb + (y * 4 + x) * 16, plane, cx, &s->y1, e->do_trellis, tl,
                                   lv ? lv + (y * 4 + x) * 16 : NULL);
            left = hc;
            e->top_c[mbx].y[x] = (uint8_t)hc;
        }
        e->left_c.y[y] = (uint8_t)left;
    }
    for (int pl = 0; pl < 2; pl++) {
        const int32_t *cb = pl ? vb : ub;
        uint8_t *lc = pl ? e->left_c.v : e->left_c.u;
        uint8_t *tc = pl ? e->top_c[mbx].v : e->top_c[mbx].u;
        for (int y = 0; y < 2; y++) {
            int left = lc[y];
            for (int x = 0; x < 2; x++) {
                int cx = left + tc[x];
                int hc = encode_coeffs(e, cb + (y * 2 + x) * 16, 2, cx, &s->uv, 0, 0,
                                       lv ? lv + (17 + 4 * pl + y * 2 + x) * 16 : NULL);
                left = hc;
                tc[x] = (uint8_t)hc;
            }
            lc[y] = (uint8_t)left;
        }
    }
}

/* write_macroblock_header vp8.rs:498-560 */
static void write_mb_header(enc_t *e, const mbinfo_t *mi, int mbx)
{
    if (e->seg_enabled && e->seg_update_map)
        be_tree(&e->hdr, SEGMENT_ID_TREE, 6, e->seg_probs, mi->segment_id < 0 ? 0 : mi->segment_id, 0);
    if (e->skip_prob >= 0) be_bool(&e->hdr, mi->skipped, e->skip_prob);
    be_tree(&e->hdr, YMODE_TREE, 8, KEYFRAME_YMODE_PROBS, mi->luma_mode, 0);
    if (mi->luma_mode == 4) {
        for (int y = 0; y < 4; y++) {
            int left = e->left_bpred[y];
            for (int x = 0; x < 4; x++) {
                int top = e->top_bpred[mbx * 4 + x];
                int m = mi->bpred[y * 4 + x];
                be_tree(&e->hdr, BMODE_TREE, 18, KEYFRAME_BPRED_MODE_PROBS[top][left], m, 0);
                left = m;
                e->top_bpred[mbx * 4 + x] = (uint8_t)m;
            }
            e->left_bpred[y] = (uint8_t)left;
        }
    } else {
        static const int intra_of[4] = {0, 2, 3, 1}; /* into_intra: DC->DC, V->VE, H->HE, TM->TM */
        for (int i = 0; i < 4; i++) {
            e->left_bpred[i] = (uint8_t)intra_of[mi->luma_mode];
            e->top_bpred[mbx * 4 + i] = (uint8_t)intra_of[mi->luma_mode];
        }
    }
    be_tree(&e->hdr, UVMODE_TREE, 6, KEYFRAME_UV_MODE_PROBS, mi->chroma_mode, 0);
}

/* ProbaStats::should_update / compute_updated_probabilities cost.rs:1226-1254, vp8.rs:1202-1238 */
static void compute_updated_probs(enc_t *e)
{
    memcpy(e->updated, e->probs, sizeof e->probs);
    int32_t total_sav = 0;
    uint32_t nup = 0;
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++)
                for (int p = 0; p < 11; p++) {
                    uint32_t st = e->stats[t][b][c][p];
                    int nb = (int)(st & 0xffff), tot = (int)(st >> 16);
                    if (tot == 0) continue;
                    uint8_t oldp = e->probs[t][b][c][p], upp = COEFF_UPDATE_PROBS[t][b][c][p];
                    uint8_t newp = (uint8_t)(255 - (uint32_t)nb * 255 / (uint32_t)tot);
                    int oc = nb * VP8_ENTROPY_COST[255 - oldp] + (tot - nb) * VP8_ENTROPY_COST[oldp] + bitcost(0, upp);
                    int nc = nb * VP8_ENTROPY_COST[255 - newp] + (tot - nb) * VP8_ENTROPY_COST[newp] + bitcost(1, upp) + 8 * 256;
                    int sav = oc - nc;
                    if (sav > 0) {
                        e->updated[t][b][c][p] = newp;
                        total_sav += sav;
                        nup++;
                    }
                }
    e->have_updated = total_sav > 0 && nup > 0;
}

/* ======================================================================== */
/* encode_image vp8.rs:1281-1488                                             */
/* ======================================================================== */

static void reset_row(enc_t *e)
{
    memset(&e->left_c, 0, sizeof e->left_c);
    memset(e->left_bpred, 0, 4);
    memset(e->left_y, 129, 17);
    memset(e->left_u, 129, 9);
    memset(e->left_v, 129, 9);
}

int or_encode(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, int quality,
              int method, uint8_t **out, size_t *out_len, or_enc_debug *dbg)
{
    return or_encode_parts(data, len, width, height, color, quality, method, 1, out, out_len, dbg);
}

/* The same with `nparts` (1, 2, 4 or 8) token partitions: MB row y's residual
 * tokens go to partition y % nparts (vp8.rs:1419-1421); the frame header codes
 * log2(nparts) (vp8.rs:352-354).  Layout after the first partition follows RFC
 * 6386 9.5 and the reference decoder (decoder/vp8.rs:421-450): the nparts - 1
 * 3-byte little-endian sizes, then the partitions.  (The reference encoder's own
 * write_partitions, vp8.rs:374-390, would interleave each size with its data;
 * it is never reached, since the encoder always has one partition, vp8.rs:273,
 * :1275.) */
int or_encode_parts(const uint8_t *data, size_t len, uint32_t width, uint32_t height, int color, int quality,
                    int method, int nparts, uint8_t **out, size_t *out_len, or_enc_debug *dbg)
{
    *out = NULL;
    *out_len = 0;
    /* error order follows the reference: u16 dims (vp8.rs:3143), data length
     * assert (vp8.rs:1307), quality panic (vp8.rs:2401) */
    if (width > 65535 || height > 65535 || width == 0 || height == 0) return OR_EINVALID_DIMENSIONS;
    static const int bpp_of[4] = {1, 2, 3, 4};
    if (color < 0 || color > 3) return OR_EINVAL;
    int bpp = bpp_of[color];
    if ((uint64_t)width * height * bpp != len) return OR_EINVALID_BUFFER_SIZE;
    if (quality > 100 || quality < 0) return OR_EINVAL;
    if (nparts != 1 && nparts != 2 && nparts != 4 && nparts != 8) return OR_EINVAL;

    enc_t E, *e = &E;
    memset(e, 0, sizeof E);
    e->nparts = nparts;
    e->dbg = dbg;
    e->width = (int)width;
    e->height = (int)height;
    e->method = method > 6 ? 6 : method;
    e->do_trellis = e->method >= 4;
    e->mbw = (e->width + 15) / 16;
    e->mbh = (e->height + 15) / 16;
    e->ys = e->mbw * 16;
    e->cs = e->mbw * 8;
    size_t ysz = (size_t)e->ys * e->mbh * 16, csz = (size_t)e->cs * e->mbh * 8;
    e->Y = (uint8_t *)calloc(ysz, 1);
    e->U = (uint8_t *)calloc(csz + 64, 1);
    e->V = (uint8_t *)calloc(csz + 64, 1);
    or_rgb_to_yuv420(data, e->width, e->height, bpp, e->Y, e->U, e->V);
    if (dbg && dbg->src_y) {
        memcpy(dbg->src_y, e->Y, ysz);
        memcpy(dbg->src_u, e->U, csz);
        memcpy(dbg->src_v, e->V, csz);
    }

    /* setup_encoding vp8.rs:2391-2508 */
    e->qi = or_quality_to_quant_index(quality);
    e->sharpness = 0;
    e->filter_level = compute_filter_level(e->qi, 0, 50);
    int nmb = e->mbw * e->mbh;
    e->top_c = (cplx_t *)calloc((size_t)e->mbw, sizeof(cplx_t));
    e->top_bpred = (uint8_t *)calloc((size_t)e->mbw * 4, 1);
    memcpy(e->probs, COEFF_PROBS, sizeof e->probs);
    e->skip_prob = 200;
    for (int i = 0; i < 4; i++) seg_from_index(&e->seg[i], e->qi, 0);
    if (nmb >= 256) {
        /* analyze_and_assign_segments vp8.rs:2278-2388 */
        uint8_t *alphas = (uint8_t *)malloc((size_t)nmb);
        uint32_t histo[256];
        or_analyze(e->Y, e->U, e->V, e->width, e->height, alphas, histo);
        uint8_t centers[4], map[256];
        int mid;
        kmeans(histo, centers, map, &mid);
        int minc = centers[0], maxc = centers[0];
        for (int i = 1; i < 4; i++) {
            if (centers[i] < minc) minc = centers[i];
            if (centers[i] > maxc) maxc = centers[i];
        }
        int range = maxc == minc ? 1 : maxc - minc;
        e->seg_map = (uint8_t *)malloc((size_t)nmb);
        for (int i = 0; i < nmb; i++) e->seg_map[i] = map[alphas[i]];
        for (int s = 0; s < 4; s++) {
            int ta = or_clamp(255 * (centers[s] - mid) / range, -127, 127);
            int sq = compute_segment_quant(e->qi, ta, 50);
            int delta = (int8_t)((int8_t)sq - (int8_t)e->qi);
            seg_from_index(&e->seg[s], sq, delta);
        }
        uint32_t cnt[4] = {0};
        for (int i = 0; i < nmb; i++) cnt[e->seg_map[i]]++;
#define GETP(a, b) ((a) + (b) == 0 ? 255 : (uint8_t)((255 * (a) + ((a) + (b)) / 2) / ((a) + (b))))
        e->seg_probs[0] = GETP(cnt[0] + cnt[1], cnt[2] + cnt[3]);
        e->seg_probs[1] = GETP(cnt[0], cnt[1]);
        e->seg_probs[2] = GETP(cnt[2], cnt[3]);
#undef GETP
        e->seg_update_map = e->seg_probs[0] != 255 || e->seg_probs[1] != 255 || e->seg_probs[2] != 255;
        e->seg_enabled = 1;
        if (dbg && dbg->mb_alpha) memcpy(dbg->mb_alpha, alphas, (size_t)nmb);
        free(alphas);
    } else {
        e->seg_enabled = 0;
        e->seg_update_map = 0;
        e->seg_map = NULL;
        e->seg_probs[0] = e->seg_probs[1] = e->seg_probs[2] = 255;
    }
    if (dbg) {
        for (int s = 0; s < 4; s++) dbg->seg_quant_index[s] = e->seg[s].quant_index;
        if (dbg->seg_map) {
            for (int i = 0; i < nmb; i++) dbg->seg_map[i] = e->seg_map ? e->seg_map[i] : 0;
        }
        dbg->segments_enabled = e->seg_enabled;
        dbg->filter_level = e->filter_level;
        dbg->base_quant_index = e->qi;
    }
    e->top_y = (uint8_t *)malloc((size_t)e->mbw * 16 + 64);
    e->top_u = (uint8_t *)malloc((size_t)e->mbw * 8 + 64);
    e->top_v = (uint8_t *)malloc((size_t)e->mbw * 8 + 64);
    memset(e->top_y, 127, (size_t)e->mbw * 16 + 64);
    memset(e->top_u, 127, (size_t)e->mbw * 8 + 64);
    memset(e->top_v, 127, (size_t)e->mbw * 8 + 64);
    e->top_derr = (int8_t(*)[2][2])calloc((size_t)e->mbw, sizeof(int8_t[2][2]));
    memset(e->left_derr, 0, sizeof e->left_derr);
    reset_row(e);

    /* ---------------- PASS 1 ---------------- */
    int trellis_p2 = e->do_trellis;
    e->do_trellis = 0;
    e->pass = 1;
    memset(e->stats, 0, sizeof e->stats);
    uint32_t total_mb = 0, skip_mb = 0;
    int32_t lb[256], ub[64], vb[64];
    for (int mby = 0; mby < e->mbh; mby++) {
        memset(&e->left_c, 0, sizeof e->left_c);
        memset(e->left_bpred, 0, 4);
        memset(e->left_y, 129, 17);
        memset(e->left_u, 129, 9);
        memset(e->left_v, 129, 9);
        /* left_derr intentionally NOT reset (quirk A5, vp8.rs:1337-1346) */
        for (int mbx = 0; mbx < e->mbw; mbx++) {
            mbinfo_t mi;
            choose_mb(e, mbx, mby, &mi);
            transform_luma(e, mbx, mby, &mi, lb);
            transform_chroma(e, mbx, mby, mi.chroma_mode, ub, vb);
            total_mb++;
            int az = all_zero(e, &mi, lb, ub, vb);
            if (dbg && dbg->p1_info) {
                or_mb_info *o = &dbg->p1_info[mby * e->mbw + mbx];
                o->luma_mode = (uint8_t)mi.luma_mode;
                memcpy(o->bpred, mi.bpred, 16);
                o->chroma_mode = (uint8_t)mi.chroma_mode;
                o->segment = (uint8_t)(mi.segment_id < 0 ? 0 : mi.segment_id);
                o->skip = (uint8_t)az;
            }
            if (az) {
                skip_mb++;
                cplx_clear(&e->left_c, mi.luma_mode != 4);
                cplx_clear(&e->top_c[mbx], mi.luma_mode != 4);
            } else {
                record_residual_stats(e, &mi, mbx, lb, ub, vb);
            }
        }
    }
    if (total_mb > 0) {
        uint32_t ns = total_mb - skip_mb;
        uint32_t p = (255 * ns + total_mb / 2) / total_mb;
        if (p > 255) p = 255;
        e->skip_prob = or_clamp((int)(uint8_t)p, 1, 254);
    }
    compute_updated_probs(e);
    lcost_calc(&e->lc, e->have_updated ? (const uint8_t(*)[8][3][11])e->updated : (const uint8_t(*)[8][3][11])e->probs);
    if (dbg) {
        memcpy(dbg->p1_stats, e->stats, sizeof e->stats);
        dbg->skip_prob = e->skip_prob;
    }
    e->do_trellis = trellis_p2;

    /* reset_for_second_pass vp8.rs:1241-1279 (top_derr NOT reset, quirk A6) */
    memset(e->top_c, 0, sizeof(cplx_t) * e->mbw);
    memset(&e->left_c, 0, sizeof e->left_c);
    memset(e->top_bpred, 0, (size_t)e->mbw * 4);
    memset(e->left_bpred, 0, 4);
    memset(e->left_y, 129, 17);
    memset(e->left_u, 129, 9);
    memset(e->left_v, 129, 9);
    memset(e->top_y, 127, (size_t)e->mbw * 16 + 64);
    memset(e->top_u, 127, (size_t)e->mbw * 8 + 64);
    memset(e->top_v, 127, (size_t)e->mbw * 8 + 64);
    for (int p = 0; p < e->nparts; p++) be_init(&e->parts[p]);
    be_init(&e->hdr);

    /* encode_compressed_frame_header vp8.rs:332-372 */
    be_lit(&e->hdr, 1, 0);
    be_lit(&e->hdr, 1, 0);
    be_flag(&e->hdr, e->seg_enabled);
    if (e->seg_enabled) {
        be_flag(&e->hdr, e->seg_update_map);
        be_flag(&e->hdr, 1);
        be_flag(&e->hdr, 0);
        for (int s = 0; s < 4; s++) {
            int ql = e->seg[s].quantizer_level;
            be_flag(&e->hdr, ql != 0);
            if (ql != 0) {
                be_lit(&e->hdr, 7, ql < 0 ? -ql : ql);
                be_flag(&e->hdr, ql < 0);
            }
        }
        for (int s = 0; s < 4; s++) be_flag(&e->hdr, 0);
        if (e->seg_update_map)
            for (int i = 0; i < 3; i++) {
                be_flag(&e->hdr, e->seg_probs[i] != 255);
                if (e->seg_probs[i] != 255) be_lit(&e->hdr, 8, e->seg_probs[i]);
            }
    }
    be_flag(&e->hdr, 0);                 /* filter_type: normal */
    be_lit(&e->hdr, 6, e->filter_level);
    be_lit(&e->hdr, 3, e->sharpness);
    be_flag(&e->hdr, 0);                 /* loop_filter_adjustments */
    be_lit(&e->hdr, 2, e->nparts == 8 ? 3 : e->nparts >> 1); /* log2(token partitions) */
    be_lit(&e->hdr, 7, e->qi);           /* yac_abs */
    for (int i = 0; i < 5; i++) be_flag(&e->hdr, 0); /* no deltas */
    be_lit(&e->hdr, 1, 0);               /* refresh entropy probs */
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++)
                for (int p = 0; p < 11; p++) {
                    uint8_t oldp = e->probs[t][b][c][p];
                    int up = e->have_updated && e->updated[t][b][c][p] != oldp;
                    if (up) {
                        be_bool(&e->hdr, 1, COEFF_UPDATE_PROBS[t][b][c][p]);
                        be_lit(&e->hdr, 8, e->updated[t][b][c][p]);
                        e->probs[t][b][c][p] = e->updated[t][b][c][p];
                    } else {
                        be_bool(&e->hdr, 0, COEFF_UPDATE_PROBS[t][b][c][p]);
                    }
                }
    e->have_updated = 0;
    be_lit(&e->hdr, 1, 1);
    be_lit(&e->hdr, 8, e->skip_prob);
    if (dbg) memcpy(dbg->final_probs, e->probs, sizeof e->probs);

    /* ---------------- PASS 2 ---------------- */
    e->pass = 2;
    for (int mby = 0; mby < e->mbh; mby++) {
        reset_row(e);
        memset(e->left_derr, 0, sizeof e->left_derr);
        e->part = &e->parts[mby % e->nparts];
        for (int mbx = 0; mbx < e->mbw; mbx++) {
            mbinfo_t mi;
            choose_mb(e, mbx, mby, &mi);
            transform_luma(e, mbx, mby, &mi, lb);
            transform_chroma(e, mbx, mby, mi.chroma_mode, ub, vb);
            mi.skipped = all_zero(e, &mi, lb, ub, vb);
            write_mb_header(e, &mi, mbx);
            int32_t *lv = (dbg && dbg->levels) ? dbg->levels + (size_t)(mby * e->mbw + mbx) * 25 * 16 : NULL;
            if (lv) memset(lv, 0, 25 * 16 * sizeof(int32_t));
            if (!mi.skipped) {
                encode_residual(e, &mi, mbx, lb, ub, vb, lv);
            } else {
                cplx_clear(&e->left_c, mi.luma_mode != 4);
                cplx_clear(&e->top_c[mbx], mi.luma_mode != 4);
            }
            if (dbg && dbg->p2_info) {
                or_mb_info *o = &dbg->p2_info[mby * e->mbw + mbx];
                o->luma_mode = (uint8_t)mi.luma_mode;
                memcpy(o->bpred, mi.bpred, 16);
                o->chroma_mode = (uint8_t)mi.chroma_mode;
                o->segment = (uint8_t)(mi.segment_id < 0 ? 0 : mi.segment_id);
                o->skip = (uint8_t)mi.skipped;
            }
        }
    }
    be_flush(&e->hdr);
    size_t plen = 0;
    for (int p = 0; p < e->nparts; p++) {
        be_flush(&e->parts[p]);
        plen += e->parts[p].len;
    }

    /* write_uncompressed_frame_header vp8.rs:315-330 + partitions */
    size_t total = 10 + e->hdr.len + 3 * (size_t)(e->nparts - 1) + plen;
    uint8_t *o = (uint8_t *)malloc(total);
    uint32_t tag = ((uint32_t)e->hdr.len << 5) | (1u << 4);
    o[0] = (uint8_t)tag; o[1] = (uint8_t)(tag >> 8); o[2] = (uint8_t)(tag >> 16);
    o[3] = 0x9d; o[4] = 0x01; o[5] = 0x2a;
    o[6] = (uint8_t)(width & 0xff); o[7] = (uint8_t)((width >> 8) & 0x3f);
    o[8] = (uint8_t)(height & 0xff); o[9] = (uint8_t)((height >> 8) & 0x3f);
    memcpy(o + 10, e->hdr.buf, e->hdr.len);
    size_t w = 10 + e->hdr.len;
    for (int p = 0; p + 1 < e->nparts; p++, w += 3) {
        o[w] = (uint8_t)e->parts[p].len; o[w + 1] = (uint8_t)(e->parts[p].len >> 8); o[w + 2] = (uint8_t)(e->parts[p].len >> 16);
    }
    for (int p = 0; p < e->nparts; p++) {
        memcpy(o + w, e->parts[p].buf, e->parts[p].len);
        w += e->parts[p].len;
    }
    *out = o;
    *out_len = total;

    free(e->hdr.buf);
    for (int p = 0; p < e->nparts; p++) free(e->parts[p].buf);
    free(e->Y); free(e->U); free(e->V);
    free(e->top_c); free(e->top_bpred); free(e->seg_map);
    free(e->top_y); free(e->top_u); free(e->top_v); free(e->top_derr);
    return OR_OK;
}

/* ---- small KAT helpers exposed for tests ---- */
int or_bool_encoder_kat(const int *ops, int nops, uint8_t *out, int out_cap)
{
    /* ops: triples (kind, a, b): kind 0 = bool(a, prob b), 1 = literal(nbits a, value b),
     * 2 = flag(a), 3 = optional signed (nbits a, value b or 0x7fff = None), 4 = ymode tree (value a) */
    benc_t e;
    be_init(&e);
    for (int i = 0; i < nops; i++) {
        int k = ops[3 * i], a = ops[3 * i + 1], b = ops[3 * i + 2];
        if (k == 0) be_bool(&e, a, b);
        else if (k == 1) be_lit(&e, a, b);
        else if (k == 2) be_flag(&e, a);
        else if (k == 3) {
            be_flag(&e, b != 0x7fff);
            if (b != 0x7fff) {
                be_lit(&e, a, b < 0 ? -b : b);
                be_flag(&e, b >= 0);
            }
        } else if (k == 4) be_tree(&e, YMODE_TREE, 8, KEYFRAME_YMODE_PROBS, a, 0);
    }
    be_flush(&e);
    int n = (int)e.len;
    if (n > out_cap) n = out_cap;
    memcpy(out, e.buf, (size_t)n);
    free(e.buf);
    return (int)e.len;
}

int or_trellis_kat(const int32_t coeffs_in[16], int q_dc, int q_ac, int iq_dc, int iq_ac, uint32_t lambda,
                   int ctype, int first, int ctx0, int use_default_costs, int32_t out_levels[16], int32_t out_coeffs[16])
{
    mtx_t m;
    mtx_init(&m, q_dc, q_ac, ctype == 3 || ctype == 0 ? 0 : (ctype == 1 ? 1 : 2));
    (void)iq_dc; (void)iq_ac;
    lcost_t L;
    memset(&L, 0, sizeof L);
    if (use_default_costs) lcost_calc(&L, COEFF_PROBS);
    int32_t c[16];
    memcpy(c, coeffs_in, sizeof c);
    int nz = trellis(c, out_levels, &m, lambda, first, &L, ctype, ctx0);
    memcpy(out_coeffs, c, sizeof c);
    return nz;
}

/* Batch form of quantize_coeff / trellis_quantize_block, same contract as the
 * product's zw_quant_blocks (levels zigzag, dequantised natural). */
void or_quant_blocks_c(int n, const int32_t *coeffs, const uint8_t *ctx0, int ctype, int first, int use_trellis,
                       uint32_t lambda, int q_dc, int q_ac, int matrix_type, const uint8_t *probs, int32_t *levels,
                       int32_t *dq_out)
{
    mtx_t m;
    mtx_init(&m, q_dc, q_ac, matrix_type);
    lcost_t *L = (lcost_t *)malloc(sizeof(lcost_t));
    lcost_calc(L, probs ? (const uint8_t(*)[8][3][11])probs : COEFF_PROBS);
    for (int b = 0; b < n; b++) {
        int32_t c[16], lv[16] = {0};
        memcpy(c, coeffs + 16 * b, sizeof c);
        if (use_trellis) {
            trellis(c, lv, &m, lambda, first, L, ctype, ctx0[b]);
        } else {
            for (int k = 0; k < 16; k++) {
                int j = ZIGZAG[k];
                lv[k] = k < first ? 0 : quant(&m, c[j], j);
            }
            for (int k = 0; k < 16; k++) {
                int j = ZIGZAG[k];
                c[j] = k < first ? 0 : dequant(&m, lv[k], j);
            }
        }
        memcpy(levels + 16 * b, lv, sizeof lv);
        memcpy(dq_out + 16 * b, c, sizeof c);
    }
    free(L);
}

uint32_t or_fixed_cost_i16(int mode) { return FIXED_COSTS_I16[mode]; }
uint32_t or_fixed_cost_uv(int mode) { return FIXED_COSTS_UV[mode]; }
int or_filter_level_for_quality(int quality) { return compute_filter_level(or_quality_to_quant_index(quality), 0, 50); }

/* ======================================================================== */
/* Known-answer-test entry points (tests/test_oracle.py pins these against  */
/* the reference's own in-crate tests).                                     */
/* ======================================================================== */
float or_fm_roundf(float x) { return (float)(int32_t)(x + 0.5f); } /* fast_math.rs:8 */
double or_fm_round(double x) { return fm_round(x); }
double or_fm_cbrt(double x) { return fm_cbrt(x); }
double or_fm_pow(double x, double n) { return fm_pow(x, n); }
uint64_t or_rd_score(uint32_t sse, uint32_t rate, uint32_t lambda) { return rd_score(sse, (uint16_t)rate, lambda); }
int or_t_transform(const uint8_t *in, int stride, const uint16_t w[16]) { return t_xform(in, stride, w); }
/* Segment::init_matrices with every quantizer = q (so qi4 = qi16 = quv = q):
 * out = {l_i4, l_i16, l_uv, l_mode, lt_i4, lt_i16, lt_uv, tlambda} */
void or_seg_lambdas(uint32_t q, uint32_t out[8])
{
    seg_t s;
    memset(&s, 0, sizeof s);
    s.ydc = s.yac = s.y2dc = s.y2ac = s.uvdc = s.uvac = (int16_t)q;
    seg_init(&s);
    const uint32_t v[8] = {s.l_i4, s.l_i16, s.l_uv, s.l_mode, s.lt_i4, s.lt_i16, s.lt_uv, s.tlambda};
    memcpy(out, v, sizeof v);
}
/* calc_i4_penalty (cost.rs:341-343): max(1000 q^2, 1).  Not on the encode
 * path (the reference never calls it outside its test, cost.rs:2110-2119);
 * restated only so the KAT pins the formula. */
uint64_t or_i4_penalty(uint32_t q)
{
    const uint64_t p = 1000ull * q * q;
    return p > 1 ? p : 1;
}
/* rd_score_with_coeffs (cost.rs:1108-1112): sse * 256 + (mode + coeff) * lambda.
 * Also off the path (used only by its test, cost.rs:2210-2223). */
uint64_t or_rd_score_with_coeffs(uint32_t sse, uint32_t mode_cost, uint32_t coeff_cost, uint32_t lambda)
{
    return (uint64_t)sse * 256u + ((uint64_t)(uint16_t)mode_cost + coeff_cost) * lambda;
}
/* VP8_ENC_BANDS (tables.rs), the band of zigzag position n (n = 16: the eob sentinel) */
int or_enc_band(int n) { return VP8_ENC_BANDS[n]; }
/* add_residue (prediction.rs:138) on a 4x4 block of stride 4 */
void or_add_residue_kat(uint8_t pblock[16], const int32_t r[16]) { or_add_residue(pblock, r, 0, 0, 4); }

/* ======================================================================== */
/* Streaming final transform over explicit per-MB records (the arithmetic of  */
/* transform_luma_block vp8.rs:2647-2780 with do_trellis off, of              */
/* transform_luma_blocks_4x4 :2785-2916 and of transform_chroma_blocks        */
/* :3039-3121 with apply_chroma_error_diffusion :572-647).  Every input the   */
/* encoder would take from its running state (the borders create_border_luma */
/* / create_border_chroma build, prediction.rs:15-130, and the incoming       */
/* top/left error-diffusion terms) comes from the MB's 96-byte record instead */
/* (layout in include/zwebp.h, zw_transform_quant_mbs), so MBs are            */
/* independent.  Checker for the device kernel k_xform_mb.                    */
/* ======================================================================== */
static void xmb_luma_ws(const uint8_t *r, uint8_t ws[OR_LUMA_WS])
{
    memset(ws, 0, OR_LUMA_WS);
    ws[0] = r[20];
    for (int i = 0; i < 20; i++) ws[1 + i] = r[24 + i];
    for (int i = 17; i < 21; i++) ws[4 * OR_BPS + i] = ws[8 * OR_BPS + i] = ws[12 * OR_BPS + i] = ws[i];
    for (int i = 0; i < 16; i++) ws[(i + 1) * OR_BPS] = r[44 + i];
}
static void xmb_chroma_ws(const uint8_t *r, int plane, uint8_t ws[OR_CHROMA_WS])
{
    memset(ws, 0, OR_CHROMA_WS);
    ws[0] = r[21 + plane];
    for (int i = 0; i < 8; i++) ws[1 + i] = r[64 + 16 * plane + i];
    for (int i = 0; i < 8; i++) ws[(i + 1) * OR_BPS] = r[72 + 16 * plane + i];
}
static void xmb_put_levels(int16_t *out, const int32_t *lvl)
{
    for (int n = 0; n < 16; n++) out[n] = (int16_t)lvl[ZIGZAG[n]];
}

void or_xform_mbs(int nframes, int mbw, int mbh, const uint8_t *Y, const uint8_t *U, const uint8_t *V,
                  const uint8_t *recs, const int32_t *seg_qi, int16_t *levels, uint8_t *RY, uint8_t *RU, uint8_t *RV)
{
    const int ys = mbw * 16, cs = mbw * 8, nmb = mbw * mbh;
    const size_t ysz = (size_t)ys * mbh * 16, csz = (size_t)cs * mbh * 8;
    for (int f = 0; f < nframes; f++) {
        seg_t seg[4];
        for (int i = 0; i < 4; i++) seg_from_index(&seg[i], seg_qi[f * 4 + i], 0);
        const uint8_t *Yf = Y + f * ysz, *Uf = U + f * csz, *Vf = V + f * csz;
        uint8_t *RYf = RY + f * ysz, *RUf = RU + f * csz, *RVf = RV + f * csz;
        for (int mb = 0; mb < nmb; mb++) {
            const int mbx = mb % mbw, mby = mb / mbw;
            const uint8_t *r = recs + ((size_t)f * nmb + mb) * 96;
            int16_t *out = levels + ((size_t)f * nmb + mb) * 25 * 16;
            const seg_t *s = &seg[r[2] & 3];
            const int has_top = r[3] & 1, has_left = (r[3] >> 1) & 1;
            uint8_t ws[OR_LUMA_WS];
            int32_t lvl[16];
            xmb_luma_ws(r, ws);
            const uint8_t *src = Yf + (size_t)mby * 16 * ys + mbx * 16;
            if (r[0] != 4) {
                switch (r[0]) {
                case 1: or_pred_v(ws, 16, 1, 1, OR_BPS); break;
                case 2: or_pred_h(ws, 16, 1, 1, OR_BPS); break;
                case 3: or_pred_tm(ws, 16, 1, 1, OR_BPS); break;
                default: or_pred_dc(ws, 16, OR_BPS, has_top, has_left); break;
                }
                int32_t lb[256], c0[16], y2d[16];
                for (int by = 0; by < 4; by++)
                    for (int bx = 0; bx < 4; bx++)
                        fdct_res(src + by * 4 * ys + bx * 4, ys, ws + (by * 4 + 1) * OR_BPS + bx * 4 + 1, OR_BPS,
                                 lb + (by * 4 + bx) * 16);
                for (int i = 0; i < 16; i++) c0[i] = lb[i * 16];
                or_wht(c0);
                for (int i = 0; i < 16; i++) {
                    c0[i] = quant(&s->y2, c0[i], i);
                    y2d[i] = dequant(&s->y2, c0[i], i);
                }
                xmb_put_levels(out + 16 * 16, c0);
                or_iwht(y2d);
                for (int i = 0; i < 16; i++) {
                    int32_t *blk = lb + i * 16;
                    lvl[0] = 0;
                    for (int k = 1; k < 16; k++) {
                        lvl[k] = quant(&s->y1, blk[k], k);
                        blk[k] = dequant(&s->y1, lvl[k], k);
                    }
                    xmb_put_levels(out + i * 16, lvl);
                    blk[0] = y2d[i];
                    or_idct(blk);
                    or_add_residue(ws, blk, 1 + (i / 4) * 4, 1 + (i % 4) * 4, OR_BPS);
                }
            } else {
                for (int i = 0; i < 16; i++) out[16 * 16 + i] = 0;
                for (int i = 0; i < 16; i++) {
                    const int sby = i / 4, sbx = i % 4, y0 = sby * 4 + 1, x0 = sbx * 4 + 1;
                    const int mode = (r[4 + i / 2] >> (4 * (i & 1))) & 15;
                    or_pred_b(ws, mode, x0, y0, OR_BPS);
                    int32_t cur[16];
                    fdct_res(src + sby * 4 * ys + sbx * 4, ys, ws + y0 * OR_BPS + x0, OR_BPS, cur);
                    for (int k = 0; k < 16; k++) {
                        lvl[k] = quant(&s->y1, cur[k], k);
                        cur[k] = dequant(&s->y1, lvl[k], k);
                    }
                    xmb_put_levels(out + i * 16, lvl);
                    or_idct(cur);
                    or_add_residue(ws, cur, y0, x0, OR_BPS);
                }
            }
            store_recon(NULL, ws, 16, OR_BPS, RYf, ys, mbx * 16, mby * 16);
            for (int plane = 0; plane < 2; plane++) {
                uint8_t cw[OR_CHROMA_WS];
                xmb_chroma_ws(r, plane, cw);
                switch (r[1]) {
                case 1: or_pred_v(cw, 8, 1, 1, OR_BPS); break;
                case 2: or_pred_h(cw, 8, 1, 1, OR_BPS); break;
                case 3: or_pred_tm(cw, 8, 1, 1, OR_BPS); break;
                default: or_pred_dc(cw, 8, OR_BPS, has_top, has_left); break;
                }
                const uint8_t *P = plane ? Vf : Uf;
                int32_t cb[64];
                for (int by = 0; by < 2; by++)
                    for (int bx = 0; bx < 2; bx++)
                        fdct_res(P + (size_t)(mby * 8 + by * 4) * cs + mbx * 8 + bx * 4, cs,
                                 cw + (by * 4 + 1) * OR_BPS + bx * 4 + 1, OR_BPS, cb + (by * 2 + bx) * 16);
                /* apply_chroma_error_diffusion: incoming top/left terms from the record */
                const int8_t *d = (const int8_t *)r + 12 + 4 * plane;
                int8_t e0 = diffuse(&cb[0], d[0], d[2], &s->uv);
                int8_t e1 = diffuse(&cb[16], d[1], e0, &s->uv);
                int8_t e2 = diffuse(&cb[32], e0, d[3], &s->uv);
                (void)diffuse(&cb[48], e1, e2, &s->uv);
                for (int b = 0; b < 4; b++) {
                    int32_t *blk = cb + b * 16;
                    for (int k = 0; k < 16; k++) {
                        lvl[k] = quant(&s->uv, blk[k], k);
                        blk[k] = dequant(&s->uv, lvl[k], k);
                    }
                    xmb_put_levels(out + (17 + 4 * plane + b) * 16, lvl);
                    or_idct(blk);
                    or_add_residue(cw, blk, 1 + (b / 2) * 4, 1 + (b % 2) * 4, OR_BPS);
                }
                store_recon(NULL, cw, 8, OR_BPS, plane ? RVf : RUf, cs, mbx * 8, mby * 8);
            }
        }
    }
}
