// zw_host_entropy.h -- host half of the encoder: the sequential boolean coder
// stays on the CPU (north star).  Restates, for the product path:
//   ArithmeticEncoder               encoder/arithmetic.rs:7-196
//   record_coeffs / ProbaStats      encoder/cost.rs:1173-1397
//   compute_updated_probabilities   encoder/vp8.rs:1202-1238
//   LevelCosts::calculate           encoder/cost.rs:1500-1545
//   encode_coefficients / residuals encoder/vp8.rs:650-958
//   headers                         encoder/vp8.rs:315-560
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <immintrin.h>
#include <algorithm>
#include <memory>
#include <vector>
#include "zw_common.h"

namespace zwh {

#define ZW_TABLE(T, N, D, ...) static const T N D = {__VA_ARGS__};
#include "zw_tables.inc"
#undef ZW_TABLE

static const int8_t SEGMENT_ID_TREE[6] = {2, 4, -0, -1, -2, -3};
static const int8_t YMODE_TREE[8] = {-4, 2, 4, 6, -0, -1, -2, -3};
static const int8_t BMODE_TREE[18] = {-0, 2, -1, 4, -2, 6, 8, 12, -3, 10, -5, -6, -4, 14, -7, 16, -8, -9};
static const int8_t UVMODE_TREE[6] = {-0, 2, -1, 4, -2, -3};
static const int8_t TOKEN_TREE[22] = {-11, 2, -0, 4, -1, 6, 8, 12, -2, 10, -3, -4,
                                      14, 16, -5, -6, 18, 20, -7, -8, -9, -10};

// ArithmeticEncoder (arithmetic.rs:7-196).  The reference renormalises one bit
// per loop iteration; here all `shift` bits of one renormalisation are taken
// at once (the same arithmetic in libvpx's batched form: `count` = -bit_num,
// `low` = bottom), with the carry into already-written bytes propagated as the
// reference's add_one does.  Byte-identical output (tests/test_host_entropy.py
// drives both forms over random decision streams).
struct BoolEncoder {
    std::vector<uint8_t> buf;
    uint32_t low = 0, range = 255;
    int count = -24;  // = -bit_num

    BoolEncoder() { buf.reserve(1 << 16); }
    void add_one()
    {
        size_t i = buf.size();
        while (i > 0) {
            i--;
            if (buf[i] < 255) {
                buf[i]++;
                return;
            }
            buf[i] = 0;
        }
        buf.insert(buf.begin(), 1);
    }
    inline void put(int bit, int prob)
    {
        const uint32_t split = 1 + (((range - 1) * (uint32_t)prob) >> 8);
        // branch-free: the coded bits are by construction unpredictable
        const uint32_t m = 0u - (uint32_t)(bit != 0);
        low += split & m;
        const uint32_t r = split ^ ((split ^ (range - split)) & m);
        // renormalise: range back to [128, 255]
        const int shift = __builtin_clz(r) - 24;
        range = r << shift;
        count += shift;
        if (count >= 0) {  // a byte is complete after `offset` of the shifts
            const int offset = shift - count;
            if ((low << (offset - 1)) & 0x80000000u) add_one();
            buf.push_back((uint8_t)(low >> (24 - offset)));
            low = (low << offset) & 0xffffffu;
            low <<= count;
            count -= 8;
        } else {
            low <<= shift;
        }
    }
    void flag(int f) { put(f, 128); }
    void literal(int nbits, int v)
    {
        for (int b = nbits - 1; b >= 0; b--) put(((1 << b) & v) > 0, 128);
    }
    void tree(const int8_t* t, int tlen, const uint8_t* probs, int value, int start = 0);
    // a precomputed tree path: n bits, MSB-first bits / probability indices
    inline void path(const uint8_t* bits, const uint8_t* pidx, int n, const uint8_t* probs)
    {
        for (int i = 0; i < n; i++) put(bits[i], probs[pidx[i]]);
    }
    void flush()  // the reference's flush (arithmetic.rs:176-196) on its state (bottom, bit_num)
    {
        const int bit_num = -count;
        int c = bit_num;
        uint32_t v = low;
        if (low & (1u << (32 - bit_num))) add_one();
        v <<= (c & 7);
        c = (c >> 3) - 1;
        while (c >= 0) {
            v <<= 8;
            c--;
        }
        for (c = 3; c >= 0; c--) {
            buf.push_back((uint8_t)(v >> 24));
            v <<= 8;
        }
    }
};

// The reference's bit-at-a-time form, kept for the equivalence test only.
struct BoolEncoderRef {
    std::vector<uint8_t> buf;
    uint32_t bottom = 0, range = 255;
    int bit_num = 24;
    void add_one()
    {
        size_t i = buf.size();
        while (i > 0) {
            i--;
            if (buf[i] < 255) {
                buf[i]++;
                return;
            }
            buf[i] = 0;
        }
        buf.insert(buf.begin(), 1);
    }
    void put(int bit, int prob)
    {
        uint32_t split = 1 + (((range - 1) * (uint32_t)prob) >> 8);
        if (bit) {
            bottom += split;
            range -= split;
        } else {
            range = split;
        }
        while (range < 128) {
            range <<= 1;
            if (bottom & (1u << 31)) add_one();
            bottom <<= 1;
            if (--bit_num == 0) {
                buf.push_back((uint8_t)(bottom >> 24));
                bottom &= (1u << 24) - 1;
                bit_num = 8;
            }
        }
    }
    void flush()
    {
        int c = bit_num;
        uint32_t v = bottom;
        if (bottom & (1u << (32 - bit_num))) add_one();
        v <<= (c & 7);
        c = (c >> 3) - 1;
        while (c >= 0) { v <<= 8; c--; }
        for (c = 3; c >= 0; c--) { buf.push_back((uint8_t)(v >> 24)); v <<= 8; }
    }
};

// Path of `value` through a VP8 tree (write_with_tree_start_index,
// arithmetic.rs:120): bits root-first and the probability index of each.
inline int tree_path(const int8_t* t, int tlen, int value, int start, uint8_t* bits, uint8_t* pidx)
{
    int cur = -1;
    for (int i = 0; i < tlen; i++)
        if (t[i] == -value) { cur = i; break; }
    int enc[16], pr[16], cnt = 0;
    for (;;) {
        if (cur == start) { enc[cnt] = 0; pr[cnt++] = cur / 2; break; }
        if (cur == start + 1) { enc[cnt] = 1; pr[cnt++] = cur / 2; break; }
        int ev = 0;
        if (cur % 2) { cur -= 1; ev = 1; }
        enc[cnt] = ev;
        pr[cnt++] = cur / 2;
        int pi = -1;
        for (int i = 0; i < tlen; i++)
            if (t[i] == cur) { pi = i; break; }
        cur = pi;
    }
    for (int i = 0; i < cnt; i++) {
        bits[i] = (uint8_t)enc[cnt - 1 - i];
        pidx[i] = (uint8_t)pr[cnt - 1 - i];
    }
    return cnt;
}

inline void BoolEncoder::tree(const int8_t* t, int tlen, const uint8_t* probs, int value, int start)
{
    uint8_t bits[16], pidx[16];
    const int n = tree_path(t, tlen, value, start, bits, pidx);
    path(bits, pidx, n, probs);
}

// Precomputed paths of the mode trees (the per-MB header symbols).
struct TreePaths {
    uint8_t n[10], bits[10][16], pidx[10][16];
    TreePaths(const int8_t* t, int tlen, int nsym)
    {
        for (int v = 0; v < nsym; v++) n[v] = (uint8_t)tree_path(t, tlen, v, 0, bits[v], pidx[v]);
    }
    template <class Enc>
    void put(Enc& E, const uint8_t* probs, int v) const
    {
        E.path(bits[v], pidx[v], n[v], probs);
    }
};

// TOKEN_TREE paths for tokens 0..11 from start index 0 / 2 (after a zero token)
struct TokenPaths {
    uint8_t n[2][12], bits[2][12][12], pidx[2][12][12];
    TokenPaths()
    {
        for (int s = 0; s < 2; s++)
            for (int v = 0; v < 12; v++) n[s][v] = (uint8_t)tree_path(TOKEN_TREE, 22, v, 2 * s, bits[s][v], pidx[s][v]);
    }
};
inline const TokenPaths& token_paths()
{
    static const TokenPaths P;
    return P;
}

inline uint16_t bitcost(int bit, int p) { return bit ? VP8_ENTROPY_COST[255 - p] : VP8_ENTROPY_COST[p]; }

// Packed MB record view (zw_pack_kernels.hip): header, sub-modes, eobs and a
// pointer to each block's zigzag levels (little-endian i16, eob of them).
struct PackedMb {
    int luma, skip, segment, chroma;
    uint8_t bpred[16];
    const uint8_t* eob;
    const uint8_t* lv[25];
};
inline const uint8_t* view_mb(const uint8_t* p, PackedMb& m)
{
    const uint8_t h = p[0];
    m.luma = h & 7;
    m.skip = (h >> 3) & 1;
    m.segment = (h >> 4) & 3;
    m.chroma = h >> 6;
    p++;
    if (m.luma == 4) {
        for (int i = 0; i < 8; i++) {
            m.bpred[2 * i] = p[i] & 15;
            m.bpred[2 * i + 1] = p[i] >> 4;
        }
        p += 8;
    }
    m.eob = p;
    p += 25;
    for (int b = 0; b < 25; b++) {
        m.lv[b] = p;
        p += 2 * m.eob[b];
    }
    return p;
}
inline int lv_at(const uint8_t* lv, int n) { return (int)(int16_t)(uint16_t)(lv[2 * n] | (lv[2 * n + 1] << 8)); }

// LevelCosts::calculate (cost.rs:1500)
inline void level_costs(ZwLevelCosts& L, const uint8_t probs[4][8][3][11])
{
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++) {
                const uint8_t* p = probs[t][b][c];
                uint16_t cost0 = c > 0 ? bitcost(1, p[0]) : 0;
                uint16_t base = (uint16_t)(bitcost(1, p[1]) + cost0);
                L.lc[t][b][c][0] = (uint16_t)(bitcost(0, p[1]) + cost0);
                for (int v = 1; v <= 67; v++) {
                    int idx = (v < 67 ? v : 67) - 1;
                    int pat = VP8_LEVEL_CODES[idx][0], bits = VP8_LEVEL_CODES[idx][1];
                    uint16_t vc = 0;
                    for (int i = 2; pat; i++) {
                        if (pat & 1) vc = (uint16_t)(vc + bitcost(bits & 1, p[i]));
                        bits >>= 1;
                        pat >>= 1;
                    }
                    L.lc[t][b][c][v] = (uint16_t)(base + vc);
                }
                L.eob[t][b][c] = bitcost(0, p[0]);
                L.init[t][b][c] = bitcost(1, p[0]);
            }
}

struct Stats {
    uint32_t s[4][8][3][11];
};

inline void rec_stat(uint32_t& s, int bit)
{
    if (s >= 0xfffe0000u) s = ((s + 1) >> 1) & 0x7fff7fffu;
    s += 0x00010000u + (bit ? 1u : 0u);
}

inline int token_of(int a)  // |level| -> token (0..10)
{
    return a <= 4 ? a : (a <= 6 ? 5 : a <= 10 ? 6 : a <= 18 ? 7 : a <= 34 ? 8 : a <= 66 ? 9 : 10);
}

// record_coeffs (cost.rs:1297) over a packed block: eob = last nonzero + 1,
// lv = its zigzag levels.  (The branchy form measured faster than walking the
// token paths: most tokens are 0 / 1 and predict well.)  Quirk
// (cost.rs:1325-1342): skip_eob is never cleared once a zero token was seen.
inline void record_coeffs(Stats& S, const uint8_t* lv, int eob, int t, int first, int ctx)
{
    if (eob <= first) {
        rec_stat(S.s[t][VP8_ENC_BANDS[first]][ctx][0], 0);
        return;
    }
    int n = first, skip_eob = 0;
    while (n < eob) {
        uint32_t* st = S.s[t][VP8_ENC_BANDS[n]][ctx];
        const int c = lv_at(lv, n);
        int v = c < 0 ? -c : c;
        n++;
        if (!skip_eob) rec_stat(st[0], 1);
        if (v == 0) {
            rec_stat(st[1], 0);
            skip_eob = 1;
            ctx = 0;
            continue;
        }
        rec_stat(st[1], 1);
        if (v == 1) {
            rec_stat(st[2], 0);
            ctx = 1;
        } else {
            rec_stat(st[2], 1);
            if (v > 67) v = 67;
            if (v <= 4) {
                rec_stat(st[3], 0);
                if (v == 2) rec_stat(st[4], 0);
                else {
                    rec_stat(st[4], 1);
                    rec_stat(st[5], v == 4);
                }
            } else if (v <= 10) {
                rec_stat(st[3], 1);
                rec_stat(st[6], 0);
                rec_stat(st[7], v > 6);
            } else {
                rec_stat(st[3], 1);
                rec_stat(st[6], 1);
                if (v < 3 + (8 << 2)) {
                    rec_stat(st[8], 0);
                    rec_stat(st[9], v >= 3 + (8 << 1));
                } else {
                    rec_stat(st[8], 1);
                    rec_stat(st[10], v >= 3 + (8 << 3));
                }
            }
            ctx = 2;
        }
    }
    if (n < 16) rec_stat(S.s[t][VP8_ENC_BANDS[n]][ctx][0], 0);
}

struct Cplx {
    uint8_t y2, y[4], u[2], v[2];
    void clear(bool with_y2)
    {
        memset(y, 0, 4);
        memset(u, 0, 2);
        memset(v, 0, 2);
        if (with_y2) y2 = 0;
    }
};

// check_all_coeffs_zero on pass-1 (simple-quant) levels: a block has a
// nonzero at index >= first exactly when its eob > first.
inline bool mb_all_zero_p1(const PackedMb& m)
{
    const bool i4 = m.luma == 4;
    if (!i4 && m.eob[16] > 0) return false;
    const int first = i4 ? 0 : 1;
    for (int b = 0; b < 16; b++)
        if (m.eob[b] > first) return false;
    for (int b = 17; b < 25; b++)
        if (m.eob[b] > 0) return false;
    return true;
}

// Skip probability from the MB counts (vp8.rs:1387-1394).
inline int skip_prob(uint32_t total, uint32_t ns)
{
    uint32_t p = (255 * ns + total / 2) / total;
    if (p > 255) p = 255;
    int sp = (int)(uint8_t)p;
    return sp < 1 ? 1 : (sp > 254 ? 254 : sp);
}

// Pass-1 statistics replay in raster order (vp8.rs:1337-1385 + record_residual_stats :1027).
// Returns the skip probability.
inline int replay_stats(Stats& S, const uint8_t* packed, int mbw, int mbh)
{
    PackedMb m;
    memset(&S, 0, sizeof S);
    std::vector<Cplx> top(mbw);
    memset(top.data(), 0, sizeof(Cplx) * mbw);
    uint32_t total = 0, skipped = 0;
    for (int y = 0; y < mbh; y++) {
        Cplx left;
        memset(&left, 0, sizeof left);
        for (int x = 0; x < mbw; x++) {
            packed = view_mb(packed, m);
            total++;
            const bool i4 = m.luma == 4;
            if (mb_all_zero_p1(m)) {
                skipped++;
                left.clear(!i4);
                top[x].clear(!i4);
                continue;
            }
            if (!i4) {
                int cx = left.y2 + top[x].y2;
                record_coeffs(S, m.lv[16], m.eob[16], 1, 0, cx < 2 ? cx : 2);
                left.y2 = top[x].y2 = m.eob[16] > 0;
            }
            const int tt = i4 ? 3 : 0, first = i4 ? 0 : 1;
            for (int by = 0; by < 4; by++) {
                int l = left.y[by];
                for (int bx = 0; bx < 4; bx++) {
                    int cx = l + top[x].y[bx];
                    const int b = by * 4 + bx;
                    record_coeffs(S, m.lv[b], m.eob[b], tt, first, cx < 2 ? cx : 2);
                    l = m.eob[b] > first;
                    top[x].y[bx] = (uint8_t)l;
                }
                left.y[by] = (uint8_t)l;
            }
            for (int pl = 0; pl < 2; pl++) {
                uint8_t* lc = pl ? left.v : left.u;
                uint8_t* tc = pl ? top[x].v : top[x].u;
                for (int by = 0; by < 2; by++) {
                    int l = lc[by];
                    for (int bx = 0; bx < 2; bx++) {
                        int cx = l + tc[bx];
                        const int b = 17 + 4 * pl + by * 2 + bx;
                        record_coeffs(S, m.lv[b], m.eob[b], 2, 0, cx < 2 ? cx : 2);
                        l = m.eob[b] > 0;
                        tc[bx] = (uint8_t)l;
                    }
                    lc[by] = (uint8_t)l;
                }
            }
        }
    }
    return skip_prob(total, total - skipped);
}

// compute_updated_probabilities (vp8.rs:1202); returns whether any update applies.
inline bool updated_probs(const Stats& S, uint8_t out[4][8][3][11])
{
    memcpy(out, COEFF_PROBS, sizeof(COEFF_PROBS));
    int32_t total = 0;
    uint32_t nup = 0;
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++)
                for (int p = 0; p < 11; p++) {
                    uint32_t st = S.s[t][b][c][p];
                    int nb = (int)(st & 0xffff), tot = (int)(st >> 16);
                    if (tot == 0) continue;
                    uint8_t oldp = COEFF_PROBS[t][b][c][p], upp = COEFF_UPDATE_PROBS[t][b][c][p];
                    uint8_t newp = (uint8_t)(255 - (uint32_t)nb * 255 / (uint32_t)tot);
                    int oc = nb * VP8_ENTROPY_COST[255 - oldp] + (tot - nb) * VP8_ENTROPY_COST[oldp] + bitcost(0, upp);
                    int nc = nb * VP8_ENTROPY_COST[255 - newp] + (tot - nb) * VP8_ENTROPY_COST[newp] + bitcost(1, upp) + 8 * 256;
                    int sav = oc - nc;
                    if (sav > 0) {
                        out[t][b][c][p] = newp;
                        total += sav;
                        nup++;
                    }
                }
    if (!(total > 0 && nup > 0)) {
        memcpy(out, COEFF_PROBS, sizeof(COEFF_PROBS));
        return false;
    }
    return true;
}

// encode_coefficients token part (vp8.rs:845-958) for an already-quantized
// packed block (eob = last nonzero + 1).
template <class Enc>
inline int emit_block(Enc& E, const uint8_t (*P)[3][11], const uint8_t* lv, int eobi, int first, int ctx)
{
    const TokenPaths& TP = token_paths();
    int skip_eob = 0;
    for (int idx = first; idx < eobi; idx++) {
        const int coeff = lv_at(lv, idx);
        const uint8_t* pr = P[COEFF_BANDS[idx]][ctx];
        const int a = coeff < 0 ? -coeff : coeff;
        const int token = token_of(a);
        E.path(TP.bits[skip_eob][token], TP.pidx[skip_eob][token], TP.n[skip_eob][token], pr);
        if (token >= 5) {
            const int cat = token;
            const uint8_t* cp = PROB_DCT_CAT[cat - 5];
            int extra = a - DCT_CAT_BASE[cat - 5];
            int mask = cat == 10 ? 1 << 10 : 1 << (cat - 5);
            for (int k = 0; k < 12 && cp[k]; k++) {
                E.put((extra & mask) > 0, cp[k]);
                mask >>= 1;
            }
        }
        skip_eob = token == 0;
        if (token != 0) E.flag(!(coeff > 0));
        ctx = token == 0 ? 0 : (token == 1 ? 1 : 2);
    }
    if (eobi < 16) {
        int bi = first > eobi ? first : eobi;
        E.path(TP.bits[0][11], TP.pidx[0][11], TP.n[0][11], P[COEFF_BANDS[bi]][ctx]);
    }
    return eobi > 0;
}

// Compressed frame header (encode_compressed_frame_header vp8.rs:332-372) with
// log2(nparts) token partitions; `probs` leaves with the probabilities in force.
template <class Enc>
inline void emit_frame_header(Enc& H, const ZwFrameParams& P, bool have_updated,
                              const uint8_t upd[4][8][3][11], int nparts, uint8_t probs[4][8][3][11])
{
    memcpy(probs, COEFF_PROBS, sizeof(COEFF_PROBS));
    H.literal(1, 0);
    H.literal(1, 0);
    H.flag(P.seg_enabled);
    if (P.seg_enabled) {
        H.flag(P.seg_update_map);
        H.flag(1);
        H.flag(0);
        for (int s = 0; s < 4; s++) {
            int ql = P.seg[s].quantizer_level;
            H.flag(ql != 0);
            if (ql != 0) {
                H.literal(7, ql < 0 ? -ql : ql);
                H.flag(ql < 0);
            }
        }
        for (int s = 0; s < 4; s++) H.flag(0);
        if (P.seg_update_map)
            for (int i = 0; i < 3; i++) {
                H.flag(P.seg_probs[i] != 255);
                if (P.seg_probs[i] != 255) H.literal(8, P.seg_probs[i]);
            }
    }
    H.flag(0);
    H.literal(6, P.filter_level);
    H.literal(3, 0);
    H.flag(0);
    H.literal(2, nparts == 8 ? 3 : nparts >> 1);  // vp8.rs:352-354
    H.literal(7, P.base_qi);
    for (int i = 0; i < 5; i++) H.flag(0);
    H.literal(1, 0);
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++)
                for (int p = 0; p < 11; p++) {
                    uint8_t oldp = probs[t][b][c][p];
                    if (have_updated && upd[t][b][c][p] != oldp) {
                        H.put(1, COEFF_UPDATE_PROBS[t][b][c][p]);
                        H.literal(8, upd[t][b][c][p]);
                        probs[t][b][c][p] = upd[t][b][c][p];
                    } else {
                        H.put(0, COEFF_UPDATE_PROBS[t][b][c][p]);
                    }
                }
    H.literal(1, 1);
    H.literal(8, P.skip_prob);
}

// write_macroblock_header (vp8.rs:498-560) of MB x of the current row.
template <class Enc>
inline void emit_mb_header(Enc& H, const ZwFrameParams& P, const PackedMb& m, uint8_t* top_bp, uint8_t left_bp[4], int x)
{
    static const TreePaths seg_t(SEGMENT_ID_TREE, 6, 4), ymode_t(YMODE_TREE, 8, 5), bmode_t(BMODE_TREE, 18, 10),
        uvmode_t(UVMODE_TREE, 6, 4);
    if (P.seg_enabled && P.seg_update_map) seg_t.put(H, P.seg_probs, m.segment);
    H.put(m.skip, P.skip_prob);
    ymode_t.put(H, KEYFRAME_YMODE_PROBS, m.luma);
    if (m.luma == 4) {
        for (int by = 0; by < 4; by++) {
            int l = left_bp[by];
            for (int bx = 0; bx < 4; bx++) {
                int t = top_bp[x * 4 + bx], md = m.bpred[by * 4 + bx];
                bmode_t.put(H, KEYFRAME_BPRED_MODE_PROBS[t][l], md);
                l = md;
                top_bp[x * 4 + bx] = (uint8_t)md;
            }
            left_bp[by] = (uint8_t)l;
        }
    } else {
        static const int intra_of[4] = {0, 2, 3, 1};
        for (int i = 0; i < 4; i++) left_bp[i] = top_bp[x * 4 + i] = (uint8_t)intra_of[m.luma];
    }
    uvmode_t.put(H, KEYFRAME_UV_MODE_PROBS, m.chroma);
}

// encode_residual_data (vp8.rs:650-800) of one MB with its left / top
// complexity (non-zero) contexts.  Without an encoder (E == nullptr) only the
// contexts advance: a block's context bit is eob > 0, as emit_block returns.
template <class Enc>
inline void emit_mb_tokens(Enc* E, const uint8_t (*probs)[8][3][11], const PackedMb& m, Cplx& left, Cplx& top)
{
    const bool i4 = m.luma == 4;
    if (m.skip) {
        left.clear(!i4);
        top.clear(!i4);
        return;
    }
    const int plane = i4 ? 3 : 0;
    if (!i4) {
        int hc = E ? emit_block(*E, probs[1], m.lv[16], m.eob[16], 0, left.y2 + top.y2) : m.eob[16] > 0;
        left.y2 = top.y2 = (uint8_t)hc;
    }
    const int first = i4 ? 0 : 1;
    for (int by = 0; by < 4; by++) {
        int l = left.y[by];
        for (int bx = 0; bx < 4; bx++) {
            const int b = by * 4 + bx;
            int hc = E ? emit_block(*E, probs[plane], m.lv[b], m.eob[b], first, l + top.y[bx]) : m.eob[b] > 0;
            l = hc;
            top.y[bx] = (uint8_t)hc;
        }
        left.y[by] = (uint8_t)l;
    }
    for (int pl = 0; pl < 2; pl++) {
        uint8_t* lc = pl ? left.v : left.u;
        uint8_t* tc = pl ? top.v : top.u;
        for (int by = 0; by < 2; by++) {
            int l = lc[by];
            for (int bx = 0; bx < 2; bx++) {
                const int b = 17 + 4 * pl + by * 2 + bx;
                int hc = E ? emit_block(*E, probs[2], m.lv[b], m.eob[b], 0, l + tc[bx]) : m.eob[b] > 0;
                l = hc;
                tc[bx] = (uint8_t)hc;
            }
            lc[by] = (uint8_t)l;
        }
    }
}

// Frame tag (write_uncompressed_frame_header vp8.rs:315-330), the first
// partition, then for nparts > 1 the nparts - 1 3-byte partition sizes and the
// token partitions (RFC 6386 9.5; read back by decoder/vp8.rs:421-450).
inline void assemble_frame(std::vector<uint8_t>& out, const std::vector<uint8_t>& H, const BoolEncoder* T, int nparts,
                           int width, int height)
{
    size_t tot = 10 + H.size() + 3 * (size_t)(nparts - 1);
    for (int p = 0; p < nparts; p++) tot += T[p].buf.size();
    out.resize(tot);
    uint8_t* o = out.data();
    uint32_t tag = ((uint32_t)H.size() << 5) | (1u << 4);
    o[0] = (uint8_t)tag;
    o[1] = (uint8_t)(tag >> 8);
    o[2] = (uint8_t)(tag >> 16);
    o[3] = 0x9d;
    o[4] = 0x01;
    o[5] = 0x2a;
    o[6] = (uint8_t)(width & 0xff);
    o[7] = (uint8_t)((width >> 8) & 0x3f);
    o[8] = (uint8_t)(height & 0xff);
    o[9] = (uint8_t)((height >> 8) & 0x3f);
    memcpy(o + 10, H.data(), H.size());
    size_t w = 10 + H.size();
    for (int p = 0; p + 1 < nparts; p++, w += 3) {
        const size_t n = T[p].buf.size();
        o[w] = (uint8_t)n;
        o[w + 1] = (uint8_t)(n >> 8);
        o[w + 2] = (uint8_t)(n >> 16);
    }
    for (int p = 0; p < nparts; p++) {
        memcpy(o + w, T[p].buf.data(), T[p].buf.size());
        w += T[p].buf.size();
    }
}

// Frame assembly: compressed header (vp8.rs:332), MB headers (:498), residual
// partition (:650), frame tag (:315).  One token partition: headers and tokens
// in one raster walk.
inline void emit_frame(std::vector<uint8_t>& out, const ZwFrameParams& P, const uint8_t* packed, int width,
                       int height, bool have_updated, const uint8_t upd[4][8][3][11])
{
    PackedMb m;
    const int mbw = P.mbw, mbh = P.mbh;
    BoolEncoder H, T;
    T.buf.reserve((size_t)mbw * mbh * 16 + 4096);
    uint8_t probs[4][8][3][11];
    emit_frame_header(H, P, have_updated, upd, 1, probs);
    std::vector<Cplx> top(mbw);
    memset(top.data(), 0, sizeof(Cplx) * mbw);
    std::vector<uint8_t> top_bp((size_t)mbw * 4, 0);
    for (int y = 0; y < mbh; y++) {
        Cplx left;
        memset(&left, 0, sizeof left);
        uint8_t left_bp[4] = {0, 0, 0, 0};
        for (int x = 0; x < mbw; x++) {
            packed = view_mb(packed, m);
            emit_mb_header(H, P, m, top_bp.data(), left_bp, x);
            emit_mb_tokens(&T, probs, m, left, top[x]);
        }
    }
    H.flush();
    T.flush();
    assemble_frame(out, H.buf, &T, 1, width, height);
}

// The same with nparts (2, 4, 8) token partitions: MB row y's tokens go to
// partition y % nparts (vp8.rs:1419-1421).  A serial walk writes the MB headers
// and records where each row's records start and the top contexts it begins
// with; the partitions are then coded independently -- concurrently through
// `run(n, fn)` (fn(i) for i < n, e.g. parallel_for), or in turn without one.
template <class Run>
inline void emit_frame_parts(std::vector<uint8_t>& out, const ZwFrameParams& P, const uint8_t* packed, int width,
                             int height, bool have_updated, const uint8_t upd[4][8][3][11], int nparts, Run run)
{
    if (nparts <= 1) {
        emit_frame(out, P, packed, width, height, have_updated, upd);
        return;
    }
    PackedMb m;
    const int mbw = P.mbw, mbh = P.mbh;
    BoolEncoder H, T[8];
    uint8_t probs[4][8][3][11];
    emit_frame_header(H, P, have_updated, upd, nparts, probs);
    std::vector<const uint8_t*> row_at((size_t)mbh);
    std::vector<Cplx> top_at((size_t)mbh * mbw), top(mbw);
    memset(top.data(), 0, sizeof(Cplx) * mbw);
    std::vector<uint8_t> top_bp((size_t)mbw * 4, 0);
    for (int y = 0; y < mbh; y++) {
        row_at[y] = packed;
        memcpy(&top_at[(size_t)y * mbw], top.data(), sizeof(Cplx) * mbw);
        Cplx left;
        memset(&left, 0, sizeof left);
        uint8_t left_bp[4] = {0, 0, 0, 0};
        for (int x = 0; x < mbw; x++) {
            packed = view_mb(packed, m);
            emit_mb_header(H, P, m, top_bp.data(), left_bp, x);
            emit_mb_tokens<BoolEncoder>(nullptr, probs, m, left, top[x]);
        }
    }
    H.flush();
    run(nparts, [&](int p) {
        PackedMb pm;
        BoolEncoder& E = T[p];
        E.buf.reserve((size_t)mbw * mbh * 16 / nparts + 4096);
        for (int y = p; y < mbh; y += nparts) {
            const uint8_t* q = row_at[y];
            Cplx* tr = &top_at[(size_t)y * mbw];
            Cplx left;
            memset(&left, 0, sizeof left);
            for (int x = 0; x < mbw; x++) {
                q = view_mb(q, pm);
                emit_mb_tokens(&E, probs, pm, left, tr[x]);
            }
        }
        E.flush();
    });
    assemble_frame(out, H.buf, T, nparts, width, height);
}

// ---------------------------------------------------------------------------
// Split emission: the token walk records each MB's decisions (bit, probability)
// and a tight loop codes them.  The boolean coder's cost is its serial
// dependence through `range` (multiply, select, count-leading-zeros, shift per
// decision); with the token logic out of that loop, the coder of two frames can
// run interleaved in one thread (emit_frames2), so the two independent chains
// overlap.  Byte-identical to emit_frame (tools/emit_bench.cpp, the equivalence
// tests): the same arithmetic in the same order per stream.
// ---------------------------------------------------------------------------
struct DecRec {  // BoolEncoder's interface; each decision appended as prob | bit << 8
    uint16_t* p;
    inline void put(int bit, int prob) { *p++ = (uint16_t)((uint32_t)prob | ((uint32_t)(bit != 0) << 8)); }
    void flag(int f) { put(f, 128); }
    void literal(int nbits, int v)
    {
        for (int b = nbits - 1; b >= 0; b--) put(((1 << b) & v) > 0, 128);
    }
    inline void path(const uint8_t* bits, const uint8_t* pidx, int n, const uint8_t* probs)
    {
        for (int i = 0; i < n; i++) put(bits[i], probs[pidx[i]]);
    }
};
// decisions of one MB's tokens: at most 25 blocks x 16 positions x (11 tree +
// 11 extra + 1 sign) + 25 end-of-block decisions
constexpr int kMbDecisionsMax = 25 * 16 * 23 + 25;

// BoolEncoder's arithmetic into a caller-sized byte buffer (one spare byte in
// front for a carry out of the first byte).
struct RawBool {
    std::vector<uint8_t> buf;
    size_t lo = 1, pos = 1;  // first byte, next byte
    uint32_t low = 0, range = 255;
    int count = -24;
    void reserve_more(size_t n)
    {
        if (pos + n + 8 > buf.size()) buf.resize((pos + n + 8) * 2);
    }
    void carry(uint8_t* b)
    {
        size_t i = pos;
        while (i > lo) {
            i--;
            if (b[i] < 255) {
                b[i]++;
                return;
            }
            b[i] = 0;
        }
        b[--lo] = 1;
    }
    void flush()
    {
        reserve_more(8);
        uint8_t* b = buf.data();
        const int bit_num = -count;
        int c = bit_num;
        uint32_t v = low;
        if (low & (1u << (32 - bit_num))) carry(b);
        v <<= (c & 7);
        c = (c >> 3) - 1;
        while (c >= 0) {
            v <<= 8;
            c--;
        }
        for (c = 3; c >= 0; c--) {
            b[pos++] = (uint8_t)(v >> 24);
            v <<= 8;
        }
    }
    const uint8_t* data() const { return buf.data() + lo; }
    size_t size() const { return pos - lo; }
};

// M streams, n decisions each, interleaved (M independent dependency chains).
// BoolEncoder's arithmetic with the low end of the interval in 64 bits: L holds
// 8 + c bits (c pending above the 8-bit range) and 48 pending bits go out at a
// time, so the byte-out branch -- unpredictable across four interleaved
// streams -- is taken once per ~64 decisions instead of ~11.  A carry out of L
// goes into the bytes already out at once.  The state enters and leaves in
// BoolEncoder's form (low, count: 16..23 bits pending once a byte is out), so
// the bytes are BoolEncoder's.  (Measured on the box, four distinct frames'
// streams: 0.93 ms per stream with 32 bits at a time, 1.07 with one byte.)
template <int M>
inline void raw_codeM(RawBool* const* S, const uint16_t* const* d, int n)
{
    uint8_t* b[M];
    uint64_t lo[M];
    uint32_t ra[M];
    int co[M];
    size_t po[M];
#pragma GCC unroll 4
    for (int k = 0; k < M; k++) {
        S[k]->reserve_more((size_t)n);
        b[k] = S[k]->buf.data();
        lo[k] = S[k]->low, ra[k] = S[k]->range, co[k] = S[k]->count + 24, po[k] = S[k]->pos;
        if (lo[k] >> (8 + co[k])) {  // (a carry BoolEncoder had not yet taken out)
            S[k]->carry(b[k]);
            lo[k] &= (1ull << (8 + co[k])) - 1;
        }
    }
    for (int i = 0; i < n; i++) {
#pragma GCC unroll 4
        for (int k = 0; k < M; k++) {
            const uint32_t D = d[k][i], prob = D & 255u, m = 0u - (D >> 8);
            const uint32_t split = 1 + (((ra[k] - 1) * prob) >> 8);
            lo[k] += split & m;
            if (__builtin_expect((lo[k] >> (8 + co[k])) != 0, 0)) {
                S[k]->pos = po[k];
                S[k]->carry(b[k]);
                lo[k] &= (1ull << (8 + co[k])) - 1;
            }
            const uint32_t r = split ^ ((split ^ (ra[k] - split)) & m);
            const int sh = __builtin_clz(r) - 24;
            ra[k] = r << sh;
            lo[k] <<= sh;
            co[k] += sh;
            if (co[k] >= 48) {  // the top 48 of the 8 + c bits, as 8 bytes (the last 2 rewritten later)
                const uint64_t be = __builtin_bswap64(lo[k] << (56 - co[k]));
                memcpy(b[k] + po[k], &be, 8);
                po[k] += 6;
                co[k] -= 48;
                lo[k] &= (1ull << (8 + co[k])) - 1;
            }
        }
    }
#pragma GCC unroll 4
    for (int k = 0; k < M; k++) {
        while (co[k] >= 24) {
            b[k][po[k]++] = (uint8_t)(lo[k] >> co[k]);
            lo[k] &= (1ull << co[k]) - 1;
            co[k] -= 8;
        }
        while (co[k] < 16 && po[k] > S[k]->lo) {  // bytes back in (at most 5)
            lo[k] |= (uint64_t)b[k][--po[k]] << (8 + co[k]);
            co[k] += 8;
        }
        S[k]->low = (uint32_t)lo[k], S[k]->range = ra[k], S[k]->count = co[k] - 24, S[k]->pos = po[k];
    }
}

// Up to 16 streams at once, one per lane of AVX-512 vectors: raw_codeM's
// arithmetic (low end in 64 bits, 48 pending bits out at a time) on 16 lanes,
// each lane's decision fetched by a gather from the shared arena `base` at
// element offset off[k] + i; lanes past their stream's length n[k] are masked.
// The rare events -- a carry, 48 bits due -- are handled per lane in scalar
// code.  Same bytes as raw_codeM (one independent coder per lane).
__attribute__((target("avx512f,avx512cd,avx512vl,avx512dq,avx512bw"))) inline void raw_code16(
    RawBool* const* S, const uint16_t* base, const uint32_t* off, const int* n, int K)
{
    alignas(64) uint64_t lo[16];
    alignas(64) uint32_t ra[16], ix[16], nn[16];
    alignas(64) int32_t co[16];
    uint8_t* b[16];
    size_t po[16];
    int nmax = 0;
    for (int k = 0; k < 16; k++) {
        if (k < K) {
            S[k]->reserve_more((size_t)n[k]);
            b[k] = S[k]->buf.data();
            lo[k] = S[k]->low, ra[k] = S[k]->range, co[k] = S[k]->count + 24, po[k] = S[k]->pos;
            if (lo[k] >> (8 + co[k])) {
                S[k]->carry(b[k]);
                lo[k] &= (1ull << (8 + co[k])) - 1;
            }
            ix[k] = off[k];
            nn[k] = (uint32_t)n[k];
            nmax = n[k] > nmax ? n[k] : nmax;
        } else {
            b[k] = nullptr;
            lo[k] = 0, ra[k] = 255, co[k] = 0, po[k] = 0, ix[k] = 0, nn[k] = 0;
        }
    }
    __m512i vlo0 = _mm512_load_si512(lo), vlo1 = _mm512_load_si512(lo + 8);
    __m512i vra = _mm512_load_si512(ra), vco = _mm512_load_si512(co), vix = _mm512_load_si512(ix);
    const __m512i vnn = _mm512_load_si512(nn), one = _mm512_set1_epi32(1), c255 = _mm512_set1_epi32(255);
    const __m512i c256 = _mm512_set1_epi32(0x100), c24 = _mm512_set1_epi32(24), c8 = _mm512_set1_epi32(8);
    const __m512i c48 = _mm512_set1_epi32(48);
    __m512i vi = _mm512_setzero_si512();
    for (int i = 0; i < nmax; i++) {
        const __mmask16 act = _mm512_cmpgt_epu32_mask(vnn, vi);
        vi = _mm512_add_epi32(vi, one);
        const __m512i d = _mm512_mask_i32gather_epi32(_mm512_setzero_si512(), act, vix, (const void*)base, 2);
        vix = _mm512_add_epi32(vix, one);
        const __m512i prob = _mm512_and_si512(d, c255);
        const __mmask16 bit = _mm512_mask_test_epi32_mask(act, d, c256);
        const __m512i split = _mm512_add_epi32(one, _mm512_srli_epi32(_mm512_mullo_epi32(_mm512_sub_epi32(vra, one), prob), 8));
        const __m512i r = _mm512_mask_sub_epi32(split, bit, vra, split);
        const __m512i sh = _mm512_maskz_sub_epi32(act, _mm512_lzcnt_epi32(r), c24);
        vra = _mm512_mask_sllv_epi32(vra, act, r, sh);
        // low += split (bit lanes), in two halves of 8 x 64 bits
        const __m512i add = _mm512_maskz_mov_epi32(bit, split);
        vlo0 = _mm512_add_epi64(vlo0, _mm512_cvtepu32_epi64(_mm512_castsi512_si256(add)));
        vlo1 = _mm512_add_epi64(vlo1, _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(add, 1)));
        const __m512i w = _mm512_add_epi32(vco, c8);  // the bits L may hold
        const __m512i w0 = _mm512_cvtepu32_epi64(_mm512_castsi512_si256(w)), w1 = _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(w, 1));
        const __mmask8 cy0 = _mm512_test_epi64_mask(_mm512_srlv_epi64(vlo0, w0), _mm512_srlv_epi64(vlo0, w0));
        const __mmask8 cy1 = _mm512_test_epi64_mask(_mm512_srlv_epi64(vlo1, w1), _mm512_srlv_epi64(vlo1, w1));
        if (__builtin_expect((cy0 | cy1) != 0, 0)) {
            _mm512_store_si512(lo, vlo0);
            _mm512_store_si512(lo + 8, vlo1);
            const unsigned cm = (unsigned)cy0 | ((unsigned)cy1 << 8);
            for (int k = 0; k < 16; k++)
                if ((cm >> k) & 1u) {
                    S[k]->pos = po[k];
                    S[k]->carry(b[k]);
                    lo[k] &= (1ull << (8 + co[k])) - 1;
                }
            vlo0 = _mm512_load_si512(lo);
            vlo1 = _mm512_load_si512(lo + 8);
        }
        vlo0 = _mm512_sllv_epi64(vlo0, _mm512_cvtepu32_epi64(_mm512_castsi512_si256(sh)));
        vlo1 = _mm512_sllv_epi64(vlo1, _mm512_cvtepu32_epi64(_mm512_extracti64x4_epi64(sh, 1)));
        vco = _mm512_add_epi32(vco, sh);
        _mm512_store_si512(co, vco);  // (co[] stays current for the scalar paths)
        const __mmask16 fm = _mm512_cmpge_epi32_mask(vco, c48);
        if (fm) {
            _mm512_store_si512(lo, vlo0);
            _mm512_store_si512(lo + 8, vlo1);
            for (unsigned m = fm; m; m &= m - 1) {
                const int k = __builtin_ctz(m);
                const uint64_t be = __builtin_bswap64(lo[k] << (56 - co[k]));
                memcpy(b[k] + po[k], &be, 8);
                po[k] += 6;
                co[k] -= 48;
                lo[k] &= (1ull << (8 + co[k])) - 1;
            }
            vlo0 = _mm512_load_si512(lo);
            vlo1 = _mm512_load_si512(lo + 8);
            vco = _mm512_load_si512(co);
        }
    }
    _mm512_store_si512(lo, vlo0);
    _mm512_store_si512(lo + 8, vlo1);
    _mm512_store_si512(ra, vra);
    _mm512_store_si512(co, vco);
    for (int k = 0; k < K; k++) {
        while (co[k] >= 24) {
            b[k][po[k]++] = (uint8_t)(lo[k] >> co[k]);
            lo[k] &= (1ull << co[k]) - 1;
            co[k] -= 8;
        }
        while (co[k] < 16 && po[k] > S[k]->lo) {
            lo[k] |= (uint64_t)b[k][--po[k]] << (8 + co[k]);
            co[k] += 8;
        }
        S[k]->low = (uint32_t)lo[k], S[k]->range = ra[k], S[k]->count = co[k] - 24, S[k]->pos = po[k];
    }
}
inline bool have_code16()
{
    static const bool ok = [] {
        if (const char* e = getenv("ZW_CODE16"))
            if (atoi(e) == 0) return false;
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512cd") &&
               __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq") &&
               __builtin_cpu_supports("avx512bw");
    }();
    return ok;
}

// K (<= 4) streams of different lengths: interleaved over the common length,
// then over the longer ones' remainders.
inline void raw_code_multi(RawBool* const* S, const uint16_t* const* d, const int* n, int K)
{
    const uint16_t* dd[4];
    int nn[4];
    for (int k = 0; k < K; k++) dd[k] = d[k], nn[k] = n[k];
    for (;;) {
        RawBool* as[4];
        const uint16_t* ad[4];
        int ai[4], m = 0, mn = 1 << 30;
        for (int k = 0; k < K; k++)
            if (nn[k] > 0) {
                as[m] = S[k];
                ad[m] = dd[k];
                ai[m++] = k;
                mn = nn[k] < mn ? nn[k] : mn;
            }
        if (m == 0) return;
        switch (m) {
        case 4: raw_codeM<4>(as, ad, mn); break;
        case 3: raw_codeM<3>(as, ad, mn); break;
        case 2: raw_codeM<2>(as, ad, mn); break;
        default: raw_codeM<1>(as, ad, mn); break;
        }
        for (int j = 0; j < m; j++) dd[ai[j]] += mn, nn[ai[j]] -= mn;
    }
}

// The token tree paths as decision templates: per (after-a-zero, token) the
// decisions bit << 8 | probability index, padded to 12 with index 0.
struct TokTmpl {
    uint8_t n[2][12];
    uint16_t d[2][12][12];
    TokTmpl()
    {
        const TokenPaths& TP = token_paths();
        for (int s = 0; s < 2; s++)
            for (int v = 0; v < 12; v++) {
                n[s][v] = TP.n[s][v];
                for (int i = 0; i < 12; i++)
                    d[s][v][i] = i < TP.n[s][v] ? (uint16_t)((TP.bits[s][v][i] << 8) | TP.pidx[s][v][i]) : 0;
            }
    }
};
inline const TokTmpl& tok_tmpl()
{
    static const TokTmpl T;
    return T;
}

// The token paths with the frame's probabilities filled in: per (type, band,
// ctx, after-a-zero, token) the path's decisions (bit << 8 | probability),
// its length in entry 15.  Built once per frame (the probabilities are fixed
// for the frame's tokens), so a token's decisions are one 32-byte copy.
struct TokRes {
    alignas(32) uint16_t d[4][8][3][2][12][16];
};
inline void tok_resolve(TokRes& R, const uint8_t (*probs)[8][3][11])
{
    const TokTmpl& TT = tok_tmpl();
    for (int t = 0; t < 4; t++)
        for (int b = 0; b < 8; b++)
            for (int c = 0; c < 3; c++)
                for (int s = 0; s < 2; s++)
                    for (int v = 0; v < 12; v++) {
                        uint16_t* o = R.d[t][b][c][s][v];
                        const int n = TT.n[s][v];
                        for (int i = 0; i < 16; i++)
                            o[i] = i < n ? (uint16_t)((TT.d[s][v][i] & 0xff00u) | probs[t][b][c][TT.d[s][v][i] & 0xffu]) : 0;
                        o[15] = (uint16_t)n;
                    }
}

// emit_block's decisions (the same sequence) recorded at o (which has 16
// entries of slack: a path is copied whole).  Rt: the block type's resolved
// paths, P its probabilities.
inline int rec_block(uint16_t*& o, const uint16_t (*Rt)[3][2][12][16], const uint8_t (*P)[3][11], const uint8_t* lv,
                     int eobi, int first, int ctx)
{
    if (eobi <= first) {  // no coefficient: the end of block at `first` (bit 0)
        *o++ = P[COEFF_BANDS[first]][ctx][0];
        return eobi > 0;
    }
    int s = 0;
    uint16_t* q = o;
    for (int idx = first; idx < eobi; idx++) {
        const int coeff = lv_at(lv, idx);
        const int a = coeff < 0 ? -coeff : coeff;
        const int token = token_of(a);
        const uint16_t* t = Rt[COEFF_BANDS[idx]][ctx][s][token];
        memcpy(q, t, 32);
        q += t[15];
        if (token >= 5) {
            const uint8_t* cp = PROB_DCT_CAT[token - 5];
            const int extra = a - DCT_CAT_BASE[token - 5];
            int mask = token == 10 ? 1 << 10 : 1 << (token - 5);
            for (int k = 0; k < 12 && cp[k]; k++) {
                *q++ = (uint16_t)(cp[k] | ((extra & mask) ? 0x100 : 0));
                mask >>= 1;
            }
        }
        // the sign (token != 0), written always and kept only for a nonzero
        *q = (uint16_t)(128u | (((uint32_t)coeff >> 31) << 8));
        q += token != 0;
        s = token == 0;
        ctx = token >= 2 ? 2 : token;
    }
    if (eobi < 16) *q++ = P[COEFF_BANDS[eobi]][ctx][0];
    o = q;
    return 1;
}

// Blocks b0 .. b0 + nb - 1 (nb <= 16) of one block type in order, contexts cx,
// ne the mask of the non-empty ones (eob > first): the empty blocks' decisions
// (an end of block each) go out as whole runs -- one copy per run, from every
// block's end-of-block decision made up front -- so only the non-empty blocks
// take a branch (most blocks are empty: 85 % of a Q75 1080p frame's).
#ifndef ZW_WALK_RUNS
#define ZW_WALK_RUNS 1
#endif
inline void rec_block_runs(uint16_t*& o, const uint16_t (*Rt)[3][2][12][16], const uint8_t (*P)[3][11],
                           const PackedMb& m, int b0, int nb, const int* cx, int first, uint32_t ne)
{
    uint16_t eobd[32];
    const uint8_t* pb = P[COEFF_BANDS[first]][0];
    for (int i = 0; i < nb; i++) eobd[i] = pb[11 * cx[i]];
    uint16_t* q = o;
    int i = 0;
    for (;;) {
        const int j = ne ? __builtin_ctz(ne) : nb;
        memcpy(q, eobd + i, 32);  // (the run i .. j - 1; the rest is rewritten)
        q += j - i;
        if (j >= nb) break;
        rec_block(q, Rt, P, m.lv[b0 + j], m.eob[b0 + j], first, cx[j]);
        ne &= ne - 1;
        i = j + 1;
    }
    o = q;
}

// emit_mb_tokens' decisions (rec_block per block), the same contexts.  A
// block's context bit is eob > 0 (what emit_block returns), so every block's
// context is taken from the eobs up front: the blocks' walks do not wait on
// each other.
inline void rec_mb_tokens(uint16_t*& o, const TokRes& R, const uint8_t (*probs)[8][3][11], const PackedMb& m, Cplx& left,
                          Cplx& top)
{
    const bool i4 = m.luma == 4;
    if (m.skip) {
        left.clear(!i4);
        top.clear(!i4);
        return;
    }
    const int plane = i4 ? 3 : 0;
    const uint8_t* e = m.eob;
    if (!i4) {
        const int c = left.y2 + top.y2;
        left.y2 = top.y2 = (uint8_t)(e[16] > 0);
        rec_block(o, R.d[1], probs[1], m.lv[16], e[16], 0, c);
    }
    const int first = i4 ? 0 : 1;
    int ctx[16];
    for (int by = 0; by < 4; by++)
        for (int bx = 0; bx < 4; bx++) {
            const int b = by * 4 + bx;
            const int l = bx ? (int)(e[b - 1] > 0) : left.y[by];
            const int t = by ? (int)(e[b - 4] > 0) : top.y[bx];
            ctx[b] = l + t;
        }
    for (int k = 0; k < 4; k++) {
        left.y[k] = (uint8_t)(e[4 * k + 3] > 0);
        top.y[k] = (uint8_t)(e[12 + k] > 0);
    }
#if ZW_WALK_RUNS
    {
        uint32_t ne = 0;
        for (int b = 0; b < 16; b++) ne |= (uint32_t)(e[b] > first) << b;
        rec_block_runs(o, R.d[plane], probs[plane], m, 0, 16, ctx, first, ne);
        int cc[8];
        uint32_t nc = 0;
        for (int pl = 0; pl < 2; pl++) {
            uint8_t* lc = pl ? left.v : left.u;
            uint8_t* tc = pl ? top.v : top.u;
            const int b0 = 17 + 4 * pl;
            cc[4 * pl] = lc[0] + tc[0];
            cc[4 * pl + 1] = (e[b0] > 0) + tc[1];
            cc[4 * pl + 2] = lc[1] + (e[b0] > 0);
            cc[4 * pl + 3] = (e[b0 + 2] > 0) + (e[b0 + 1] > 0);
            lc[0] = (uint8_t)(e[b0 + 1] > 0);
            lc[1] = (uint8_t)(e[b0 + 3] > 0);
            tc[0] = (uint8_t)(e[b0 + 2] > 0);
            tc[1] = (uint8_t)(e[b0 + 3] > 0);
            for (int k = 0; k < 4; k++) nc |= (uint32_t)(e[b0 + k] > 0) << (4 * pl + k);
        }
        rec_block_runs(o, R.d[2], probs[2], m, 17, 8, cc, 0, nc);
        return;
    }
#endif
    for (int b = 0; b < 16; b++) rec_block(o, R.d[plane], probs[plane], m.lv[b], e[b], first, ctx[b]);
    for (int pl = 0; pl < 2; pl++) {
        uint8_t* lc = pl ? left.v : left.u;
        uint8_t* tc = pl ? top.v : top.u;
        const int b0 = 17 + 4 * pl;
        const int c0 = lc[0] + tc[0], c1 = (e[b0] > 0) + tc[1], c2 = lc[1] + (e[b0] > 0),
                  c3 = (e[b0 + 2] > 0) + (e[b0 + 1] > 0);
        lc[0] = (uint8_t)(e[b0 + 1] > 0);
        lc[1] = (uint8_t)(e[b0 + 3] > 0);
        tc[0] = (uint8_t)(e[b0 + 2] > 0);
        tc[1] = (uint8_t)(e[b0 + 3] > 0);
        rec_block(o, R.d[2], probs[2], m.lv[b0], e[b0], 0, c0);
        rec_block(o, R.d[2], probs[2], m.lv[b0 + 1], e[b0 + 1], 0, c1);
        rec_block(o, R.d[2], probs[2], m.lv[b0 + 2], e[b0 + 2], 0, c2);
        rec_block(o, R.d[2], probs[2], m.lv[b0 + 3], e[b0 + 3], 0, c3);
    }
}

inline void assemble_frame1(std::vector<uint8_t>& out, const RawBool& H, const RawBool& T, int width, int height)
{
    const size_t hs = H.size(), ts = T.size();
    out.resize(10 + hs + ts);
    uint8_t* o = out.data();
    const uint32_t tag = ((uint32_t)hs << 5) | (1u << 4);
    o[0] = (uint8_t)tag;
    o[1] = (uint8_t)(tag >> 8);
    o[2] = (uint8_t)(tag >> 16);
    o[3] = 0x9d;
    o[4] = 0x01;
    o[5] = 0x2a;
    o[6] = (uint8_t)(width & 0xff);
    o[7] = (uint8_t)((width >> 8) & 0x3f);
    o[8] = (uint8_t)(height & 0xff);
    o[9] = (uint8_t)((height >> 8) & 0x3f);
    memcpy(o + 10, H.data(), hs);
    memcpy(o + 10 + hs, T.data(), ts);
}

// The buffers of emit_frames (decision records, coders, row state) for up to
// four frames.  Kept between calls (a caller's pool, or one per thread): the
// record buffers are sized for the worst case, and allocating and faulting
// them in afresh cost more than the emission of a frame.
struct EmitWs {
    static constexpr int kMax = 16;
    struct Fr {
        RawBool H, T;
        std::vector<Cplx> top;
        std::vector<uint8_t> top_bp;
        uint8_t probs[4][8][3][11];
        TokRes res;
    } F[kMax];
    // decision records, kMax frames' each in one arena (the 16-lane coder gathers
    // from it by 32-bit offsets); sized for the worst case and left uninitialised,
    // so only the pages a frame writes are ever touched
    std::unique_ptr<uint16_t[]> hd, td;
    size_t hcap = 0, tcap = 0;
    int hk = 0, tk = 0;  // frames the arenas hold
    std::vector<uint8_t> out[kMax], alph;  // (for the caller: container assembly)
};

// K coders over their decision runs d[k] (n[k] decisions each): the 16-lane
// coder when the host has AVX-512, there are more than four and the runs lie
// within 2^31 elements of `base` (its gather offsets), else four at a time.
inline void code_streams(RawBool* const* S, const uint16_t* base, const uint16_t* const* d, const int* n, int K)
{
    if (K > 4 && have_code16()) {
        uint32_t off[16];
        bool fit = true;
        for (int k = 0; k < K; k++) {
            const size_t o = (size_t)(d[k] - base);
            fit = fit && o + (size_t)n[k] < ((size_t)1 << 31);
            off[k] = (uint32_t)o;
        }
        if (fit) {
            raw_code16(S, base, off, n, K);
            return;
        }
    }
    for (int k0 = 0; k0 < K; k0 += 4) raw_code_multi(S + k0, d + k0, n + k0, std::min(4, K - k0));
}

// emit_frame of K (1..16) frames of one size at once (one token partition):
// each MB row's header and token decisions are recorded per frame, then the
// K frames' coders run side by side.  Byte-identical to emit_frame per frame.
// Bytes of emit_frames' decision arenas per frame of a group (worst case, mostly
// never touched): callers size their groups with it.
inline size_t emit_arena_bytes(int mbw, int mbh)
{
    return 2 * ((4 * 8 * 3 * 11 * 9 + 256 + (size_t)mbw * mbh * 160) + ((size_t)mbw * kMbDecisionsMax + 32));
}

inline void emit_frames(std::vector<uint8_t>* const* out, const ZwFrameParams* const* P, const uint8_t* const* packed,
                        int K, int width, int height, const bool* have_updated, const uint8_t (*const* upd)[8][3][11],
                        EmitWs* ws = nullptr)
{
    using Fr = EmitWs::Fr;
    thread_local std::unique_ptr<EmitWs> own;
    if (!ws) {
        if (!own) own.reset(new EmitWs);
        ws = own.get();
    }
    Fr* F = ws->F;
    const int mbw = P[0]->mbw, mbh = P[0]->mbh;
    // the frame header's decisions (at most 4 x 8 x 3 x 11 x 9 probability updates
    // and ~100 others), then the MB headers' (whole frame; at most 2 + 1 + 4 + 16 x 9
    // + 3 per MB); a row's token decisions (+ rec_block's slack, + the gather's)
    const size_t hcap = 4 * 8 * 3 * 11 * 9 + 256 + (size_t)mbw * mbh * 160;
    const size_t tcap = (size_t)mbw * kMbDecisionsMax + 32;
    if (ws->hcap < hcap || ws->hk < K) {
        ws->hd.reset();
        ws->hd.reset(new uint16_t[hcap * (size_t)K + 32]);
        ws->hcap = hcap;
        ws->hk = K;
    }
    if (ws->tcap < tcap || ws->tk < K) {
        ws->td.reset();
        ws->td.reset(new uint16_t[tcap * (size_t)K + 32]);
        ws->tcap = tcap;
        ws->tk = K;
    }
    uint16_t* const hd = ws->hd.get();
    uint16_t* const td = ws->td.get();
    const size_t hst = ws->hcap, tst = ws->tcap;
    const uint8_t* q[EmitWs::kMax];
    size_t hn[EmitWs::kMax];
    for (int k = 0; k < K; k++) {
        Fr& f = F[k];
        for (RawBool* r : {&f.H, &f.T}) {
            r->lo = r->pos = 1;
            r->low = 0;
            r->range = 255;
            r->count = -24;
        }
        f.T.reserve_more((size_t)mbw * mbh * 16 + 4096);
        f.top.assign(mbw, Cplx{});
        f.top_bp.assign((size_t)mbw * 4, 0);
        DecRec R{hd + (size_t)k * hst};
        emit_frame_header(R, *P[k], have_updated[k], upd[k], 1, f.probs);
        tok_resolve(f.res, f.probs);
        q[k] = packed[k];
        hn[k] = (size_t)(R.p - (hd + (size_t)k * hst));
    }
    RawBool* ts[EmitWs::kMax];
    const uint16_t* tp[EmitWs::kMax];
    int tn[EmitWs::kMax];
    for (int y = 0; y < mbh; y++) {
        for (int k = 0; k < K; k++) {
            Fr& f = F[k];
            Cplx left;
            memset(&left, 0, sizeof left);
            uint8_t left_bp[4] = {0, 0, 0, 0};
            DecRec R{hd + (size_t)k * hst + hn[k]};
            uint16_t* const o0 = td + (size_t)k * tst;
            uint16_t* o = o0;
            for (int x = 0; x < mbw; x++) {
                PackedMb m;
                q[k] = view_mb(q[k], m);
                emit_mb_header(R, *P[k], m, f.top_bp.data(), left_bp, x);
                rec_mb_tokens(o, f.res, f.probs, m, left, f.top[x]);
            }
            hn[k] = (size_t)(R.p - (hd + (size_t)k * hst));
            tp[k] = o0;
            tn[k] = (int)(o - o0);
            ts[k] = &f.T;
        }
        code_streams(ts, td, tp, tn, K);
    }
    // the header partitions
    RawBool* hs[EmitWs::kMax];
    const uint16_t* hp[EmitWs::kMax];
    int hl[EmitWs::kMax];
    for (int k = 0; k < K; k++) {
        hp[k] = hd + (size_t)k * hst;
        hl[k] = (int)hn[k];
        hs[k] = &F[k].H;
    }
    code_streams(hs, hd, hp, hl, K);
    for (int k = 0; k < K; k++) {
        F[k].H.flush();
        F[k].T.flush();
        assemble_frame1(*out[k], F[k].H, F[k].T, width, height);
    }
}

// quality_to_quant_index (vp8.rs:37-55) with fast_math::cbrt/round (fast_math.rs:15-42).
inline int quality_to_qi(int quality)
{
    double c = (double)quality / 100.0;
    double lin = c < 0.75 ? c * (2.0 / 3.0) : 2.0 * c - 1.0;
    double y = 0.0;
    if (lin != 0.0) {
        uint64_t bits;
        memcpy(&bits, &lin, 8);
        uint64_t ab = bits / 3 + (uint64_t)(1023ull * 2 / 3) * (1ull << 52);
        memcpy(&y, &ab, 8);
        for (int i = 0; i < 4; i++) {
            double y2 = y * y;
            y = (2.0 * y + lin / y2) / 3.0;
        }
    }
    double r = (double)(int64_t)(127.0 * (1.0 - y) + 0.5);
    int q = (int)r;
    return q < 0 ? 0 : (q > 127 ? 127 : q);
}

// compute_filter_level (cost.rs:271) with sharpness 0, strength 50.
inline int filter_level_for(int qi)
{
    uint32_t level0 = 250;
    int qstep = (uint8_t)(VP8_AC_TABLE[qi] >> 2);
    uint32_t base = LEVELS_FROM_DELTA[0][qstep < 63 ? qstep : 63];
    uint32_t f = base * level0 / 256;
    if (f < 2) return 0;
    return f > 63 ? 63 : (int)f;
}

}  // namespace zwh
