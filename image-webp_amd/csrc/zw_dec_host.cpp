// zw_dec_host.cpp -- VP8 keyframe decoder: host bool decoder + device
// reconstruction / loop filter.
//
//   host  : frame header (decoder/vp8.rs:553-670), partitions (:421-450),
//           quantiser indices (:452-504), MB modes (:681-734) and residual
//           tokens (:872-1058) -> one packed record per macroblock.  The
//           boolean decoder follows decoder/bit_reader.rs (libwebp-style
//           56-bit refill, one zero byte past the end then eof).
//   device: k_dec_recon (dequant, iWHT, iDCT, prediction) and k_loopfilter.
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <new>
#include <string>
#include <vector>

#include "../../include/zwebp.h"
#include "zw_common.h"
#include "zw_host_entropy.h"
#include "zw_host_internal.h"

extern "C" {
hipError_t zwk_dec_recon(hipStream_t s, const uint8_t* recs, const uint32_t* moff, const uint64_t* fbase,
                         const void* quant, uint8_t* Y, uint8_t* U, uint8_t* V, uint8_t* flags, int mbw, int mbh,
                         size_t ysz, size_t csz, int nframes, uint8_t* tiles);
hipError_t zwk_yuv2rgb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, size_t ysz, size_t csz,
                       int w, int h, int ys, int cs, int bpp, int fancy, uint8_t* out, int nframes);
hipError_t zwk_dec_rows(hipStream_t s, int phase, const uint8_t* recs, const uint32_t* moff, const uint64_t* fbase,
                        const void* quant, uint8_t* Y, uint8_t* U, uint8_t* V, uint8_t* flags, const ZwFilterParams* fp,
                        int mbw, int mbh, size_t ysz, size_t csz, int nframes, int* rowsync, uint8_t* borders, int rows);
hipError_t zwk_dec_rows_init(hipStream_t s, int* rowsync, int mbh, int nframes);
size_t zw_dec_rows_sync_bytes(int mbh, int nframes);
size_t zw_dec_rows_border_bytes(int mbw, int nframes);
hipError_t zwk_loopfilter(hipStream_t s, uint8_t* Y, uint8_t* U, uint8_t* V, const uint8_t* flags,
                          const ZwFilterParams* fp, size_t ysz, size_t csz, int nframes, int mbw, const uint8_t* tiles);
hipError_t zwk_dec_tok_count(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                             const uint8_t* modes, const uint32_t* cls, uint8_t* snaps, int* err1, uint32_t* sizes,
                             int* err2, uint32_t* moff, uint64_t* fbase, int* terr, uint64_t* d_total,
                             uint64_t* host_total, int mbw, int mbh, int n, hipEvent_t stage1_done);
hipError_t zwk_dec_tok_write(hipStream_t s, const uint8_t* blob, const ZwTokFrame* tf, const uint8_t* probs,
                             const uint8_t* modes, const uint8_t* snaps, const int* err1, const uint32_t* moff,
                             const uint64_t* fbase, uint8_t* recs, int nmb, int n);
size_t zw_tok1_lds_bytes(int mbw);
}
#include "zw_tokl.h"

namespace {

using namespace zwh;

struct DecQuant {
    int32_t ydc, yac, y2dc, y2ac, uvdc, uvac;
};

// bit_reader.rs:254-640
struct BitReader {
    const uint8_t* d = nullptr;
    size_t len = 0, pos = 0;
    uint64_t value = 0;
    uint32_t range = 254;  // range - 1
    int bits = -8;
    bool eof = false;

    void init(const uint8_t* data, size_t n)
    {
        d = data;
        len = n;
        pos = 0;
        value = 0;
        range = 254;
        bits = -8;
        eof = false;
        load();
    }
    void load()
    {
        const size_t rem = len - pos;
        if (rem >= 7) {
            uint64_t v = 0;
            if (rem >= 8) {
                for (int i = 0; i < 8; i++) v = (v << 8) | d[pos + i];
                v >>= 8;
            } else {
                for (int i = 0; i < 7; i++) v = (v << 8) | d[pos + i];
            }
            value = v | (value << 56);
            bits += 56;
            pos += 7;
        } else if (pos < len) {
            bits += 8;
            value = (uint64_t)d[pos] | (value << 8);
            pos++;
        } else if (!eof) {
            value <<= 8;
            bits += 8;
            eof = true;
        } else {
            bits = 0;
        }
    }
    // branch-free: the decoded bit selects the new range and the value
    // update by masks (a data-dependent branch here mispredicts on every
    // other token bit; 25 % faster measured on 1080p streams)
    inline int bit(int prob)
    {
        if (bits < 0) load();
        const uint32_t r = range;
        const int p = bits;
        const uint32_t split = (r * (uint32_t)prob) >> 8;
        const uint32_t v = (uint32_t)(value >> p);
        const uint32_t b = v > split;
        const uint32_t m = 0u - b;  // all ones when the bit is 1
        const uint32_t nr = ((r - split) & m) | ((split + 1) & ~m);
        value -= (uint64_t)((split + 1) & m) << p;
        const int shift = 7 ^ (31 ^ __builtin_clz(nr));
        bits -= shift;
        range = (nr << shift) - 1;
        return (int)b;
    }
    int lit(int n)
    {
        int v = 0;
        for (int i = 0; i < n; i++) v = (v << 1) | bit(128);
        return v;
    }
    int sgn(int n)
    {
        if (!bit(128)) return 0;
        const int m = lit(n);
        return bit(128) ? -m : m;
    }
    int tree(const int8_t* t, const uint8_t* probs)
    {
        int i = 0;
        for (;;) {
            const int n = t[i + bit(probs[i >> 1])];
            if (n <= 0) return -n;
            i = n;
        }
    }
};

struct DecFrame {
    int width = 0, height = 0, mbw = 0, mbh = 0;
    int filter_type = 0, filter_level = 0, sharpness = 0;
    int segments_enabled = 0, seg_update_map = 0, seg_delta_values = 0;
    int lf_adj_enabled = 0, ref_delta0 = 0, mode_delta0 = 0;
    int8_t seg_quant[4] = {0, 0, 0, 0}, seg_lf[4] = {0, 0, 0, 0};
    uint8_t seg_probs[3] = {255, 255, 255};
    int nparts = 1;
    int skip_prob = -1;
    DecQuant q[4];
    uint8_t probs[4][8][3][11];
    BitReader hdr;
    BitReader part[8];
};

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// read_frame_header decoder/vp8.rs:553-670 (+ partitions :421-450, quant :452-504)
static int parse_header(DecFrame& F, const uint8_t* data, size_t len)
{
    if (len < 3) return ZW_EBITSTREAM;
    const uint32_t tag = data[0] | (data[1] << 8) | (data[2] << 16);
    if (tag & 1) return ZW_EUNSUPPORTED_FEATURE;  // interframes
    const uint32_t fps = tag >> 5;
    if (len < 6) return ZW_EBITSTREAM;
    if (data[3] != 0x9d || data[4] != 0x01 || data[5] != 0x2a) return ZW_EVP8_MAGIC;
    if (len < 10) return ZW_EBITSTREAM;
    F.width = (data[6] | (data[7] << 8)) & 0x3fff;
    F.height = (data[8] | (data[9] << 8)) & 0x3fff;
    F.mbw = (F.width + 15) / 16;
    F.mbh = (F.height + 15) / 16;
    size_t off = 10;
    if (len - off < fps) return ZW_EBITSTREAM;
    if (fps == 0) return ZW_ENOT_ENOUGH_INIT_DATA;
    BitReader& b = F.hdr;
    b.init(data + off, fps);
    off += fps;
    const int cs = b.lit(1);
    (void)b.lit(1);
    if (cs != 0) return ZW_ECOLORSPACE;
    F.segments_enabled = b.bit(128);
    int delta_values[4] = {0, 0, 0, 0};
    if (F.segments_enabled) {
        F.seg_update_map = b.bit(128);
        if (b.bit(128)) {
            const int mode = b.bit(128);
            for (int i = 0; i < 4; i++) delta_values[i] = !mode;
            for (int i = 0; i < 4; i++) F.seg_quant[i] = (int8_t)b.sgn(7);
            for (int i = 0; i < 4; i++) F.seg_lf[i] = (int8_t)b.sgn(6);
        }
        if (F.seg_update_map)
            for (int i = 0; i < 3; i++) F.seg_probs[i] = b.bit(128) ? (uint8_t)b.lit(8) : 255;
        if (b.eof) return ZW_EBITSTREAM;
    }
    F.filter_type = b.bit(128);
    F.filter_level = b.lit(6);
    F.sharpness = b.lit(3);
    F.lf_adj_enabled = b.bit(128);
    if (F.lf_adj_enabled) {
        if (b.bit(128)) {
            int rd[4], md[4];
            for (int i = 0; i < 4; i++) rd[i] = b.sgn(6);
            for (int i = 0; i < 4; i++) md[i] = b.sgn(6);
            F.ref_delta0 = rd[0];
            F.mode_delta0 = md[0];
        }
        if (b.eof) return ZW_EBITSTREAM;
    }
    F.nparts = 1 << b.lit(2);
    if (b.eof) return ZW_EBITSTREAM;
    const size_t sz_off = off;
    if (F.nparts > 1) {
        if (len - off < (size_t)(3 * F.nparts - 3)) return ZW_EBITSTREAM;
        off += 3 * F.nparts - 3;
    }
    for (int p = 0; p < F.nparts; p++) {
        size_t psz;
        if (p < F.nparts - 1) {
            const uint8_t* s = data + sz_off + 3 * p;
            psz = s[0] | (s[1] << 8) | (s[2] << 16);
            if (len - off < psz) return ZW_EBITSTREAM;
        } else {
            psz = len - off;
        }
        F.part[p].init(data + off, psz);
        off += psz;
    }
    const int yac = b.lit(7);
    const int ydc_d = b.sgn(4), y2dc_d = b.sgn(4), y2ac_d = b.sgn(4), uvdc_d = b.sgn(4), uvac_d = b.sgn(4);
    const int n = F.segments_enabled ? 4 : 1;
    for (int i = 0; i < n; i++) {
        const int base = F.segments_enabled ? (delta_values[i] ? F.seg_quant[i] + yac : F.seg_quant[i]) : yac;
        DecQuant& s = F.q[i];
        s.ydc = DC_QUANT[clampi(base + ydc_d, 0, 127)];
        s.yac = AC_QUANT[clampi(base, 0, 127)];
        s.y2dc = DC_QUANT[clampi(base + y2dc_d, 0, 127)] * 2;
        s.y2ac = AC_QUANT[clampi(base + y2ac_d, 0, 127)] * 155 / 100;
        s.uvdc = DC_QUANT[clampi(base + uvdc_d, 0, 127)];
        s.uvac = AC_QUANT[clampi(base + uvac_d, 0, 127)];
        if (s.y2ac < 8) s.y2ac = 8;
        if (s.uvdc > 132) s.uvdc = 132;
    }
    for (int i = n; i < 4; i++) F.q[i] = F.q[0];
    if (b.eof) return ZW_EBITSTREAM;
    (void)b.lit(1);  // refresh_entropy_probs
    memcpy(F.probs, COEFF_PROBS, sizeof F.probs);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++)
            for (int k = 0; k < 3; k++)
                for (int t = 0; t < 11; t++)
                    if (b.bit(COEFF_UPDATE_PROBS[i][j][k][t])) F.probs[i][j][k][t] = (uint8_t)b.lit(8);
    if (b.eof) return ZW_EBITSTREAM;
    F.skip_prob = b.lit(1) ? b.lit(8) : -1;
    if (b.eof) return ZW_EBITSTREAM;
    F.seg_delta_values = delta_values[0];
    return ZW_OK;
}

// read_coefficients decoder/vp8.rs:872-1058: one block's levels (not
// dequantised), written as the zigzag prefix straight into dst (the packed
// record's level array, zw_common.h ZW_DREC_*): positions 0..eob-1, zeros
// included (position 0 is 0 when first = 1); *eob = last nonzero position + 1.
// Returns -1 on eof, else whether the run was non-empty.
static int read_levels_into(BitReader& r, const uint8_t P[8][3][11], int16_t* dst, int first, int ctx, int* eob)
{
    *eob = 0;
    int n = first, written = 0;
    const uint8_t* p = P[COEFF_BANDS[n]][ctx];
    while (n < 16) {
        if (!r.bit(p[0])) break;
        while (!r.bit(p[1])) {
            n++;
            if (n >= 16) return r.eof ? -1 : 1;
            p = P[COEFF_BANDS[n]][0];
        }
        int v, nctx;
        if (!r.bit(p[2])) {
            v = 1;
            nctx = 1;
        } else {
            if (!r.bit(p[3])) {
                if (!r.bit(p[4])) v = 2;
                else v = 3 + r.bit(p[5]);
            } else if (!r.bit(p[6])) {
                if (!r.bit(p[7])) v = 5 + r.bit(159);
                else {
                    v = 7 + 2 * r.bit(165);
                    v += r.bit(145);
                }
            } else {
                const int b1 = r.bit(p[8]);
                const int b0 = r.bit(p[9 + b1]);
                const int cat = 2 * b1 + b0;
                const uint8_t* cp = PROB_DCT_CAT[2 + cat];
                int extra = 0;
                for (int k = 0; k < 12 && cp[k]; k++) extra = extra + extra + r.bit(cp[k]);
                v = 3 + (8 << cat) + extra;
            }
            nctx = 2;
        }
        while (written < n) dst[written++] = 0;
        dst[n] = (int16_t)(r.bit(128) ? -v : v);
        written = n + 1;
        n++;
        *eob = n;
        if (n < 16) p = P[COEFF_BANDS[n]][nctx];
    }
    if (r.eof) return -1;
    return n > first;
}

// MB headers + tokens for the whole frame (decoder/vp8.rs:681-734, :1060-1168),
// as packed records in raster order into recs (room for nmb * ZW_DREC_MAX
// bytes); moff[i] = byte offset of MB i's record (moff[nmb] = total).
static int parse_mbs(DecFrame& F, uint8_t* recs, uint32_t* moff)
{
    size_t used = 0;
    const int mbw = F.mbw, mbh = F.mbh;
    std::vector<uint8_t> top_cx((size_t)mbw * 9, 0), top_bp((size_t)mbw * 4, 0);
    BitReader& b = F.hdr;
    for (int mby = 0; mby < mbh; mby++) {
        BitReader& pr = F.part[mby % F.nparts];
        uint8_t left_cx[9] = {0}, left_bp[4] = {0};
        for (int mbx = 0; mbx < mbw; mbx++) {
            moff[(size_t)mby * mbw + mbx] = (uint32_t)used;
            // the record is built in place: header, level starts, levels
            uint8_t* rec = recs + used;
            memset(rec, 0, ZW_DREC_HDR);
            uint16_t* start = (uint16_t*)(rec + 16);
            int16_t* lv = (int16_t*)(rec + ZW_DREC_HDR);
            uint8_t* tcx = &top_cx[(size_t)mbx * 9];
            uint8_t* tbp = &top_bp[(size_t)mbx * 4];
            int seg = 0;
            if (F.segments_enabled && F.seg_update_map) seg = b.tree(SEGMENT_ID_TREE, F.seg_probs);
            const int skip = F.skip_prob >= 0 ? b.bit(F.skip_prob) : 0;
            const int lm = b.tree(YMODE_TREE, KEYFRAME_YMODE_PROBS);
            if (lm == 4) {
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) {
                        const int m = b.tree(BMODE_TREE, KEYFRAME_BPRED_MODE_PROBS[tbp[x]][left_bp[y]]);
                        rec[8 + ((x + y * 4) >> 1)] |= (uint8_t)(m << (4 * ((x + y * 4) & 1)));
                        tbp[x] = (uint8_t)m;
                        left_bp[y] = (uint8_t)m;
                    }
            } else {
                static const uint8_t intra_of[4] = {0, 2, 3, 1};  // DC,V,H,TM -> B_DC,B_VE,B_HE,B_TM
                for (int i = 0; i < 4; i++) tbp[i] = left_bp[i] = intra_of[lm];
            }
            const int cm = b.tree(UVMODE_TREE, KEYFRAME_UV_MODE_PROBS);
            if (b.eof) return ZW_EBITSTREAM;
            rec[0] = (uint8_t)(lm | (cm << 3) | (skip << 5));
            rec[1] = (uint8_t)seg;
            if (skip) {
                if (lm != 4) left_cx[0] = tcx[0] = 0;
                for (int i = 1; i < 9; i++) left_cx[i] = tcx[i] = 0;
                used += ZW_DREC_HDR;  // no levels (every start 0); 80 is a multiple of 16
                continue;
            }
            uint32_t nzm = 0;
            int first = 0, eob, nlv = 0;
            if (lm != 4) {  // Y2 (parsed first) goes first
                const int nz = read_levels_into(pr, F.probs[1], lv, 0, tcx[0] + left_cx[0], &nlv);
                if (nz < 0) return ZW_EBITSTREAM;
                left_cx[0] = tcx[0] = (uint8_t)nz;
                first = 1;
            }
            auto block = [&](int i, const uint8_t P[8][3][11], int fst, int ctx) -> int {
                start[i] = (uint16_t)nlv;
                const int nz = read_levels_into(pr, P, lv + nlv, fst, ctx, &eob);
                if (nz > 0 && fst == 1) lv[nlv] = 0;  // position 0 of an I16 luma block
                nlv += eob;
                return nz;
            };
            const int plane = lm != 4 ? 0 : 3;
            for (int y = 0; y < 4; y++) {
                int left = left_cx[y + 1];
                for (int x = 0; x < 4; x++) {
                    const int i = x + y * 4;
                    const int nz = block(i, F.probs[plane], first, tcx[x + 1] + left);
                    if (nz < 0) return ZW_EBITSTREAM;
                    nzm |= (uint32_t)nz << i;
                    left = nz;
                    tcx[x + 1] = (uint8_t)nz;
                }
                left_cx[y + 1] = (uint8_t)left;
            }
            for (int j = 5; j <= 7; j += 2) {
                for (int y = 0; y < 2; y++) {
                    int left = left_cx[y + j];
                    for (int x = 0; x < 2; x++) {
                        const int i = x + y * 2 + (j == 5 ? 16 : 20);
                        const int nz = block(i, F.probs[2], 0, tcx[x + j] + left);
                        if (nz < 0) return ZW_EBITSTREAM;
                        nzm |= (uint32_t)nz << i;
                        left = nz;
                        tcx[x + j] = (uint8_t)nz;
                    }
                    left_cx[y + j] = (uint8_t)left;
                }
            }
            start[24] = (uint16_t)nlv;  // the end of block 23
            memcpy(rec + 4, &nzm, 4);
            const size_t bytes = ZW_DREC_HDR + (size_t)nlv * 2, padded = (bytes + 15) & ~(size_t)15;
            memset(rec + bytes, 0, padded - bytes);
            used += padded;
        }
    }
    moff[(size_t)mbw * mbh] = (uint32_t)used;
    return ZW_OK;
}

// The first partition's half of parse_mbs for the device token parse
// (k_dec_tokl): each MB's modes, segment, skip flag and I4 sub-modes as the
// first ZW_TOK_MODE bytes of its record header (decoder/vp8.rs:681-734), from
// the same bool decoder in the same order, so the same streams fail.
static int parse_modes(DecFrame& F, uint8_t* mrec)
{
    const int mbw = F.mbw, mbh = F.mbh;
    std::vector<uint8_t> top_bp((size_t)mbw * 4, 0);
    BitReader& b = F.hdr;
    for (int mby = 0; mby < mbh; mby++) {
        uint8_t left_bp[4] = {0};
        for (int mbx = 0; mbx < mbw; mbx++) {
            uint8_t* rec = mrec + ((size_t)mby * mbw + mbx) * ZW_TOK_MODE;
            memset(rec, 0, ZW_TOK_MODE);
            uint8_t* tbp = &top_bp[(size_t)mbx * 4];
            int seg = 0;
            if (F.segments_enabled && F.seg_update_map) seg = b.tree(SEGMENT_ID_TREE, F.seg_probs);
            const int skip = F.skip_prob >= 0 ? b.bit(F.skip_prob) : 0;
            const int lm = b.tree(YMODE_TREE, KEYFRAME_YMODE_PROBS);
            if (lm == 4) {
                for (int y = 0; y < 4; y++)
                    for (int x = 0; x < 4; x++) {
                        const int m = b.tree(BMODE_TREE, KEYFRAME_BPRED_MODE_PROBS[tbp[x]][left_bp[y]]);
                        rec[8 + ((x + y * 4) >> 1)] |= (uint8_t)(m << (4 * ((x + y * 4) & 1)));
                        tbp[x] = (uint8_t)m;
                        left_bp[y] = (uint8_t)m;
                    }
            } else {
                static const uint8_t intra_of[4] = {0, 2, 3, 1};  // DC,V,H,TM -> B_DC,B_VE,B_HE,B_TM
                for (int i = 0; i < 4; i++) tbp[i] = left_bp[i] = intra_of[lm];
            }
            const int cm = b.tree(UVMODE_TREE, KEYFRAME_UV_MODE_PROBS);
            if (b.eof) return ZW_EBITSTREAM;
            rec[0] = (uint8_t)(lm | (cm << 3) | (skip << 5));
            rec[1] = (uint8_t)seg;
        }
    }
    return ZW_OK;
}

// calculate_filter_parameters decoder/vp8.rs:1470-1523, tabulated per
// (segment, is_i4).
static void filter_table(ZwFilterParams& fp, int filter_type, int filter_level, int sharpness, int seg_enabled,
                         int seg_delta, const int8_t* seg_lf, int adj, int ref_delta0, int mode_delta0, int mbw, int mbh)
{
    memset(&fp, 0, sizeof fp);
    fp.filter_type = filter_type;
    fp.mbw = mbw;
    fp.mbh = mbh;
    for (int s = 0; s < 4; s++)
        for (int i4 = 0; i4 < 2; i4++) {
            int fl = filter_level, L = 0, I = 0, H = 0;
            if (fl != 0) {
                if (seg_enabled) fl = seg_delta ? fl + seg_lf[s] : seg_lf[s];
                fl = clampi(fl, 0, 63);
                if (adj) {
                    fl += ref_delta0;
                    if (i4) fl += mode_delta0;
                }
                fl = clampi(fl, 0, 63);
                int il = fl;
                if (sharpness > 0) {
                    il >>= sharpness > 4 ? 2 : 1;
                    if (il > 9 - sharpness) il = 9 - sharpness;
                }
                if (il == 0) il = 1;
                L = fl;
                I = il;
                H = fl >= 40 ? 2 : (fl >= 15 ? 1 : 0);
            }
            fp.level[s][i4] = (uint8_t)L;
            fp.ilimit[s][i4] = (uint8_t)I;
            fp.hev[s][i4] = (uint8_t)H;
        }
}

static size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

// Decoded frame buffers (zw_frame.y, and decode_rgb_batch's zw_bytes) are
// recycled.  A fresh multi-MB malloc is first touched by the fan-out's copy,
// so each of its 4 KB pages faults and is zeroed by the kernel, on the same
// host threads the bool decoder needs (1024 1080p frames on the box: 4 474-
// 5 022 decodes/s with fresh buffers, 5 132-5 221 recycled).  zw_frame_free /
// zw_bytes_free hand a buffer back to this process-wide pool (keyed by size,
// bounded by ZW_DEC_POOL_MB, default 4096; 0 = off) and the next batch of that
// size takes it.  Only while a context is alive: the last zw_ctx_destroy (and
// every zw_ctx_release_buffers) frees what the pool holds, and buffers freed
// after that go straight back to free().  Buffers the pool handed out are tracked, so zw_bytes_free
// still free()s the encoder's outputs.  (bench decode_path, 1024 1080p
// frames: fan-out 96 -> 67 ms, 5 013 -> 5 289 decodes/s.)
struct FramePool {
    std::mutex m;
    std::unordered_map<size_t, std::vector<uint8_t*>> free_;
    std::unordered_map<uint8_t*, size_t> live;
    size_t bytes = 0, cap = 0;
    FramePool()
    {
        const char* e = getenv("ZW_DEC_POOL_MB");
        cap = (size_t)(e ? std::max(0L, atol(e)) : 4096L) << 20;
    }
    uint8_t* get(size_t n)
    {
        std::lock_guard<std::mutex> g(m);
        uint8_t* p = nullptr;
        auto it = free_.find(n);
        if (it != free_.end() && !it->second.empty()) {
            p = it->second.back();
            it->second.pop_back();
            bytes -= n;
        } else {
            p = (uint8_t*)malloc(n);
            if (!p) return nullptr;
        }
        live[p] = n;
        return p;
    }
    // frees every buffer the pool holds (those handed out stay tracked)
    void trim()
    {
        std::vector<uint8_t*> drop;
        {
            std::lock_guard<std::mutex> g(m);
            for (auto& kv : free_)
                for (uint8_t* b : kv.second) drop.push_back(b);
            free_.clear();
            bytes = 0;
        }
        for (uint8_t* b : drop) free(b);
    }
    // false: p did not come from the pool.  Over the cap, buffers of other
    // sizes are dropped first (the latest frame size is the one reused).
    bool put(void* q)
    {
        uint8_t* p = (uint8_t*)q;
        std::vector<uint8_t*> drop;
        {
            std::lock_guard<std::mutex> g(m);
            auto it = live.find(p);
            if (it == live.end()) return false;
            const size_t n = it->second;
            live.erase(it);
            if (!zw_ctx_any_alive()) {
                free(p);
                return true;
            }
            for (auto& kv : free_) {
                while (bytes + n > cap && kv.first != n && !kv.second.empty()) {
                    drop.push_back(kv.second.back());
                    kv.second.pop_back();
                    bytes -= kv.first;
                }
            }
            if (bytes + n <= cap) {
                free_[n].push_back(p);
                bytes += n;
                p = nullptr;
            }
        }
        for (uint8_t* d : drop) free(d);
        free(p);
        return true;
    }
};
// never destroyed: Python finalizers may free frames during interpreter exit
static FramePool& frame_pool()
{
    static FramePool* P = new FramePool();
    return *P;
}

}  // namespace

bool zw_dec_pool_put(void* p) { return frame_pool().put(p); }
void zw_dec_pool_trim() { frame_pool().trim(); }

extern "C" void zw_frame_free(zw_frame* f)
{
    if (f && f->y) {
        if (!frame_pool().put(f->y)) free(f->y);
        f->y = f->u = f->v = nullptr;
    }
}

// Decoded planes of a batch, resident in the context's device scratch.
struct DecBatch {
    std::vector<DecFrame> F;
    hipEvent_t* ev = nullptr;  // [0] recon start, [1] recon done, [2] filter done, [3] caller's
    uint8_t* d = nullptr;  // device scratch base
    size_t o_y = 0, o_u = 0, o_v = 0, o_extra = 0, ysz = 0, csz = 0;
    int mbw = 0, mbh = 0;
    const int* d_rs = nullptr;  // row-parallel kernels' per-frame sync words (null: workgroup-per-frame kernels)
    const int* d_terr = nullptr;  // k_dec_tokl's per-frame error words (null: the host parsed the tokens)
    int n = 0;
    // a chunk whose tokens the device parsed (DecTok): its records, MB offsets and
    // frame bases are in device memory already; the kernels wait for x_done
    const uint8_t* x_recs = nullptr;
    const uint32_t* x_moff = nullptr;
    const uint64_t* x_fbase = nullptr;
    hipEvent_t x_done = nullptr;
    // host parse results waiting for dec_launch
    std::vector<DecQuant> quant;
    std::vector<ZwFilterParams> fps;
    uint8_t* stage = nullptr;  // pinned upload staging (records, MB offsets, frame bases)
    size_t up_bytes = 0, o_moff = 0, o_base = 0, rec_bytes = 0;
    double parse_ms = 0;
};

// Test hook (ZW_DEC_FORCE_ERROR=1): pre-set frame 0's row-sync error word, as a
// wave that gave up waiting would, so the host-side check below is exercised.
static bool dec_force_error() { return getenv("ZW_DEC_FORCE_ERROR") != nullptr; }

// A row-parallel wave that gives up waiting (k_dec_recon_rows / k_loopfilter_rows
// bounded spins) reports through its frame's error word rowsync[f][2] instead of
// hanging the GPU; the planes of such a frame are incomplete.  Read the words
// after the kernels completed (SDMA: the kernel stream may already run the next
// chunk) and fail the call with ZW_EDEVICE.
static int tokens_error(zw_ctx* ctx, const int* d_terr, int n)
{
    if (!d_terr) return ZW_OK;
    int* e = (int*)ctx_pinned(ctx, 3, (size_t)n * sizeof(int));
    if (!e) return ZW_ENOMEM;
    if (int r = ctx_d2h(ctx, e, d_terr, (size_t)n * sizeof(int))) return r;
    for (int f = 0; f < n; f++) {
        if (e[f] == 1) return ZW_EBITSTREAM;  // a token partition ran out (parse_mbs: read_levels_into < 0)
        if (e[f]) {
            fprintf(stderr, "zwebp: device token parse gave up waiting on frame %d of %d\n", f, n);
            return ZW_EDEVICE;
        }
    }
    return ZW_OK;
}

static int rows_error(zw_ctx* ctx, const int* d_rs, int n, int mbh)
{
    if (!d_rs) return ZW_OK;
    const size_t words = (size_t)n * (4 + 2 * mbh);
    int* rs = (int*)ctx_pinned(ctx, 3, words * sizeof(int));
    if (!rs) return ZW_ENOMEM;
    if (int r = ctx_d2h(ctx, rs, d_rs, words * sizeof(int))) return r;
    for (int f = 0; f < n; f++)
        if (rs[(size_t)f * (4 + 2 * mbh) + 2]) {
            fprintf(stderr, "zwebp: row-parallel decode gave up waiting on frame %d of %d\n", f, n);
            return ZW_EDEVICE;
        }
    return ZW_OK;
}

// Vp8Decoder::decode_frame for n frames of identical dimensions, one device
// pass: host header/token parse (parallel over frames) -> k_dec_recon ->
// k_loopfilter.  Leaves the filtered planes in device scratch (plus
// `extra_bytes` of scratch at B.o_extra for the caller) with the kernel
// stream's work queued; dev_ev[2] marks the end of the loop filter.
static double dec_now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static bool dec_timing() { static const bool on = getenv("ZW_DEC_TIMING") != nullptr; return on; }

// bi: which of the context's two staging / scratch / event sets (the
// pipelined batches alternate between them).
// Host half: headers, modes and tokens of n frames into packed MB records in
// the pinned upload staging of set bi (no device work).
static int dec_parse(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, DecBatch& B, int bi)
{
    const double t0 = dec_now_ms();
    B.F.assign(n, DecFrame());
    std::vector<DecFrame>& F = B.F;
    std::vector<int> rc(n, ZW_OK);
    parallel_for(n, [&](int i) { rc[i] = parse_header(F[i], data[i], lens[i]); });
    for (int i = 0; i < n; i++)
        if (rc[i] != ZW_OK) return rc[i];
    const int mbw = F[0].mbw, mbh = F[0].mbh;
    for (int i = 1; i < n; i++)
        if (F[i].mbw != mbw || F[i].mbh != mbh) return ZW_EINVAL;
    if (mbw == 0 || mbh == 0) return ZW_EINVALID_DIMENSIONS;
    B.x_recs = nullptr;
    B.d_terr = nullptr;
    const size_t nmb = (size_t)mbw * mbh;
    const size_t ysz = nmb * 256, csz = nmb * 64;
    // packed MB records (zw_common.h ZW_DREC_*): each frame is parsed into its
    // own worst-case pageable buffer (only the pages written are touched), then
    // the used prefixes are packed back to back (256-B aligned frame bases) into
    // pinned staging sized by the measured bytes -- ~1 MB per 1080p frame at
    // Q75 instead of the 7 MB worst case -- followed by the MB offsets and the
    // frame bases; one upload carries all of it.
    const size_t slot = nmb * ZW_DREC_MAX;
    std::vector<uint32_t> moffv((size_t)n * (nmb + 1));
    std::vector<zw_ctx::RecBuf>& recs = ctx->dec_recs[bi];
    if (recs.size() < (size_t)n) recs.resize(n);
    std::vector<DecQuant>& quant = B.quant;
    std::vector<ZwFilterParams>& fps = B.fps;
    quant.assign((size_t)n * 4, DecQuant());
    fps.assign(n, ZwFilterParams());
    parallel_for(n, [&](int i) {
        if (recs[i].cap < slot) {
            recs[i].p.reset(new (std::nothrow) uint8_t[slot]);
            recs[i].cap = recs[i].p ? slot : 0;
            if (!recs[i].p) {
                rc[i] = ZW_ENOMEM;
                return;
            }
        }
        rc[i] = parse_mbs(F[i], recs[i].p.get(), moffv.data() + (size_t)i * (nmb + 1));
        for (int s = 0; s < 4; s++) quant[(size_t)i * 4 + s] = F[i].q[s];
        filter_table(fps[i], F[i].filter_type, F[i].filter_level, F[i].sharpness, F[i].segments_enabled,
                     F[i].seg_delta_values, F[i].seg_lf, F[i].lf_adj_enabled, F[i].ref_delta0, F[i].mode_delta0, mbw,
                     mbh);
    });
    for (int i = 0; i < n; i++)
        if (rc[i] != ZW_OK) return rc[i];
    std::vector<uint64_t> fb(n);
    size_t rec_bytes = 0, rec_span = 0;
    for (int i = 0; i < n; i++) {
        fb[i] = rec_span;
        const size_t used = moffv[(size_t)i * (nmb + 1) + nmb];
        rec_bytes += used;
        rec_span = al256(rec_span + used);
    }
    const size_t off_bytes = (size_t)n * (nmb + 1) * 4, base_bytes = (size_t)n * 8;
    const size_t o_moff = rec_span, o_base = o_moff + al256(off_bytes);
    const size_t up_bytes = o_base + base_bytes;
    uint8_t* stage = (uint8_t*)ctx_pinned(ctx, bi ? 2 : 0, up_bytes);
    if (!stage) return ZW_ENOMEM;
    parallel_for(n, [&](int i) {
        memcpy(stage + fb[i], recs[i].p.get(), moffv[(size_t)i * (nmb + 1) + nmb]);
    });
    memcpy(stage + o_moff, moffv.data(), off_bytes);
    memcpy(stage + o_base, fb.data(), base_bytes);
    B.stage = stage;
    B.up_bytes = up_bytes;
    B.o_moff = o_moff;
    B.o_base = o_base;
    B.rec_bytes = rec_bytes;
    B.mbw = mbw;
    B.mbh = mbh;
    B.ysz = ysz;
    B.csz = csz;
    B.n = n;
    B.parse_ms = dec_now_ms() - t0;
    return ZW_OK;
}

// Device half: upload set bi's records, reconstruct, filter (leaving
// `extra_bytes` of scratch at B.o_extra for the caller).
static int dec_launch(zw_ctx* ctx, size_t extra_bytes, DecBatch& B, int bi)
{
    const double t1 = dec_now_ms();
    const int n = B.n, mbw = B.mbw, mbh = B.mbh;
    const size_t nmb = (size_t)mbw * mbh, ysz = B.ysz, csz = B.csz;
    const size_t up_bytes = B.up_bytes, o_moff = B.o_moff, o_base = B.o_base;
    const std::vector<DecQuant>& quant = B.quant;
    const std::vector<ZwFilterParams>& fps = B.fps;
    uint8_t* stage = B.stage;
    HIPOK(hipSetDevice(ctx->device));
    const size_t o_mbs = 0, o_q = al256(o_mbs + up_bytes);
    const size_t o_fp = al256(o_q + quant.size() * sizeof(DecQuant));
    const size_t o_fl = al256(o_fp + fps.size() * sizeof(ZwFilterParams));
    const size_t o_y = al256(o_fl + (size_t)n * nmb * 4);
    const size_t o_u = al256(o_y + (size_t)n * ysz), o_v = al256(o_u + (size_t)n * csz);
    // Small batches run the row-parallel kernels (one wave per MB row, the x+2y
    // wavefront spread over up to mbh CUs); large ones fill the GPU with one
    // workgroup per frame.  ZW_DEC_ROWS=0/1 forces either.
    const int rows_env = getenv("ZW_DEC_ROWS") ? atoi(getenv("ZW_DEC_ROWS")) : -1;
    const bool rows = rows_env >= 0 ? rows_env != 0 : n < 128;  // measured: rows faster up to 64, slower at 256
    const size_t o_rs = al256(o_v + (size_t)n * csz);
    const size_t o_bd = al256(o_rs + (rows ? zw_dec_rows_sync_bytes(mbh, n) : 0));
    const size_t o_t = al256(o_bd + (rows ? zw_dec_rows_border_bytes(mbw, n) : 0));  // batch: recon -> filter MB tiles
    const size_t o_extra = al256(o_t + (rows ? 0 : (size_t)n * nmb * 384));
    const size_t total = al256(o_extra + extra_bytes);
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total, bi);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    hipEvent_t* ev = bi ? ctx->dev_ev1 : ctx->dev_ev;
    B.ev = ev;
    if (up_bytes) HIPOK(hipMemcpyAsync(d + o_mbs, stage, up_bytes, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_q, quant.data(), quant.size() * sizeof(DecQuant), hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_fp, fps.data(), fps.size() * sizeof(ZwFilterParams), hipMemcpyHostToDevice, s));
    for (int e = 0; e < 4; e++)  // blocking sync: finish() sleeps on them (ctx_d2h_stream)
        if (!ev[e]) HIPOK(hipEventCreateWithFlags(&ev[e], hipEventBlockingSync));
    // the kernels read the packed records straight from the upload, or, for a
    // chunk whose tokens the device parsed, from k_dec_tokl's output
    const uint8_t* recs = d + o_mbs;
    const uint32_t* moff = (const uint32_t*)(d + o_mbs + o_moff);
    const uint64_t* fbase = (const uint64_t*)(d + o_mbs + o_base);
    if (B.x_recs) {
        HIPOK(hipStreamWaitEvent(s, B.x_done, 0));
        recs = B.x_recs;
        moff = B.x_moff;
        fbase = B.x_fbase;
    } else if (const char* dump = getenv("ZW_DEC_TOKENS_DUMP")) {  // debug: frame 0's host records to <dump>.host
        const uint32_t* mo = (const uint32_t*)(stage + o_moff);
        std::string p0 = std::string(dump) + ".host";
        if (FILE* fo = fopen(p0.c_str(), "wb")) {
            fwrite(mo, 4, nmb + 1, fo);
            fwrite(stage, 1, mo[nmb], fo);
            fclose(fo);
        }
    }
    HIPOK(hipEventRecord(ev[0], s));
    // two wavefront kernels (a fused recon + filter wavefront measured slower: the
    // per-MB latencies add up in one chain, and its registers spilled)
    if (rows) {
        int* rs = (int*)(d + o_rs);
        HIPOK(zwk_dec_rows_init(s, rs, mbh, n));
        if (dec_force_error()) HIPOK(hipMemsetAsync(rs + 2, 1, sizeof(int), s));
        HIPOK(zwk_dec_rows(s, 1, recs, moff, fbase, d + o_q, d + o_y, d + o_u, d + o_v, d + o_fl,
                           (const ZwFilterParams*)(d + o_fp), mbw, mbh, ysz, csz, n, rs, d + o_bd, mbh));
        HIPOK(hipEventRecord(ev[1], s));
        HIPOK(zwk_dec_rows(s, 2, nullptr, nullptr, nullptr, d + o_q, d + o_y, d + o_u, d + o_v, d + o_fl,
                           (const ZwFilterParams*)(d + o_fp), mbw, mbh, ysz, csz, n, rs, d + o_bd, mbh));
    } else {
        HIPOK(zwk_dec_recon(s, recs, moff, fbase, d + o_q, d + o_y, d + o_u, d + o_v, d + o_fl, mbw, mbh, ysz, csz, n,
                            d + o_t));
        HIPOK(hipEventRecord(ev[1], s));
        HIPOK(zwk_loopfilter(s, d + o_y, d + o_u, d + o_v, d + o_fl, (const ZwFilterParams*)(d + o_fp), ysz, csz, n, mbw,
                             d + o_t));
    }
    HIPOK(hipEventRecord(ev[2], s));
    if (dec_timing()) {
        HIPOK(hipEventSynchronize(ev[2]));
        fprintf(stderr, "[dec] n=%d parse %.2f ms, upload+kernels %.2f ms (records %.1f MB)\n", n, B.parse_ms,
                dec_now_ms() - t1, B.rec_bytes / 1e6);
    }
    B.d = d;
    B.o_y = o_y;
    B.o_u = o_u;
    B.o_v = o_v;
    B.o_extra = o_extra;
    B.d_rs = rows ? (const int*)(d + o_rs) : nullptr;
    return ZW_OK;
}

// Parts a chunk's plane download is split into, each fanned out while the next
// lands (ZW_DEC_DL_PARTS).
static int dec_dl_parts()
{
    const char* e = getenv("ZW_DEC_DL_PARTS");
    const int p = e ? atoi(e) : 4;  // 1024 1080p frames: 4 901 vs 4 724 decodes/s with one part
    return p > 0 ? p : 4;
}

// A chunk's download in parts on a second thread, each part (frames [a, b))
// handed to fan(a, b) as soon as copy(a, b) has landed it, so the fan-out into
// the callers' buffers overlaps the rest of the download.  Returns the first
// copy error; *dl_ms = the download's wall time.
template <class CP, class FAN>
static int dec_download_fan(zw_ctx* ctx, int cn, CP&& copy, FAN&& fan, double* dl_ms)
{
    const int parts = std::max(1, std::min(cn, dec_dl_parts()));
    std::mutex mu;
    std::condition_variable cv;
    int landed = 0, err = ZW_OK;
    const double t0 = dec_now_ms();
    std::thread dl([&]() {
        (void)hipSetDevice(ctx->device);
        for (int p = 0; p < parts; p++) {
            const int r = copy(cn * p / parts, cn * (p + 1) / parts);
            std::lock_guard<std::mutex> g(mu);
            if (r) {
                err = r;
                break;
            }
            landed = p + 1;
            cv.notify_one();
        }
        *dl_ms = dec_now_ms() - t0;
        std::lock_guard<std::mutex> g(mu);
        landed = parts + 1;  // (done, or stopped on an error)
        cv.notify_one();
    });
    // the waiting thread sleeps (a spinning one took a CPU from the parse threads)
    for (int p = 0; p < parts; p++) {
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return landed > p || err != ZW_OK; });
            if (err != ZW_OK) break;
        }
        fan(cn * p / parts, cn * (p + 1) / parts);
    }
    dl.join();
    return err;
}

// Threads of a fan-out part (ZW_DEC_FAN_THREADS; 0 = every host thread).  The
// copies into recycled buffers run beside the next chunk's parse; capping them
// did not help it (1 024 1080p frames: all 16 threads 5 061-5 120 decodes/s,
// 8: 5 018-5 107, 4: 4 753-4 873; profiles/r04_dec_fan_ab.txt).
static int dec_fan_threads()
{
    static const int t = [] {
        const char* e = getenv("ZW_DEC_FAN_THREADS");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    return t;
}

// Frames per pipelined chunk.  ZW_DEC_CHUNK overrides.
static int dec_chunk_frames()
{
    const char* e = getenv("ZW_DEC_CHUNK");
    const int c = e ? atoi(e) : 128;  // measured on 256 1080p frames: 32 / 64 / 128 / 256 -> 3198 / 3559 / 3771 / 3267 per s
    return c > 0 ? c : 128;
}

// ---------------------------------------------------------------------------
// Device token parse (zw_dec_tokens.hip) for the tail of a batch.  A frame's
// token partition is one serial chain of bool decisions: ≈2.7 ms on a host core
// for a 1080p Q75 frame, much longer on one GPU lane, but one launch runs 64
// frames per wave side by side, so its time hardly depends on how many frames it
// holds.  So a batch splits: the frames [h0, n) are header/mode-parsed on the
// host up front (the first partition, a short chain) and their tokens go to the
// device on its own stream, while the chunk pipeline parses the frames [0, h0)
// on the host as before; the device chunks' reconstruction waits for the
// device's records.  The device parse runs in two stages: k_dec_tok1 (the
// decision chains alone, a snapshot per MB) and k_dec_tok2 (every MB replayed
// from its snapshot in parallel: a count pass, offsets, then the records into a
// buffer sized from the count, so the records take what they use -- ≈1 MB per
// 1080p Q75 frame -- and no worst-case slots).  By default (auto) the host keeps
// as many whole chunks as it parses in the device's time, from the rates the
// last batches measured, and the device takes the rest (none when the host
// alone would finish first).  ZW_DEC_TOKENS=host / device / mixed forces the
// host, the device or a split at ZW_DEC_TOKENS_HOST (the host's share, 0.5).
//
// Device memory the parse keeps in the context after a batch (freed by
// zw_ctx_release_buffers / zw_ctx_destroy; grow-only between): per device frame
// its partition, modes (16 B per MB), probabilities, a 16-byte snapshot and a
// 4-byte size and offset per MB (≈0.4 MB per 1080p frame) plus its records.
// ---------------------------------------------------------------------------
struct DecTok {
    int h0 = 0, nd = 0;  // device frames [h0, h0 + nd)
    std::vector<DecFrame> F;
    std::vector<DecQuant> quant;
    std::vector<ZwFilterParams> fps;
    size_t nmb = 0;
    // device buffers of the write pass (ctx_scratch_tok)
    uint8_t* d = nullptr;
    size_t o_b = 0, o_tf = 0, o_p = 0, o_m = 0, o_sn = 0, o_e1 = 0;
    const uint32_t* moff = nullptr;
    const uint64_t* fbase = nullptr;
    const int* err = nullptr;
    // set by dec_tok_finish
    const uint8_t* recs = nullptr;
    hipEvent_t done = nullptr;
    int state = 0;  // 0 launched (count), 1 records queued, -1 failed (the host parses the rest)
};

// The host's frames [0, h0) of a batch of n frames of nmb MBs (C frames per chunk).
static int dec_tok_split(zw_ctx* ctx, int n, int C, size_t nmb)
{
    const char* e = getenv("ZW_DEC_TOKENS");
    const int force = !e ? -1 : (!strcmp(e, "device") ? 1 : (!strcmp(e, "host") ? 0 : (!strcmp(e, "mixed") ? 2 : -1)));
    if (force == 0) return n;
    if (force == 1) return 0;
    if (force == 2) {
        const char* h = getenv("ZW_DEC_TOKENS_HOST");
        const double frac = h ? atof(h) : 0.5;
        return std::max(0, std::min(n, (int)(n * frac) / C * C));  // whole host chunks
    }
    // auto.  Defaults until measured: 0.19 ms of chunk time per 1080p frame (16 host
    // threads) and a 100 ms device parse for 1080p frames
    const double host_f = ctx->dec_host_ms_per_frame > 0 ? ctx->dec_host_ms_per_frame : 0.19 * (double)nmb / 8160.0;
    const double tok = (ctx->dec_tok_ms_per_mb > 0 ? ctx->dec_tok_ms_per_mb : 100.0 / 8160.0) * (double)nmb;
    const double tail = 0.06 * tok;  // the device frames' reconstruction and download after the parse, per frame of
                                     // host work that the parse's length leaves (an estimate; errs toward the host)
    if (n * host_f <= tok + tail) return n;  // the host alone finishes first
    const int h0 = (int)(tok / host_f) / C * C;
    return std::max(0, std::min(n, h0));
}

// Parses the headers and modes of frames [h0, n), stages them and launches the
// device parse's first half (stage 1, the count pass, offsets) on the context's
// token stream.  Returns false (and leaves the frames to the host chunks, which
// then report any error in frame order) when a frame has several token
// partitions, another size, or a header / mode error.
static bool dec_tok_prepare(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, int h0, DecTok& T)
{
    const int nd = n - h0;
    if (nd <= 0) return false;
    T.F.assign(nd, DecFrame());
    std::vector<DecFrame>& F = T.F;
    std::vector<int> rc(nd, ZW_OK);
    parallel_for(nd, [&](int i) { rc[i] = parse_header(F[i], data[h0 + i], lens[h0 + i]); });
    for (int i = 0; i < nd; i++)
        if (rc[i] != ZW_OK || F[i].nparts != 1 || F[i].mbw != F[0].mbw || F[i].mbh != F[0].mbh || F[i].mbw == 0 ||
            F[i].mbh == 0)
            return false;
    const int mbw = F[0].mbw, mbh = F[0].mbh;
    // stage 1 keeps per-lane top contexts in LDS (very wide frames stay on the host) and
    // addresses a wave's 64 frames of snapshots through one buffer (< 2 GB)
    const size_t nmb = (size_t)mbw * mbh, ncw = (nmb + 15) / 16;
    if (mbw < 2 || zw_tok1_lds_bytes(mbw) > 160 * 1024 || 64 * nmb * 16 >= ((size_t)1 << 31)) return false;
    const size_t probs_b = (size_t)tokl::PROBS;
    std::vector<size_t> boff(nd);
    size_t blob = 0;
    for (int i = 0; i < nd; i++) {
        boff[i] = blob;
        blob += (F[i].part[0].len + 15) & ~(size_t)15;
    }
    blob += 16;  // (16 zero bytes at the end)
    const size_t o_m = 0, o_c = al256(o_m + (size_t)nd * nmb * ZW_TOK_MODE), o_p = al256(o_c + (size_t)nd * ncw * 4);
    const size_t o_tf = al256(o_p + (size_t)nd * probs_b), o_b = al256(o_tf + (size_t)nd * sizeof(ZwTokFrame));
    const size_t up_bytes = al256(o_b + blob);
    uint8_t* stage = (uint8_t*)ctx_pinned(ctx, 4, up_bytes);
    if (!stage) return false;
    T.quant.assign((size_t)nd * 4, DecQuant());
    T.fps.assign(nd, ZwFilterParams());
    parallel_for(nd, [&](int i) {
        uint8_t* mr = stage + o_m + (size_t)i * nmb * ZW_TOK_MODE;
        rc[i] = parse_modes(F[i], mr);
        uint32_t* cw = (uint32_t*)(stage + o_c) + (size_t)i * ncw;  // 2 bits per MB: I4, skipped
        memset(cw, 0, ncw * 4);
        for (size_t j = 0; j < nmb; j++) {
            const uint8_t b0 = mr[j * ZW_TOK_MODE];
            cw[j >> 4] |= ((uint32_t)((b0 & 7) == 4) | (uint32_t)((b0 >> 5) & 1) << 1) << (2 * (j & 15));
        }
        memcpy(stage + o_p + (size_t)i * probs_b, F[i].probs, tokl::PROBS);  // [type][band][ctx][node]
        const ZwTokFrame tf = {boff[i], (uint32_t)F[i].part[0].len, 0};
        memcpy(stage + o_tf + (size_t)i * sizeof(ZwTokFrame), &tf, sizeof tf);
        const size_t len = F[i].part[0].len, al = (len + 15) & ~(size_t)15;
        memcpy(stage + o_b + boff[i], F[i].part[0].d, len);
        memset(stage + o_b + boff[i] + len, 0, al - len);
        for (int q = 0; q < 4; q++) T.quant[(size_t)i * 4 + q] = F[i].q[q];
        filter_table(T.fps[i], F[i].filter_type, F[i].filter_level, F[i].sharpness, F[i].segments_enabled,
                     F[i].seg_delta_values, F[i].seg_lf, F[i].lf_adj_enabled, F[i].ref_delta0, F[i].mode_delta0, mbw,
                     mbh);
    });
    for (int i = 0; i < nd; i++)
        if (rc[i] != ZW_OK) return false;
    memset(stage + o_b + blob - 16, 0, 16);
    const size_t o_sn = up_bytes, o_sz = al256(o_sn + (size_t)nd * nmb * 16), o_mo = al256(o_sz + (size_t)nd * nmb * 4);
    const size_t o_fb = al256(o_mo + (size_t)nd * (nmb + 1) * 4), o_e1 = al256(o_fb + (size_t)nd * 8);
    const size_t o_e2 = al256(o_e1 + (size_t)nd * 4), o_te = al256(o_e2 + (size_t)nd * 4);
    const size_t o_tot = al256(o_te + (size_t)nd * 4), total = al256(o_tot + 8);
    uint8_t* d = (uint8_t*)ctx_scratch_tok(ctx, total);
    if (!d) return false;
    if (!ctx->tok_total && hipHostMalloc((void**)&ctx->tok_total, 256, hipHostMallocDefault) != hipSuccess) {
        ctx->tok_total = nullptr;
        return false;
    }
    if (!ctx->tok_ && hipStreamCreateWithFlags(&ctx->tok_, hipStreamNonBlocking) != hipSuccess) return false;
    for (hipEvent_t& e : ctx->tok_ev)
        if (!e && hipEventCreate(&e) != hipSuccess) return false;
    hipStream_t s = ctx->tok_;
    if (hipMemcpyAsync(d, stage, up_bytes, hipMemcpyHostToDevice, s) != hipSuccess) return false;
    if (hipEventRecord(ctx->tok_ev[0], s) != hipSuccess) return false;
    if (zwk_dec_tok_count(s, d + o_b, (const ZwTokFrame*)(d + o_tf), d + o_p, d + o_m, (const uint32_t*)(d + o_c),
                          d + o_sn, (int*)(d + o_e1), (uint32_t*)(d + o_sz), (int*)(d + o_e2), (uint32_t*)(d + o_mo),
                          (uint64_t*)(d + o_fb), (int*)(d + o_te), (uint64_t*)(d + o_tot), ctx->tok_total, mbw, mbh,
                          nd, ctx->tok_ev[3]) != hipSuccess ||
        hipEventRecord(ctx->tok_ev[2], s) != hipSuccess) {
        (void)hipStreamSynchronize(s);  // (work may be in flight: let it finish before the host takes over)
        return false;
    }
    T.h0 = h0;
    T.nd = nd;
    T.nmb = nmb;
    T.d = d;
    T.o_b = o_b;
    T.o_tf = o_tf;
    T.o_p = o_p;
    T.o_m = o_m;
    T.o_sn = o_sn;
    T.o_e1 = o_e1;
    T.moff = (const uint32_t*)(d + o_mo);
    T.fbase = (const uint64_t*)(d + o_fb);
    T.err = (const int*)(d + o_te);
    T.state = 0;
    return true;
}

// The device parse's second half, once, before the first device chunk: waits
// for the count (the host thread blocks; the previous chunk's download and
// fan-out run on their own thread meanwhile), sizes the record buffer and
// queues the record pass.  false: the host parses the device frames instead.
static bool dec_tok_finish(zw_ctx* ctx, DecTok& T)
{
    if (T.state != 0) return T.state > 0;
    T.state = -1;
    if (hipEventSynchronize(ctx->tok_ev[2]) != hipSuccess) return false;
    const size_t bytes = std::max<size_t>(256, (size_t)*ctx->tok_total);
    uint8_t* recs = (uint8_t*)ctx_scratch_rec(ctx, bytes);
    if (!recs) return false;
    hipStream_t s = ctx->tok_;
    if (zwk_dec_tok_write(s, T.d + T.o_b, (const ZwTokFrame*)(T.d + T.o_tf), T.d + T.o_p, T.d + T.o_m, T.d + T.o_sn,
                          (const int*)(T.d + T.o_e1), T.moff, T.fbase, recs, (int)T.nmb, T.nd) != hipSuccess ||
        hipEventRecord(ctx->tok_ev[1], s) != hipSuccess) {
        (void)hipStreamSynchronize(s);
        return false;
    }
    T.recs = recs;
    T.done = ctx->tok_ev[1];
    T.state = 1;
    if (const char* dump = getenv("ZW_DEC_TOKENS_DUMP")) {  // debug: device frame 0's records to <dump>.dev
        if (hipStreamSynchronize(s) == hipSuccess) {
            std::vector<uint32_t> mo(T.nmb + 1);
            uint64_t fb0 = 0;
            (void)hipMemcpy(mo.data(), T.moff, (T.nmb + 1) * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(&fb0, T.fbase, 8, hipMemcpyDeviceToHost);
            std::vector<uint8_t> dev(mo[T.nmb]);
            (void)hipMemcpy(dev.data(), recs + fb0, mo[T.nmb], hipMemcpyDeviceToHost);
            std::string p0 = std::string(dump) + ".dev";
            if (FILE* fo = fopen(p0.c_str(), "wb")) {
                fwrite(mo.data(), 4, T.nmb + 1, fo);
                fwrite(dev.data(), 1, dev.size(), fo);
                fclose(fo);
            }
        }
    }
    return true;
}

// A chunk of device frames [first, first + cnt): no host parse; its records are the device parse's.
static void dec_parse_dev(const DecTok& T, int first, int cnt, DecBatch& B)
{
    const int j0 = first - T.h0;
    B.F.assign(T.F.begin() + j0, T.F.begin() + j0 + cnt);
    B.quant.assign(T.quant.begin() + (size_t)j0 * 4, T.quant.begin() + (size_t)(j0 + cnt) * 4);
    B.fps.assign(T.fps.begin() + j0, T.fps.begin() + j0 + cnt);
    B.mbw = T.F[0].mbw;
    B.mbh = T.F[0].mbh;
    B.ysz = T.nmb * 256;
    B.csz = T.nmb * 64;
    B.n = cnt;
    B.stage = nullptr;
    B.up_bytes = B.o_moff = B.o_base = B.rec_bytes = 0;
    B.x_recs = T.recs;
    B.x_moff = T.moff + (size_t)j0 * (T.nmb + 1);
    B.x_fbase = T.fbase + j0;
    B.x_done = T.done;
    B.d_terr = T.err + j0;
    B.parse_ms = 0;
}

// Runs the batch in chunks, alternating the two buffer sets.  Per step c the
// host parses chunk c while a second thread finishes chunk c-1 (waits for its
// kernels, downloads and fans out -- mostly a DMA wait), then chunk c is
// uploaded and launched; the device runs chunk c-1 during both.  enqueue(B,
// first, count) queues caller work after the filter (or does nothing);
// finish(B, first, count) waits for it, downloads and fans out.  Device times
// of all chunks add up in ctx->dec_ms.
template <class ENQ, class FIN>
static int dec_pipeline(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, size_t extra_per_frame,
                        ENQ&& enqueue, FIN&& finish)
{
    const int C = dec_chunk_frames();
    DecBatch B[2];
    ctx->dec_ms[0] = ctx->dec_ms[1] = ctx->dec_ms[2] = 0.f;
    ctx->dec_tok_ms = 0.f;
    ctx->dec_tok_stage_ms[0] = ctx->dec_tok_stage_ms[1] = ctx->dec_tok_stage_ms[2] = 0.f;
    ctx->dec_host_ms[0] = ctx->dec_host_ms[1] = ctx->dec_host_ms[2] = 0;
    // the device's share of the tokens first (its launch runs beside the host chunks)
    DecTok T;
    {
        const double t0 = dec_now_ms();
        size_t nmb = 0;
        if (n > 0 && lens[0] >= 10) {  // (the first frame's dimensions; dec_tok_prepare checks every frame)
            const uint8_t* d = data[0];
            nmb = (size_t)((((d[6] | (d[7] << 8)) & 0x3fff) + 15) / 16) * (size_t)((((d[8] | (d[9] << 8)) & 0x3fff) + 15) / 16);
        }
        const int h0 = nmb ? dec_tok_split(ctx, n, C, nmb) : n;
        if (h0 >= n || !dec_tok_prepare(ctx, n, data, lens, h0, T)) T.h0 = n;
        ctx->dec_host_ms[0] += dec_now_ms() - t0;
    }
    double host_parse_ms = 0;
    int host_frames = 0;
    // chunks: C frames while the host parses, then the device-parsed frames in chunks
    // of up to ZW_DEC_DEV_CHUNK (512): their records are all ready at once when the
    // device parse ends, so fewer, longer chunks download back to back behind it
    // (1 024 1080p frames: the tail after the device parse 68 -> ~45 ms)
    std::vector<int> cb;
    {
        static const int DC = [] {
            const char* e = getenv("ZW_DEC_DEV_CHUNK");
            const int v = e ? atoi(e) : 512;
            return v > 0 ? v : 512;
        }();
        for (int f = 0; f < n;) {
            cb.push_back(f);
            f += f < T.h0 ? std::min(C, T.h0 - f) : DC;
        }
        cb.push_back(n);
    }
    const int nch = (int)cb.size() - 1;
    auto first = [&](int c) { return cb[c]; };
    auto count = [&](int c) { return std::min(cb[c + 1], n) - cb[c]; };
    int err = ZW_OK;
    // ZW_DEC_TRACE: the chunk timeline (ms from the batch start) on stderr
    static const bool trace = getenv("ZW_DEC_TRACE") != nullptr;
    const double tb = dec_now_ms();
    for (int c = 0; c <= nch && !err; c++) {
        int err_f = ZW_OK, err_p = ZW_OK;
        std::thread fin;
        double tf0 = 0, tf1 = 0, tp0 = 0, tp1 = 0;
        if (c >= 1) {
            fin = std::thread([&, c]() {
                (void)hipSetDevice(ctx->device);
                DecBatch& b = B[(c - 1) & 1];
                tf0 = dec_now_ms() - tb;
                err_f = finish(b, first(c - 1), count(c - 1));
                tf1 = dec_now_ms() - tb;
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, b.ev[0], b.ev[1]) == hipSuccess) ctx->dec_ms[0] += ms;
                if (hipEventElapsedTime(&ms, b.ev[1], b.ev[2]) == hipSuccess) ctx->dec_ms[1] += ms;
            });
        }
        tp0 = dec_now_ms() - tb;
        if (c < nch) {
            if (first(c) >= T.h0 && dec_tok_finish(ctx, T)) {
                dec_parse_dev(T, first(c), count(c), B[c & 1]);
            } else {
                err_p = dec_parse(ctx, count(c), data + first(c), lens + first(c), B[c & 1], c & 1);
                host_parse_ms += B[c & 1].parse_ms;
                host_frames += count(c);
            }
            ctx->dec_host_ms[0] += B[c & 1].parse_ms;
        }
        tp1 = dec_now_ms() - tb;
        if (fin.joinable()) fin.join();
        err = err_f ? err_f : err_p;
        if (c < nch && !err) {
            DecBatch& b = B[c & 1];
            err = dec_launch(ctx, extra_per_frame * count(c), b, c & 1);
            if (!err) err = enqueue(b, first(c), count(c));
        }
        if (trace)
            fprintf(stderr, "[dec trace] c=%d %s parse %.1f-%.1f, finish(c-1) %.1f-%.1f, launched %.1f ms\n", c,
                    c < nch && first(c) >= T.h0 ? "dev " : "host", tp0, tp1, tf0, tf1, dec_now_ms() - tb);
    }
    if (T.nd > 0) {
        if (T.state == 0) (void)hipStreamSynchronize(ctx->tok_);  // (an error before the first device chunk)
        float ms = 0.f;
        if (T.state > 0 && hipEventSynchronize(T.done) == hipSuccess &&
            hipEventElapsedTime(&ms, ctx->tok_ev[0], ctx->tok_ev[1]) == hipSuccess) {
            ctx->dec_tok_ms = ms;
            for (int k = 0; k < 3; k++) {
                float m = 0.f;
                static const int e0[3] = {0, 3, 2}, e1[3] = {3, 2, 1};
                if (hipEventElapsedTime(&m, ctx->tok_ev[e0[k]], ctx->tok_ev[e1[k]]) == hipSuccess) ctx->dec_tok_stage_ms[k] = m;
            }
            if (!err && ms > 0) ctx->dec_tok_ms_per_mb = ms / (double)T.nmb;
        }
    }
    // (a chunk's parse runs while the previous chunk downloads: the chunk time is its share of the pipe)
    if (!err && host_frames >= C && host_parse_ms > 0) ctx->dec_host_ms_per_frame = host_parse_ms / host_frames;
    if (err) (void)hipStreamSynchronize(ctx_stream(ctx));  // nothing queued may outlive the call
    return err;
}

// A batch's frames in runs of one size: each run decodes as a batch of its own
// (the device buffers and the packed images of a run are per size), in frame
// order, so the first failing frame's error is the one returned, as a sequence
// of decode_frame calls (decoder/vp8.rs:1526) would report it.  Returns the
// end of the run starting at i0 (frames too short for dimensions stand alone).
static int dec_run_end(int n, const uint8_t* const* data, const size_t* lens, int i0)
{
    auto key = [&](int i) -> uint32_t {
        if (!data[i] || lens[i] < 10) return 0xffffffffu;
        const uint8_t* d = data[i];
        return (uint32_t)((d[6] | (d[7] << 8)) & 0x3fff) | ((uint32_t)((d[8] | (d[9] << 8)) & 0x3fff) << 16);
    };
    const uint32_t k0 = key(i0);
    int i1 = i0 + 1;
    if (k0 != 0xffffffffu)
        while (i1 < n && key(i1) == k0) i1++;
    return i1;
}

static int dec_batch_one(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, zw_frame* outs);

extern "C" int zw_vp8_decode_batch(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, zw_frame* outs)
{
    if (!ctx || n <= 0 || !data || !lens || !outs) return ZW_EINVAL;
    for (int i = 0; i < n; i++) memset(&outs[i], 0, sizeof(zw_frame));
    for (int i0 = 0; i0 < n;) {
        const int i1 = dec_run_end(n, data, lens, i0);
        if (const int r = dec_batch_one(ctx, i1 - i0, data + i0, lens + i0, outs + i0)) {
            for (int k = 0; k < i0; k++) zw_frame_free(&outs[k]);
            return r;
        }
        i0 = i1;
    }
    return ZW_OK;
}

static int dec_batch_one(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, zw_frame* outs)
{
    for (int i = 0; i < n; i++) memset(&outs[i], 0, sizeof(zw_frame));
    int mbw0 = -1, mbh0 = -1;
    auto enqueue = [&](DecBatch& B, int, int) -> int {
        if (mbw0 < 0) mbw0 = B.mbw, mbh0 = B.mbh;
        return B.mbw == mbw0 && B.mbh == mbh0 ? ZW_OK : ZW_EINVAL;  // one size per batch, as in one chunk
    };
    auto finish = [&](DecBatch& B, int f0, int cn) -> int {
        const std::vector<DecFrame>& F = B.F;
        const size_t ysz = B.ysz, csz = B.csz;
        uint8_t* d = B.d;
        // planes down through pinned staging, then fanned out into one buffer per frame
        const size_t fsz = ysz + 2 * csz;
        uint8_t* hout = (uint8_t*)ctx_pinned(ctx, 1, (size_t)cn * fsz);
        if (!hout) return ZW_ENOMEM;
        HIPOK(hipEventSynchronize(B.ev[2]));
        if (int r = tokens_error(ctx, B.d_terr, B.n)) return r;
        if (int r = rows_error(ctx, B.d_rs, B.n, B.mbh)) return r;
        const double td = dec_now_ms();
        // planes down in parts (three plane copies per frame range), each part
        // fanned out into the frames' buffers while the next lands
        const double tf = dec_now_ms();
        std::vector<int> oom(cn, 0);
        double dl_ms = 0;
        const int dr = dec_download_fan(
            ctx, cn,
            [&](int a, int b) {
                const size_t A = (size_t)a, N = (size_t)(b - a);
                int r = ctx_d2h_stream(ctx, hout + A * ysz, d + B.o_y + A * ysz, N * ysz);
                if (!r) r = ctx_d2h_stream(ctx, hout + (size_t)cn * ysz + A * csz, d + B.o_u + A * csz, N * csz);
                if (!r) r = ctx_d2h_stream(ctx, hout + (size_t)cn * (ysz + csz) + A * csz, d + B.o_v + A * csz, N * csz);
                return r;
            },
            [&](int a, int b) {
                parallel_for(b - a, [&](int k) {
                    const int i = a + k;
                    uint8_t* buf = frame_pool().get(fsz);
                    if (!buf) {
                        oom[i] = 1;
                        return;
                    }
                    memcpy(buf, hout + (size_t)i * ysz, ysz);
                    memcpy(buf + ysz, hout + (size_t)cn * ysz + (size_t)i * csz, csz);
                    memcpy(buf + ysz + csz, hout + (size_t)cn * (ysz + csz) + (size_t)i * csz, csz);
                    outs[f0 + i].y = buf;
                }, dec_fan_threads());
            },
            &dl_ms);
        ctx->dec_host_ms[1] += dl_ms;
        if (dr) return dr;
        ctx->dec_host_ms[2] += dec_now_ms() - tf;
        if (dec_timing()) fprintf(stderr, "[dec] download+fanout %.2f ms\n", dec_now_ms() - td);
        int r = ZW_OK;
        for (int i = 0; i < cn; i++) {
            zw_frame& o = outs[f0 + i];
            if (oom[i]) {
                r = ZW_ENOMEM;
                continue;
            }
            uint8_t* buf = o.y;
            o.width = (uint16_t)F[i].width;
            o.height = (uint16_t)F[i].height;
            o.y_stride = (uint32_t)B.mbw * 16;
            o.uv_stride = (uint32_t)B.mbw * 8;
            o.mb_rows = (uint32_t)B.mbh;
            o.y = buf;
            o.u = buf + ysz;
            o.v = buf + ysz + csz;
            o.filter_type = (uint8_t)F[i].filter_type;
            o.filter_level = (uint8_t)F[i].filter_level;
            o.sharpness_level = (uint8_t)F[i].sharpness;
        }
        return r;
    };
    const int r = dec_pipeline(ctx, n, data, lens, 0, enqueue, finish);
    if (r)
        for (int k = 0; k < n; k++) zw_frame_free(&outs[k]);
    return r;
}

// Frame::fill_rgb / fill_rgba (decoder/vp8.rs:200-258) after decode_frame, on
// the device: decode -> k_yuv2rgb -> packed RGB(A) down.  Every frame of the
// batch must have the same dimensions (their packed images are contiguous).
// The images land either in new buffers (outs) or in the caller's buffers
// (dst[i], dst_lens[i] bytes, rows `stride` bytes apart: decode_rgba_into /
// decode_rgb_into, api.rs:1004-1128), where a repeated decode touches no fresh
// pages.
static int dec_rgb_batch(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, int bpp, int upsampling,
                         zw_bytes* outs, uint8_t* const* dst, const size_t* dst_lens, size_t stride, uint32_t* widths,
                         uint32_t* heights)
{
    if (!ctx || n <= 0 || !data || !lens || (!outs && !dst) || (bpp != 3 && bpp != 4) ||
        (upsampling != ZW_UPSAMPLE_BILINEAR && upsampling != ZW_UPSAMPLE_SIMPLE))
        return ZW_EINVAL;
    if (outs)
        for (int i = 0; i < n; i++) outs[i].data = nullptr, outs[i].len = 0;
    // dimensions first (they size the device output)
    size_t w = 0, h = 0;
    {
        DecFrame f0;
        const int r = parse_header(f0, data[0], lens[0]);
        if (r) return r;
        w = f0.width;
        h = f0.height;
    }
    const size_t row = w * (size_t)bpp, fbytes = row * h;
    if (dst) {  // decode_rgba_into: stride >= width * bpp, buffer >= stride * height
        if (!dst_lens || stride < row) return ZW_EINVAL;
        for (int i = 0; i < n; i++)
            if (!dst[i] || dst_lens[i] < stride * h) return ZW_EINVAL;
    }
    hipStream_t s = ctx_stream(ctx);
    auto enqueue = [&](DecBatch& B, int, int cn) -> int {
        for (int i = 0; i < cn; i++)
            if ((size_t)B.F[i].width != w || (size_t)B.F[i].height != h) return ZW_EINVAL;
        HIPOK(zwk_yuv2rgb(s, B.d + B.o_y, B.d + B.o_u, B.d + B.o_v, B.ysz, B.csz, (int)w, (int)h, B.mbw * 16,
                          B.mbw * 8, bpp, upsampling == ZW_UPSAMPLE_BILINEAR, B.d + B.o_extra, cn));
        HIPOK(hipEventRecord(B.ev[3], s));
        return ZW_OK;
    };
    auto finish = [&](DecBatch& B, int f0, int cn) -> int {
        uint8_t* hout = (uint8_t*)ctx_pinned(ctx, 1, (size_t)cn * fbytes);
        if (!hout) return ZW_ENOMEM;
        HIPOK(hipEventSynchronize(B.ev[3]));
        if (int r = tokens_error(ctx, B.d_terr, B.n)) return r;
        if (int r = rows_error(ctx, B.d_rs, B.n, B.mbh)) return r;
        const double tf = dec_now_ms();
        std::vector<int> oom(cn, 0);
        double dl_ms = 0;
        const int dr = dec_download_fan(
            ctx, cn,
            [&](int a, int b) {
                return ctx_d2h_stream(ctx, hout + (size_t)a * fbytes, B.d + B.o_extra + (size_t)a * fbytes,
                                      (size_t)(b - a) * fbytes);
            },
            [&](int a, int b) {
                parallel_for(b - a, [&](int k) {
                    const int i = a + k;
                    const uint8_t* src = hout + (size_t)i * fbytes;
                    if (dst) {
                        uint8_t* o = dst[f0 + i];
                        if (stride == row) {
                            memcpy(o, src, fbytes);
                        } else {
                            for (size_t y = 0; y < h; y++) memcpy(o + y * stride, src + y * row, row);
                        }
                        return;
                    }
                    uint8_t* buf = frame_pool().get(fbytes ? fbytes : 1);
                    if (!buf) {
                        oom[i] = 1;
                        return;
                    }
                    memcpy(buf, src, fbytes);
                    outs[f0 + i].data = buf;
                    outs[f0 + i].len = fbytes;
                }, dec_fan_threads());
            },
            &dl_ms);
        ctx->dec_host_ms[1] += dl_ms;
        ctx->dec_host_ms[2] += dec_now_ms() - tf;
        if (dr) return dr;
        for (int i = 0; i < cn; i++)
            if (oom[i]) return ZW_ENOMEM;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, B.ev[2], B.ev[3]) == hipSuccess) ctx->dec_ms[2] += ms;
        return ZW_OK;
    };
    const int r = dec_pipeline(ctx, n, data, lens, fbytes, enqueue, finish);
    if (r) {
        if (outs)
            for (int k = 0; k < n; k++) zw_bytes_free(&outs[k]);
        return r;
    }
    for (int i = 0; i < n; i++) {
        if (widths) widths[i] = (uint32_t)w;
        if (heights) heights[i] = (uint32_t)h;
    }
    return ZW_OK;
}

extern "C" int zw_vp8_decode_rgb_batch(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens, int bpp,
                                       int upsampling, zw_bytes* outs, uint32_t* widths, uint32_t* heights)
{
    if (!outs || n <= 0 || !data || !lens) return ZW_EINVAL;
    for (int i = 0; i < n; i++) outs[i].data = nullptr, outs[i].len = 0;
    for (int i0 = 0; i0 < n;) {  // runs of one size (dec_run_end)
        const int i1 = dec_run_end(n, data, lens, i0);
        if (const int r = dec_rgb_batch(ctx, i1 - i0, data + i0, lens + i0, bpp, upsampling, outs + i0, nullptr,
                                        nullptr, 0, widths ? widths + i0 : nullptr, heights ? heights + i0 : nullptr)) {
            for (int k = 0; k < i0; k++) zw_bytes_free(&outs[k]);
            return r;
        }
        i0 = i1;
    }
    return ZW_OK;
}

extern "C" int zw_vp8_decode_rgb_batch_into(zw_ctx* ctx, int n, const uint8_t* const* data, const size_t* lens,
                                            int bpp, int upsampling, uint8_t* const* outs, const size_t* out_lens,
                                            uint32_t stride_bytes, uint32_t* widths, uint32_t* heights)
{
    if (!outs || n <= 0 || !data || !lens || !out_lens) return ZW_EINVAL;
    for (int i0 = 0; i0 < n;) {  // runs of one size (dec_run_end)
        const int i1 = dec_run_end(n, data, lens, i0);
        if (const int r = dec_rgb_batch(ctx, i1 - i0, data + i0, lens + i0, bpp, upsampling, nullptr, outs + i0,
                                        out_lens + i0, stride_bytes, widths ? widths + i0 : nullptr,
                                        heights ? heights + i0 : nullptr))
            return r;
        i0 = i1;
    }
    return ZW_OK;
}

extern "C" int zw_vp8_decode_rgb(zw_ctx* ctx, const uint8_t* vp8, size_t len, int bpp, int upsampling, zw_bytes* out,
                                 uint32_t* width, uint32_t* height)
{
    if (!vp8 && len) return ZW_EINVAL;
    const uint8_t* d[1] = {vp8};
    size_t l[1] = {len};
    return zw_vp8_decode_rgb_batch(ctx, 1, d, l, bpp, upsampling, out, width, height);
}

// Kernel-level entry: fill_rgb_buffer_fancy / _simple (decoder/yuv.rs:82, :402)
// of one image's planes (host buffers; rows of y_stride / uv_stride bytes,
// ceil(h/2) chroma rows) into out (w*h*bpp bytes, packed).
extern "C" int zw_yuv_to_rgb(zw_ctx* ctx, const uint8_t* y, const uint8_t* u, const uint8_t* v, uint32_t width,
                             uint32_t height, uint32_t y_stride, uint32_t uv_stride, int bpp, int upsampling,
                             uint8_t* out)
{
    if (!ctx || !y || !u || !v || !out || width == 0 || height == 0 || y_stride < width ||
        uv_stride < (width + 1) / 2 || (bpp != 3 && bpp != 4) ||
        (upsampling != ZW_UPSAMPLE_BILINEAR && upsampling != ZW_UPSAMPLE_SIMPLE))
        return ZW_EINVAL;
    const size_t ch = (height + 1) / 2;
    const size_t ysz = (size_t)y_stride * height, csz = (size_t)uv_stride * ch;
    const size_t obytes = (size_t)width * height * bpp;
    const size_t o_y = 0, o_u = al256(ysz), o_v = al256(o_u + csz), o_o = al256(o_v + csz);
    HIPOK(hipSetDevice(ctx->device));
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, al256(o_o + obytes));
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_y, y, ysz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_u, u, csz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_v, v, csz, hipMemcpyHostToDevice, s));
    HIPOK(zwk_yuv2rgb(s, d + o_y, d + o_u, d + o_v, ysz, csz, (int)width, (int)height, (int)y_stride, (int)uv_stride,
                      bpp, upsampling == ZW_UPSAMPLE_BILINEAR, d + o_o, 1));
    HIPOK(hipMemcpyAsync(out, d + o_o, obytes, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return ZW_OK;
}

extern "C" int zw_decode_kernel_times(zw_ctx* ctx, float* ms)
{
    if (!ctx || !ms) return ZW_EINVAL;
    ms[0] = ctx->dec_ms[0];
    ms[1] = ctx->dec_ms[1];
    return ZW_OK;
}

extern "C" int zw_decode_token_ms(zw_ctx* ctx, float* ms)
{
    if (!ctx || !ms) return ZW_EINVAL;
    *ms = ctx->dec_tok_ms;
    return ZW_OK;
}

extern "C" int zw_decode_token_stages(zw_ctx* ctx, float* ms)
{
    if (!ctx || !ms) return ZW_EINVAL;
    for (int i = 0; i < 3; i++) ms[i] = ctx->dec_tok_stage_ms[i];
    return ZW_OK;
}

extern "C" int zw_decode_stage_times(zw_ctx* ctx, float* ms)
{
    if (!ctx || !ms) return ZW_EINVAL;
    for (int i = 0; i < 3; i++) ms[i] = (float)ctx->dec_host_ms[i];
    return ZW_OK;
}

extern "C" int zw_decode_rgb_kernel_ms(zw_ctx* ctx, float* ms)
{
    if (!ctx || !ms) return ZW_EINVAL;
    *ms = ctx->dec_ms[2];
    return ZW_OK;
}

extern "C" int zw_vp8_decode_frame(zw_ctx* ctx, const uint8_t* vp8, size_t len, zw_frame* out)
{
    if (!vp8 && len) return ZW_EINVAL;
    const uint8_t* d[1] = {vp8};
    size_t l[1] = {len};
    return zw_vp8_decode_batch(ctx, 1, d, l, out);
}

extern "C" int zw_loop_filter_frame(zw_ctx* ctx, uint8_t* y, uint8_t* u, uint8_t* v, uint32_t mbw, uint32_t mbh,
                                    const uint8_t* mb_flags, int filter_type, int filter_level, int sharpness,
                                    int segments_enabled, int seg_delta_values, const int8_t seg_lf_level[4],
                                    int lf_adj_enabled, int ref_delta0, int mode_delta0)
{
    if (!ctx || !y || !u || !v || !mb_flags || mbw == 0 || mbh == 0) return ZW_EINVAL;
    const int8_t zero[4] = {0, 0, 0, 0};
    ZwFilterParams fp;
    filter_table(fp, filter_type, filter_level, sharpness, segments_enabled, seg_delta_values,
                 seg_lf_level ? seg_lf_level : zero, lf_adj_enabled, ref_delta0, mode_delta0, (int)mbw, (int)mbh);
    const size_t nmb = (size_t)mbw * mbh, ysz = nmb * 256, csz = nmb * 64;
    const size_t o_fp = 0, o_fl = 256, o_y = al256(o_fl + nmb * 4), o_u = al256(o_y + ysz), o_v = al256(o_u + csz);
    const size_t o_rs = al256(o_v + csz);
    const size_t total = al256(o_rs + zw_dec_rows_sync_bytes((int)mbh, 1));
    const int rows_env = getenv("ZW_DEC_ROWS") ? atoi(getenv("ZW_DEC_ROWS")) : -1;  // as decode_to_device, n = 1
    HIPOK(hipSetDevice(ctx->device));
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_fp, &fp, sizeof fp, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_fl, mb_flags, nmb * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_y, y, ysz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_u, u, csz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_v, v, csz, hipMemcpyHostToDevice, s));
    if (rows_env != 0) {
        HIPOK(zwk_dec_rows_init(s, (int*)(d + o_rs), (int)mbh, 1));
        if (dec_force_error()) HIPOK(hipMemsetAsync(d + o_rs + 2 * sizeof(int), 1, sizeof(int), s));
        HIPOK(zwk_dec_rows(s, 2, nullptr, nullptr, nullptr, nullptr, d + o_y, d + o_u, d + o_v, d + o_fl, (const ZwFilterParams*)(d + o_fp),
                           (int)mbw, (int)mbh, ysz, csz, 1, (int*)(d + o_rs), nullptr, (int)mbh));
    } else {
        HIPOK(zwk_loopfilter(s, d + o_y, d + o_u, d + o_v, d + o_fl, (const ZwFilterParams*)(d + o_fp), ysz, csz, 1,
                             (int)mbw, nullptr));
    }
    HIPOK(hipMemcpyAsync(y, d + o_y, ysz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(u, d + o_u, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(v, d + o_v, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return rows_env != 0 ? rows_error(ctx, (const int*)(d + o_rs), 1, (int)mbh) : ZW_OK;
}

// ---------------------------------------------------------------------------
// CPU check of the device token parse (zw_tokl.h, the code k_dec_tok1 and
// k_dec_tok2 run per lane): the same functions step one frame here over host
// memory -- stage 1 over the whole frame (snapshots), stage 2 per MB from each
// snapshot (count, offsets, records) -- and the records must equal parse_mbs's
// byte for byte (or both fail).  Test hook only (tests/test_tokl.py); no device work.
// ---------------------------------------------------------------------------
namespace {
static uint64_t host_bits64(const uint8_t* stream, size_t len, uint32_t bp)
{
    uint64_t v = 0;
    const size_t b0 = bp >> 3;
    for (int i = 0; i < 9; i++) {
        const uint64_t byte = b0 + i < len ? stream[b0 + i] : 0;
        if (i < 8) v = (v << 8) | byte;
        else v = (bp & 7) ? (v << (bp & 7)) | (byte >> (8 - (bp & 7))) : v;
    }
    return v;
}

struct HostTok1Mem {
    static constexpr uint32_t U = 1;
    const uint32_t* T1;
    const uint8_t* P;
    const uint8_t* stream;
    size_t len;
    const uint8_t* modes;
    uint32_t nmb, mbw;
    std::vector<uint16_t> tcxv;
    std::vector<uint32_t> snaps;  // 4 words per MB
    uint32_t prob_at(uint32_t a) const { return P[a]; }
    void tt1(uint32_t s8, uint32_t& t0, uint32_t& t1) const
    {
        t0 = T1[s8 / 4];
        t1 = T1[s8 / 4 + 1];
    }
    void desc1(uint32_t i, uint32_t* d) const { tok1::desc1<1>(i / tok1::NDESC1, i % tok1::NDESC1, d); }
    uint64_t bits64(uint32_t bp) const { return host_bits64(stream, len, bp); }
    uint32_t cls(uint32_t mbi) const
    {
        const uint8_t b0 = modes[(size_t)mbi * ZW_TOK_MODE];
        return (uint32_t)((b0 & 7) == 4) | ((uint32_t)((b0 >> 5) & 1) << 1);
    }
    uint32_t tcx(uint32_t mbx) const { return tcxv[mbx]; }
    void set_tcx(uint32_t mbx, uint32_t v) { tcxv[mbx] = (uint16_t)v; }
    void snap(bool c, uint32_t mbi, uint32_t s0, uint32_t s1, uint32_t tl)
    {
        if (!c) return;
        uint32_t* w = &snaps[(size_t)mbi * 4];
        w[0] = s0;
        w[1] = s1;
        w[2] = tl;
        w[3] = 0;
    }
};

struct HostTok2Mem {
    static constexpr uint32_t U = 1;
    static constexpr uint32_t lane0 = 0;
    const uint32_t* TT;
    const uint8_t* P;
    const uint8_t* stream;
    size_t len;
    uint8_t* rec = nullptr;  // null: count only
    uint32_t lim = 0;        // the MB's record end (stores past it belong to the next MB)

    void tt(uint32_t st, uint32_t& t0, uint32_t& t1) const
    {
        t0 = TT[2 * st];
        t1 = TT[2 * st + 1];
    }
    void desc(uint32_t i, uint32_t* d) const { tokl::desc(i / tokl::NDESC, i % tokl::NDESC, d); }
    uint32_t prob_at(uint32_t i) const { return P[i]; }
    uint64_t bits64(uint32_t bp) const { return host_bits64(stream, len, bp); }
    void st16c(bool c, uint32_t off, uint32_t v)
    {
        const uint16_t h = (uint16_t)v;
        if (rec && c && off < lim) memcpy(rec + off, &h, 2);
    }
    void st128(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d)
    {
        const uint32_t w[4] = {a, b, c, d};
        if (rec) memcpy(rec + off, w, 16);
    }
};

// stage 2 for MB i of a frame (its record at hb); returns the record's bytes, *bad = the eof rule failed
static uint32_t host_tok2_mb(HostTok2Mem& m, const uint8_t* modes, const uint32_t* snap, uint32_t hb, bool* bad)
{
    uint32_t mr[4];
    memcpy(mr, modes, 16);
    if ((mr[0] >> 5) & 1u) {
        tokl::mb_skip(m, hb, mr);
        return ZW_DREC_HDR;
    }
    tokl::Lane L;
    tokl::from_snapshot(L, m, snap[0], snap[1], (uint32_t)m.len);
    L.hb = hb;
    tokl::mb_begin(L, m, mr, snap[2]);
    while (L.phase == tokl::PH_DECIDE) {
        if (L.vb < 8) tokl::topup(L, m);
        tokl::step(L, m);
    }
    tokl::mb_end(L, m);
    *bad = *bad || L.bad;
    return L.hb - hb;
}
}  // namespace

extern "C" int zw_dbg_tokl_frame(const uint8_t* vp8, size_t len, int* match)
{
    if (!match || (!vp8 && len)) return ZW_EINVAL;
    *match = -1;
    DecFrame A, B;
    if (int r = parse_header(A, vp8, len)) return r;
    (void)parse_header(B, vp8, len);
    const size_t nmb = (size_t)A.mbw * A.mbh;
    if (nmb == 0) return ZW_EINVALID_DIMENSIONS;
    std::vector<uint8_t> ref(nmb * ZW_DREC_MAX), modes(nmb * ZW_TOK_MODE);
    std::vector<uint32_t> moff_ref(nmb + 1), moff(nmb + 1);
    const int rc = parse_mbs(A, ref.data(), moff_ref.data());
    if (B.nparts != 1 || B.mbw < 2 || parse_modes(B, modes.data()) != ZW_OK) return rc;  // the host keeps such frames
    // stage 1
    static const tok1::Table<1> T1;
    HostTok1Mem m1;
    m1.T1 = T1.e;
    m1.P = &B.probs[0][0][0][0];
    m1.stream = B.part[0].d;
    m1.len = B.part[0].len;
    m1.modes = modes.data();
    m1.nmb = (uint32_t)nmb;
    m1.mbw = (uint32_t)B.mbw;
    m1.tcxv.assign(B.mbw + 1, 0);
    m1.snaps.assign(nmb * 4, 0);
    tok1::Lane1 L1;
    tok1::init1(L1, true);
    for (uint64_t st = 0; L1.k != tok1::K_DONE; st++) {
        if ((st & 7) == 0) tok1::topup1(L1, m1);  // (the device's schedule)
        tok1::step1(L1, m1);  // (as the device: a lane waiting for its MB phase steps in SINK)
        if ((st & 15) == 15)
            for (int r = 0; r < 8 && L1.k == tok1::K_MB; r++) tok1::mb1(L1, m1);
    }
    // stage 2: count, offsets, records
    static const uint32_t TT[2 * tokl::NST] = ZW_TOKL_TT_INIT;
    HostTok2Mem m2;
    m2.TT = TT;
    m2.P = &B.probs[0][0][0][0];
    m2.stream = B.part[0].d;
    m2.len = B.part[0].len;
    bool bad = false;
    moff[0] = 0;
    for (size_t i = 0; i < nmb; i++)
        moff[i + 1] = moff[i] + host_tok2_mb(m2, modes.data() + i * ZW_TOK_MODE, &m1.snaps[i * 4], 0, &bad);
    std::vector<uint8_t> rec(moff[nmb] + 16);
    m2.rec = rec.data();
    bool bad2 = false;
    for (size_t i = 0; i < nmb; i++) {
        m2.lim = moff[i + 1];
        const uint32_t sz = host_tok2_mb(m2, modes.data() + i * ZW_TOK_MODE, &m1.snaps[i * 4], moff[i], &bad2);
        if (sz != moff[i + 1] - moff[i]) return ZW_EINVAL;  // (the two passes must agree)
    }
    if (rc != ZW_OK || bad) {
        *match = (rc == ZW_EBITSTREAM && bad) ? 1 : 0;
        return rc;
    }
    *match = moff == moff_ref && !memcmp(rec.data(), ref.data(), moff_ref[nmb]) ? 1 : 0;
    return rc;
}

// ---------------------------------------------------------------------------
// WebP container, lossy subset: WebPDecoder::new -> read_data
// (decoder/api.rs:334-510) for a simple "VP8 " file or a VP8X file whose image
// is a VP8 chunk, then read_image (:640-700) + decode_rgb / decode_rgba
// (:938-993).  Lossless (VP8L), alpha (ALPH) and animation are outside the
// lossy block-transform path: ZW_EUNSUPPORTED.
// ---------------------------------------------------------------------------
namespace {
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint32_t rd24(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16); }
bool fourcc_is(const uint8_t* p, const char* s) { return memcmp(p, s, 4) == 0; }
}  // namespace

extern "C" int zw_webp_parse(const uint8_t* data, size_t len, zw_webp_info* info)
{
    if (!info || (!data && len)) return ZW_EINVAL;
    memset(info, 0, sizeof *info);
    if (len < 8) return ZW_EBITSTREAM;
    if (!fourcc_is(data, "RIFF")) return ZW_ECHUNK_HEADER;  // ChunkHeaderInvalid(b"RIFF")
    const uint64_t riff_size = rd32(data + 4);
    if (len < 12) return ZW_EBITSTREAM;
    if (!fourcc_is(data + 8, "WEBP")) return ZW_EWEBP_SIGNATURE;
    if (len < 20) return ZW_EBITSTREAM;
    const uint8_t* ch = data + 12;
    const uint64_t csize = rd32(ch + 4), crounded = csize + (csize & 1);
    const uint64_t start = 20;
    if (fourcc_is(ch, "VP8 ")) {
        if (len < start + 10) return ZW_EBITSTREAM;
        const uint32_t tag = rd24(data + start);
        if (tag & 1) return ZW_EUNSUPPORTED_FEATURE;  // non-keyframe
        const uint8_t* m = data + start + 3;
        if (m[0] != 0x9d || m[1] != 0x01 || m[2] != 0x2a) return ZW_EVP8_MAGIC;
        info->width = (data[start + 6] | (data[start + 7] << 8)) & 0x3fff;
        info->height = (data[start + 8] | (data[start + 9] << 8)) & 0x3fff;
        if (info->width == 0 || info->height == 0) return ZW_EINCONSISTENT_SIZES;
        info->is_lossy = 1;
        info->vp8_offset = start;
        info->vp8_len = csize;
    } else if (fourcc_is(ch, "VP8L")) {
        info->is_lossless = 1;
        return ZW_EUNSUPPORTED;
    } else if (fourcc_is(ch, "VP8X")) {
        if (len < start + 10) return ZW_EBITSTREAM;
        const uint8_t flags = data[start];
        info->has_alpha = (flags & 0x10) != 0;
        info->is_animated = (flags & 0x02) != 0;
        info->width = rd24(data + start + 4) + 1;
        info->height = rd24(data + start + 7) + 1;
        if ((uint64_t)info->width * info->height > 0xffffffffull) return ZW_EIMAGE_TOO_LARGE;
        uint64_t pos = start + crounded;
        const uint64_t max_pos = pos + (riff_size > 12 ? riff_size - 12 : 0);
        int have_vp8 = 0, have_vp8l = 0;
        while (pos < max_pos) {
            if (pos + 8 > len) break;  // read_chunk_header hits the end: BitStreamError -> stop scanning
            const uint8_t* c = data + pos;
            const uint64_t sz = rd32(c + 4), rsz = sz + (sz & 1);
            if (fourcc_is(c, "VP8 ") && !have_vp8) {
                have_vp8 = 1;
                info->vp8_offset = pos + 8;
                info->vp8_len = sz;
            } else if (fourcc_is(c, "VP8L")) {
                have_vp8l = 1;
            }
            pos += 8 + rsz;
        }
        info->is_lossy = have_vp8;
        info->is_lossless = have_vp8l && !have_vp8;
        if (info->is_animated || have_vp8l || info->has_alpha) return ZW_EUNSUPPORTED;
        if (!have_vp8) return ZW_ECHUNK_MISSING;
    } else {
        return ZW_ECHUNK_HEADER;
    }
    if (info->vp8_offset + info->vp8_len > len) return ZW_EBITSTREAM;
    return ZW_OK;
}

// decode_rgba_into / decode_rgb_into (decoder/api.rs:1004-1128): a lossy WebP
// file into the caller's buffer with a row stride.
extern "C" int zw_webp_decode_into(zw_ctx* ctx, const uint8_t* data, size_t len, int bpp, int upsampling, uint8_t* out,
                                   size_t out_len, uint32_t stride_bytes, uint32_t* width, uint32_t* height)
{
    if (!ctx || !out) return ZW_EINVAL;
    zw_webp_info info;
    if (int r = zw_webp_parse(data, len, &info)) return r;
    if ((size_t)stride_bytes < (size_t)info.width * bpp || out_len < (size_t)stride_bytes * info.height)
        return ZW_EINVAL;  // InvalidParameter: stride / output buffer too small
    const uint8_t* d[1] = {data + info.vp8_offset};
    const size_t l[1] = {(size_t)info.vp8_len};
    uint8_t* o[1] = {out};
    const size_t ol[1] = {out_len};
    uint32_t w = 0, h = 0;
    if (int r = dec_rgb_batch(ctx, 1, d, l, bpp, upsampling, nullptr, o, ol, stride_bytes, &w, &h)) return r;
    if (w != info.width || h != info.height) return ZW_EINCONSISTENT_SIZES;
    if (width) *width = w;
    if (height) *height = h;
    return ZW_OK;
}

extern "C" int zw_webp_decode(zw_ctx* ctx, const uint8_t* data, size_t len, int bpp, int upsampling, zw_bytes* out,
                              uint32_t* width, uint32_t* height)
{
    if (!ctx || !out) return ZW_EINVAL;
    out->data = nullptr;
    out->len = 0;
    zw_webp_info info;
    if (int r = zw_webp_parse(data, len, &info)) return r;
    uint32_t w = 0, h = 0;
    if (int r = zw_vp8_decode_rgb(ctx, data + info.vp8_offset, (size_t)info.vp8_len, bpp, upsampling, out, &w, &h))
        return r;
    if (w != info.width || h != info.height) {  // read_image: InconsistentImageSizes
        zw_bytes_free(out);
        return ZW_EINCONSISTENT_SIZES;
    }
    if (width) *width = w;
    if (height) *height = h;
    return ZW_OK;
}
