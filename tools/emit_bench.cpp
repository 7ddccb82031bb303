// Host emission micro-benchmark: replays one frame's emission input (dumped by
// the pipeline with ZW_DUMP_EMIT=<path>) through the host coder and reports the
// time per frame and the output's size and FNV-1a hash, so that changes to the
// host coder can be timed on the CPU and checked byte-for-byte.
//   g++ -O3 -march=native -std=c++17 -I image-webp_amd/csrc tools/emit_bench.cpp -o /tmp/emit_bench
//   /tmp/emit_bench dump.bin [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "zw_host_entropy.h"

static uint64_t fnv(const std::vector<uint8_t>& v)
{
    uint64_t h = 1469598103934665603ull;
    for (uint8_t b : v) h = (h ^ b) * 1099511628211ull;
    return h;
}

template <class F>
static double best_ms(int reps, F fn)
{
    double best = 1e30;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        fn();
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < best) best = ms;
    }
    return best;
}

// coder variants (timing only; their bytes are compared with zwh::raw_codeM's)
// 64-bit low, 32 pending bits written at a time (BoolEncoder's state on exit)
template <int M, int FB = 32>
static void code64(zwh::RawBool* const* S, const uint16_t* const* d, int n)
{
    uint8_t* b[M];
    uint64_t lo[M];
    uint32_t ra[M];
    int co[M];
    size_t po[M];
    for (int k = 0; k < M; k++) {
        S[k]->reserve_more((size_t)n);
        b[k] = S[k]->buf.data();
        lo[k] = S[k]->low, ra[k] = S[k]->range, co[k] = S[k]->count + 24, po[k] = S[k]->pos;
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
            if (co[k] >= FB) {
                if (FB == 32) {
                    const uint32_t w = (uint32_t)(lo[k] >> (co[k] - 24));
                    const uint32_t be = __builtin_bswap32(w);
                    memcpy(b[k] + po[k], &be, 4);
                } else {  // FB bits: the top FB of the 8 + co bits, left-aligned in 64
                    const uint64_t w = lo[k] << (56 - co[k]);
                    const uint64_t be = __builtin_bswap64(w);
                    memcpy(b[k] + po[k], &be, 8);
                }
                po[k] += FB / 8;
                co[k] -= FB;
                lo[k] &= (1ull << (8 + co[k])) - 1;
            }
        }
    }
    for (int k = 0; k < M; k++) {
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
// 32-bit BoolEncoder with the byte output branch-free (the byte is stored
// every decision, the position advanced when it is due); only the carry branches
template <int M>
static void codebl(zwh::RawBool* const* S, const uint16_t* const* d, int n)
{
    uint8_t* b[M];
    uint32_t lo[M], ra[M];
    int co[M];
    size_t po[M];
    for (int k = 0; k < M; k++) {
        S[k]->reserve_more((size_t)n);
        b[k] = S[k]->buf.data();
        lo[k] = S[k]->low, ra[k] = S[k]->range, co[k] = S[k]->count, po[k] = S[k]->pos;
    }
    for (int i = 0; i < n; i++) {
#pragma GCC unroll 4
        for (int k = 0; k < M; k++) {
            const uint32_t D = d[k][i], prob = D & 255u, m = 0u - (D >> 8);
            const uint32_t split = 1 + (((ra[k] - 1) * prob) >> 8);
            uint32_t L = lo[k] + (split & m);
            const uint32_t r = split ^ ((split ^ (ra[k] - split)) & m);
            const int sh = __builtin_clz(r) - 24;
            ra[k] = r << sh;
            const int c = co[k] + sh;
            const bool out = c >= 0;
            // (out) offset = sh - c: the byte is L >> (24 - offset), the carry bit 32 - offset
            const int off = out ? sh - c : 1;
            if (__builtin_expect(out && ((L << (off - 1)) & 0x80000000u), 0)) {
                S[k]->pos = po[k];
                S[k]->carry(b[k]);
            }
            b[k][po[k]] = (uint8_t)(L >> (24 - off));
            po[k] += out;
            const uint32_t Lo = ((L << off) & 0xffffffu) << (c & 31);
            lo[k] = out ? Lo : (L << sh);
            co[k] = out ? c - 8 : c;
        }
    }
    for (int k = 0; k < M; k++) S[k]->low = lo[k], S[k]->range = ra[k], S[k]->count = co[k], S[k]->pos = po[k];
}

int main(int argc, char** argv)
{
    if (argc < 2) {
        fprintf(stderr, "usage: %s dump.bin [reps]\n", argv[0]);
        return 2;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 50;
    FILE* fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    uint32_t hdr[4];
    ZwFrameParams P;
    uint8_t have = 0;
    static uint8_t upd[4][8][3][11];
    unsigned long long n = 0;
    if (fread(hdr, sizeof hdr, 1, fp) != 1 || hdr[0] != 0x4d45575au || hdr[1] != sizeof(ZwFrameParams) ||
        fread(&P, sizeof P, 1, fp) != 1 || fread(&have, 1, 1, fp) != 1 || fread(upd, sizeof upd, 1, fp) != 1 ||
        fread(&n, sizeof n, 1, fp) != 1) {
        fprintf(stderr, "bad dump\n");
        return 2;
    }
    std::vector<uint8_t> rec(n);
    if (fread(rec.data(), 1, n, fp) != n) return 2;
    fclose(fp);
    const int w = (int)hdr[2], h = (int)hdr[3];

    std::vector<uint8_t> ref, out, outb[2];
    const double t_ref = best_ms(reps, [&] { zwh::emit_frame(ref, P, rec.data(), w, h, have != 0, upd); });
    printf("%dx%d: emit_frame %.3f ms, %zu bytes, fnv %016llx\n", w, h, t_ref, ref.size(), (unsigned long long)fnv(ref));
    for (int K : {1, 2, 4}) {
        std::vector<uint8_t> o[4];
        std::vector<uint8_t>* op[4] = {&o[0], &o[1], &o[2], &o[3]};
        const ZwFrameParams* Ps[4] = {&P, &P, &P, &P};
        const uint8_t* recs[4] = {rec.data(), rec.data(), rec.data(), rec.data()};
        const bool haves[4] = {have != 0, have != 0, have != 0, have != 0};
        const uint8_t(*upds[4])[8][3][11] = {upd, upd, upd, upd};
        const double t = best_ms(reps, [&] { zwh::emit_frames(op, Ps, recs, K, w, h, haves, upds); });
        bool same = true;
        for (int k = 0; k < K; k++) same = same && o[k] == ref;
        printf("  emit_frames K=%d: %.3f ms per frame, %s\n", K, t / K, same ? "identical" : "DIFFERENT");
    }
    // distinct: K = 4 different frames, as the pipeline's groups have (the same
    // frame four times lets the branch predictor learn each row's branches):
    // copy k has the MB rows rotated by 17 k rows (a valid record stream, not
    // the same bitstream), the caches swept (256 MB) before every rep
    std::vector<uint8_t> cp[16];
    {
        std::vector<size_t> row_off((size_t)P.mbh + 1);
        {
            zwh::PackedMb m;
            const uint8_t* q = rec.data();
            for (int y = 0; y < P.mbh; y++) {
                row_off[y] = (size_t)(q - rec.data());
                for (int x = 0; x < P.mbw; x++) q = zwh::view_mb(q, m);
            }
            row_off[P.mbh] = (size_t)(q - rec.data());
        }
        for (int k = 0; k < 16; k++)
            for (int y = 0; y < P.mbh; y++) {
                const int ry = (y + 17 * k + (k >= 4 ? 5 : 0)) % P.mbh;
                cp[k].insert(cp[k].end(), rec.begin() + (long)row_off[ry], rec.begin() + (long)row_off[ry + 1]);
            }
        std::vector<uint8_t> sweep((size_t)256 << 20, 1);
        for (int K : {4, 16}) {
            std::vector<uint8_t> o[16];
            std::vector<uint8_t>* op[16];
            const ZwFrameParams* Ps[16];
            const uint8_t* recs[16];
            bool haves[16];
            const uint8_t(*upds[16])[8][3][11];
            for (int k = 0; k < 16; k++) op[k] = &o[k], Ps[k] = &P, recs[k] = cp[k].data(), haves[k] = have != 0, upds[k] = upd;
            double best = 1e30, sum = 0;
            const int nr = reps < 10 ? reps : 10;
            for (int r = 0; r < nr; r++) {
                for (size_t i = 0; i < sweep.size(); i += 64) sweep[i]++;
                const auto t0 = std::chrono::steady_clock::now();
                for (int k0 = 0; k0 < 16; k0 += K) zwh::emit_frames(op + k0, Ps + k0, recs + k0, K, w, h, haves + k0, upds + k0);
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                best = ms < best ? ms : best;
                sum += ms;
            }
            printf("  distinct K=%d (16 row-rotated frames, caches swept): best %.3f, mean %.3f ms per frame%s\n", K,
                   best / 16, sum / nr / 16, K > 4 && zwh::have_code16() ? " (16-lane coder)" : "");
        }
    }
    // breakdown: the walk recording every token decision of the frame (and
    // the headers'), then the coder alone over the token decisions
    std::vector<uint16_t> all((size_t)P.mbw * P.mbh * 400 + (1 << 20)), hd((size_t)P.mbw * P.mbh * 160 + 4096);
    size_t nd = 0;
    const double t_rec = best_ms(reps, [&] {
        zwh::PackedMb m;
        uint8_t probs[4][8][3][11];
        zwh::DecRec H{hd.data()};
        zwh::emit_frame_header(H, P, have != 0, upd, 1, probs);
        static zwh::TokRes res;
        zwh::tok_resolve(res, probs);
        std::vector<zwh::Cplx> top(P.mbw, zwh::Cplx{});
        std::vector<uint8_t> top_bp((size_t)P.mbw * 4, 0);
        const uint8_t* q = rec.data();
        uint16_t* o = all.data();
        for (int y = 0; y < P.mbh; y++) {
            zwh::Cplx left{};
            uint8_t left_bp[4] = {0, 0, 0, 0};
            for (int x = 0; x < P.mbw; x++) {
                q = zwh::view_mb(q, m);
                zwh::emit_mb_header(H, P, m, top_bp.data(), left_bp, x);
                zwh::rec_mb_tokens(o, res, probs, m, left, top[x]);
            }
        }
        nd = (size_t)(o - all.data());
    });
    // the walk's parts: record parsing alone, + MB headers
    volatile int sink = 0;
    const double t_view = best_ms(reps, [&] {
        zwh::PackedMb m;
        const uint8_t* q = rec.data();
        int acc = 0;
        for (int i = 0; i < P.mbw * P.mbh; i++) {
            q = zwh::view_mb(q, m);
            acc += m.eob[3];
        }
        sink = acc;
    });
    const double t_hdr = best_ms(reps, [&] {
        zwh::PackedMb m;
        zwh::DecRec H{hd.data()};
        std::vector<uint8_t> top_bp((size_t)P.mbw * 4, 0);
        const uint8_t* q = rec.data();
        for (int y = 0; y < P.mbh; y++) {
            uint8_t left_bp[4] = {0, 0, 0, 0};
            for (int x = 0; x < P.mbw; x++) {
                q = zwh::view_mb(q, m);
                zwh::emit_mb_header(H, P, m, top_bp.data(), left_bp, x);
            }
        }
    });
    printf("  walk parts: record views %.3f ms, + MB headers %.3f ms\n", t_view, t_hdr);
    (void)sink;
    auto reset = [](zwh::RawBool& S) {
        S.lo = S.pos = 1;
        S.low = 0;
        S.range = 255;
        S.count = -24;
    };
    zwh::RawBool Q[4];
    zwh::RawBool* qp[4] = {&Q[0], &Q[1], &Q[2], &Q[3]};
    const uint16_t* dp[4] = {all.data(), all.data(), all.data(), all.data()};
    double tc[5] = {0, 0, 0, 0, 0};
    tc[1] = best_ms(reps, [&] { reset(Q[0]); zwh::raw_codeM<1>(qp, dp, (int)nd); });
    tc[2] = best_ms(reps, [&] { for (auto& x : Q) reset(x); zwh::raw_codeM<2>(qp, dp, (int)nd); });
    tc[4] = best_ms(reps, [&] { for (auto& x : Q) reset(x); zwh::raw_codeM<4>(qp, dp, (int)nd); });
    printf("  %zu token decisions (%.2f per output bit): walk+record %.3f ms; coder per stream: x1 %.3f ms "
           "(%.2f ns/decision), x2 %.3f, x4 %.3f ms\n",
           nd, (double)nd / (8.0 * (double)ref.size()), t_rec, tc[1], 1e6 * tc[1] / (double)nd, tc[2] / 2, tc[4] / 4);

    // the distinct frames: the walk alone per frame, then the coders over their
    // four decision streams (the pipeline's case for both)
    std::vector<uint16_t> d4[4];
    size_t n4[4];
    double t_walk4 = 0;
    for (int k = 0; k < 4; k++) {
        d4[k].resize((size_t)P.mbw * P.mbh * 400 + (1 << 20));
        t_walk4 += best_ms(reps, [&] {
            zwh::PackedMb m;
            uint8_t probs[4][8][3][11];
            zwh::DecRec H{hd.data()};
            zwh::emit_frame_header(H, P, have != 0, upd, 1, probs);
            static zwh::TokRes res;
            zwh::tok_resolve(res, probs);
            std::vector<zwh::Cplx> top(P.mbw, zwh::Cplx{});
            std::vector<uint8_t> top_bp((size_t)P.mbw * 4, 0);
            const uint8_t* q = cp[k].data();
            uint16_t* o = d4[k].data();
            for (int y = 0; y < P.mbh; y++) {
                zwh::Cplx left{};
                uint8_t left_bp[4] = {0, 0, 0, 0};
                for (int x = 0; x < P.mbw; x++) {
                    q = zwh::view_mb(q, m);
                    zwh::emit_mb_header(H, P, m, top_bp.data(), left_bp, x);
                    zwh::rec_mb_tokens(o, res, probs, m, left, top[x]);
                }
            }
            n4[k] = (size_t)(o - d4[k].data());
        });
    }
    int nmin = (int)std::min(std::min(n4[0], n4[1]), std::min(n4[2], n4[3]));
    const uint16_t* dp4[4] = {d4[0].data(), d4[1].data(), d4[2].data(), d4[3].data()};
    const double ta = best_ms(reps, [&] { for (auto& x : Q) reset(x); zwh::raw_codeM<4>(qp, dp4, nmin); });
    std::vector<uint8_t> outa[4];
    for (int k = 0; k < 4; k++) outa[k].assign(Q[k].buf.begin() + 1, Q[k].buf.begin() + (long)Q[k].pos);
    const double tb = best_ms(reps, [&] { for (auto& x : Q) reset(x); code64<4>(qp, dp4, nmin); });
    bool same_b = true;
    for (int k = 0; k < 4; k++) same_b &= std::vector<uint8_t>(Q[k].buf.begin() + 1, Q[k].buf.begin() + (long)Q[k].pos) == outa[k];
    const double t48 = best_ms(reps, [&] { for (auto& x : Q) reset(x); code64<4, 48>(qp, dp4, nmin); });
    bool same_48 = true;
    for (int k = 0; k < 4; k++) same_48 &= std::vector<uint8_t>(Q[k].buf.begin() + 1, Q[k].buf.begin() + (long)Q[k].pos) == outa[k];
    const double ta2 = best_ms(reps, [&] { for (auto& x : Q) reset(x); zwh::raw_codeM<4>(qp, dp4, nmin); });
    printf("  distinct frames: 64-bit, 48 bits at a time %.3f (%s); the library's again %.3f\n", t48 / 4,
           same_48 ? "same" : "DIFFERENT", ta2 / 4);
    const double tcl = best_ms(reps, [&] { for (auto& x : Q) reset(x); codebl<4>(qp, dp4, nmin); });
    bool same_c = true;
    for (int k = 0; k < 4; k++) same_c &= std::vector<uint8_t>(Q[k].buf.begin() + 1, Q[k].buf.begin() + (long)Q[k].pos) == outa[k];
    printf("  distinct frames: walk+record %.3f ms per frame; coder x4 per stream (%d decisions): branchy %.3f, "
           "64-bit %.3f (%s), branch-free bytes %.3f (%s)\n",
           t_walk4 / 4, nmin, ta / 4, tb / 4, same_b ? "same" : "DIFFERENT", tcl / 4, same_c ? "same" : "DIFFERENT");
    return 0;
}
