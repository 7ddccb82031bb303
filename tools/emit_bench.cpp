// Host emission micro-benchmark: replays one frame's emission input (dumped by
// the pipeline with ZW_DUMP_EMIT=<path>) through the host coder and reports the
// time per frame and the output's size and FNV-1a hash, so that changes to the
// host coder can be timed on the CPU and checked byte-for-byte.
//   g++ -O3 -march=native -std=c++17 -I image-webp_amd/csrc tools/emit_bench.cpp -o /tmp/emit_bench
//   /tmp/emit_bench dump.bin [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
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
    return 0;
}
