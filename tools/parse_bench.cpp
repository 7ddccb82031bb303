// Host token-parse micro-benchmark: times the decoder's own parse_header +
// parse_mbs (zw_dec_host.cpp, compiled in) on one thread over VP8 frames
// written by tools/parse_bench_streams.py, and prints an FNV-1a digest of
// every record byte and MB offset so a change to the parser can be checked
// byte for byte on the CPU before the GPU decode tests.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off tools/parse_bench.cpp -o /tmp/parse_bench \
//       -Limage-webp_amd/zwebp -lzwebp -Wl,-rpath,$PWD/image-webp_amd/zwebp
//   /tmp/parse_bench /tmp/parse_bench_0.vp8 /tmp/parse_bench_1.vp8 [reps]
#include "../image-webp_amd/csrc/zw_dec_host.cpp"

#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv)
{
    std::vector<std::vector<uint8_t>> frames;
    int reps = 20;
    for (int a = 1; a < argc; a++) {
        FILE* f = fopen(argv[a], "rb");
        if (!f) {
            reps = atoi(argv[a]);
            continue;
        }
        std::vector<uint8_t> d;
        uint8_t buf[65536];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + k);
        fclose(f);
        frames.push_back(std::move(d));
    }
    if (frames.empty()) return 2;
    uint64_t dig = 1469598103934665603ull;
    double best = 1e30;
    size_t rec_total = 0;
    for (int r = 0; r < reps; r++) {
        double t = 0;
        for (auto& fr : frames) {
            DecFrame F;
            const double t0 = dec_now_ms();
            if (parse_header(F, fr.data(), fr.size()) != ZW_OK) return 3;
            const size_t nmb = (size_t)F.mbw * F.mbh;
            static std::vector<uint8_t> recs;
            static std::vector<uint32_t> moff;
            if (recs.size() < nmb * ZW_DREC_MAX) recs.resize(nmb * ZW_DREC_MAX);
            moff.resize(nmb + 1);
            if (parse_mbs(F, recs.data(), moff.data()) != ZW_OK) return 4;
            t += dec_now_ms() - t0;
            if (r == 0) {
                const size_t used = moff[nmb];
                rec_total += used;
                for (size_t i = 0; i < used; i++) dig = (dig ^ recs[i]) * 1099511628211ull;
                for (size_t i = 0; i <= nmb; i++) dig = (dig ^ moff[i]) * 1099511628211ull;
            }
        }
        if (t < best) best = t;
    }
    printf("frames %zu  best %.3f ms/frame  records %zu B/frame  digest %016llx\n", frames.size(),
           best / frames.size(), rec_total / frames.size(), (unsigned long long)dig);
    return 0;
}
