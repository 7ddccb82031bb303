// Equivalence and speed of the batched bool encoder against the reference's
// bit-at-a-time form: g++ -O2 -I image-webp_amd/csrc tools/bool_equiv.cpp
#include <chrono>
#include <cstdio>
#include <random>
#include "zw_host_entropy.h"
int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000000;
    std::mt19937 rng(7);
    for (int trial = 0; trial < 40; trial++) {
        zwh::BoolEncoder A;
        zwh::BoolEncoderRef B;
        const int m = trial < 30 ? (int)(rng() % 5000) : n;
        std::vector<uint8_t> bits(m), probs(m);
        for (int i = 0; i < m; i++) {
            probs[i] = (uint8_t)(trial % 3 == 0 ? 1 + rng() % 255 : (rng() % 2 ? 1 + rng() % 8 : 247 + rng() % 9));
            bits[i] = (uint8_t)((rng() % 256) >= probs[i]);
            if (trial % 5 == 1) bits[i] = 1;  // long carry runs
        }
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < m; i++) A.put(bits[i], probs[i]);
        A.flush();
        auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < m; i++) B.put(bits[i], probs[i]);
        B.flush();
        auto t2 = std::chrono::steady_clock::now();
        if (A.buf != B.buf) {
            printf("MISMATCH trial %d (m=%d): %zu vs %zu bytes\n", trial, m, A.buf.size(), B.buf.size());
            return 1;
        }
        if (m == n)
            printf("trial %d: %d decisions, batched %.2f ns/bit, reference %.2f ns/bit\n", trial, m,
                   std::chrono::duration<double, std::nano>(t1 - t0).count() / m,
                   std::chrono::duration<double, std::nano>(t2 - t1).count() / m);
    }
    printf("equivalent\n");
    return 0;
}
