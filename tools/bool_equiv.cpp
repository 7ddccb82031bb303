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
    // code_pair (two recorded streams coded interleaved) == each coded alone
    for (int trial = 0; trial < 20; trial++) {
        zwh::DecisionRecorder ra, rb;
        ra.reset(16);
        rb.reset(16);
        const int na = (int)(rng() % 20000), nb = trial == 3 ? 0 : (int)(rng() % 20000);
        for (int k = 0; k < 2; k++) {
            zwh::DecisionRecorder& r = k ? rb : ra;
            for (int i = 0; i < (k ? nb : na); i++) {
                const int pr = 1 + (int)(rng() % 255);
                r.put((int)(rng() % 256) >= pr || trial % 4 == 1, pr);
            }
        }
        zwh::BoolEncoder A, B, A1, B1;
        zwh::code_pair(A, ra, B, rb);
        for (size_t i = 0; i < ra.n; i++) A1.put(ra.b[i], ra.p[i]);
        for (size_t i = 0; i < rb.n; i++) B1.put(rb.b[i], rb.p[i]);
        A.flush(); B.flush(); A1.flush(); B1.flush();
        if (A.buf != A1.buf || B.buf != B1.buf) {
            printf("PAIR MISMATCH trial %d\n", trial);
            return 1;
        }
    }
    printf("equivalent\n");
    return 0;
}
