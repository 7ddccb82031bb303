// record_coeffs (zw_host_entropy.h) against a direct
// restatement of the reference's branchy form (encoder/cost.rs:1297-1397,
// including its never-cleared skip_eob) on random blocks:
// g++ -O1 -I image-webp_amd/csrc tools/stats_equiv.cpp
#include <cstdio>
#include <random>
#include "zw_host_entropy.h"

static void rec(uint32_t& s, int bit) { zwh::rec_stat(s, bit); }
static void record_direct(zwh::Stats& S, const int16_t* lv, int eob, int t, int first, int ctx)
{
    if (eob <= first) {
        rec(S.s[t][zwh::VP8_ENC_BANDS[first]][ctx][0], 0);
        return;
    }
    int n = first, skip_eob = 0;
    while (n < eob) {
        uint32_t* st = S.s[t][zwh::VP8_ENC_BANDS[n]][ctx];
        int v = lv[n] < 0 ? -lv[n] : lv[n];
        n++;
        if (!skip_eob) rec(st[0], 1);
        if (v == 0) {
            rec(st[1], 0);
            skip_eob = 1;
            ctx = 0;
            continue;
        }
        rec(st[1], 1);
        if (v == 1) {
            rec(st[2], 0);
            ctx = 1;
        } else {
            rec(st[2], 1);
            if (v > 67) v = 67;
            if (v <= 4) {
                rec(st[3], 0);
                if (v == 2) rec(st[4], 0);
                else {
                    rec(st[4], 1);
                    rec(st[5], v == 4);
                }
            } else if (v <= 10) {
                rec(st[3], 1);
                rec(st[6], 0);
                rec(st[7], v > 6);
            } else {
                rec(st[3], 1);
                rec(st[6], 1);
                if (v < 35) {
                    rec(st[8], 0);
                    rec(st[9], v >= 19);
                } else {
                    rec(st[8], 1);
                    rec(st[10], v >= 67);
                }
            }
            ctx = 2;
        }
    }
    if (n < 16) rec(S.s[t][zwh::VP8_ENC_BANDS[n]][ctx][0], 0);
}

int main()
{
    std::mt19937 rng(3);
    zwh::Stats A, B;
    memset(&A, 0, sizeof A);
    memset(&B, 0, sizeof B);
    for (int trial = 0; trial < 400000; trial++) {  // accumulated: exercises the halving at 0xfffe0000
        int16_t lv[16] = {0};
        const int first = rng() % 2, eob = first + rng() % (17 - first);
        for (int n = first; n < eob; n++) {
            const int r = rng() % 10;
            int v = r < 4 ? 0 : (r < 7 ? 1 + rng() % 4 : (r < 9 ? rng() % 70 : rng() % 2000));
            lv[n] = (int16_t)(rng() % 2 ? -v : v);
        }
        if (eob > first && lv[eob - 1] == 0) lv[eob - 1] = 1;
        const int t = rng() % 4, ctx = rng() % 3;
        zwh::record_coeffs(A, (const uint8_t*)lv, eob, t, first, ctx);
        record_direct(B, lv, eob, t, first, ctx);
        if (memcmp(&A, &B, sizeof A)) {
            printf("MISMATCH at trial %d\n", trial);
            return 1;
        }
    }
    printf("equivalent\n");
    return 0;
}
