// Equivalence of the split emission (zwh::emit_frames: recorded decisions,
// K frames' coders interleaved) with zwh::emit_frame, and of the interleaved
// coder (raw_code_multi) with the reference's bit-at-a-time encoder, on
// synthetic inputs: random packed MB records (every luma mode, skips, segments,
// sub-modes, levels of every token category and sign, empty and full blocks)
// and random decision streams with long carry runs.
//   g++ -O2 -std=c++17 -I image-webp_amd/csrc tools/emit_equiv.cpp
#include <cstdio>
#include <algorithm>
#include <random>
#include "zw_host_entropy.h"

static std::mt19937 rng(11);
static int rnd(int n) { return (int)(rng() % (uint32_t)n); }

// one frame's packed records (zw_pack_kernels.hip layout, see zwh::view_mb)
static std::vector<uint8_t> synth_records(int mbw, int mbh, int style)
{
    std::vector<uint8_t> r;
    for (int i = 0; i < mbw * mbh; i++) {
        const int luma = style == 1 ? 4 : rnd(5), skip = rnd(4) == 0, seg = rnd(4), chroma = rnd(4);
        r.push_back((uint8_t)(luma | skip << 3 | seg << 4 | chroma << 6));
        if (luma == 4)
            for (int k = 0; k < 8; k++) r.push_back((uint8_t)(rnd(10) | rnd(10) << 4));
        uint8_t eob[25];
        for (int b = 0; b < 25; b++) {
            const bool y1ac = luma != 4 && b < 16;  // (DC at index 0 stays zero)
            int e = skip || (luma == 4 && b == 16) ? 0 : (rnd(3) == 0 ? 0 : rnd(17));
            if (y1ac && e == 1) e = 2;
            eob[b] = (uint8_t)e;
            r.push_back(eob[b]);
        }
        for (int b = 0; b < 25; b++)
            for (int n = 0; n < eob[b]; n++) {
                int v;
                if (luma != 4 && b < 16 && n == 0) v = 0;
                else if (n + 1 == eob[b]) v = 1 + rnd(style == 2 ? 2047 : 12);
                else v = rnd(5) ? rnd(3) : rnd(style == 2 ? 2048 : 80);
                if (rnd(2)) v = -v;
                r.push_back((uint8_t)(v & 255));
                r.push_back((uint8_t)((v >> 8) & 255));
            }
    }
    return r;
}

int main()
{
    // 1) the interleaved coder against the bit-at-a-time reference
    for (int trial = 0; trial < 30; trial++) {
        const int K = 1 + trial % 4;
        std::vector<uint16_t> d[4];
        std::vector<uint8_t> want[4];
        for (int k = 0; k < K; k++) {
            const int m = rnd(20000);
            zwh::BoolEncoderRef R;
            for (int i = 0; i < m; i++) {
                const int p = trial % 3 == 0 ? 1 + rnd(255) : (rnd(2) ? 1 + rnd(8) : 247 + rnd(9));
                int bit = rnd(256) >= p;
                if (trial % 5 == 1) bit = 1;  // long carry runs
                d[k].push_back((uint16_t)(p | bit << 8));
                R.put(bit, p);
            }
            R.flush();
            want[k] = R.buf;
        }
        zwh::RawBool S[4];
        zwh::RawBool* sp[4] = {&S[0], &S[1], &S[2], &S[3]};
        const uint16_t* dp[4];
        int n[4];
        for (int k = 0; k < K; k++) dp[k] = d[k].data(), n[k] = (int)d[k].size();
        // in pieces, as the emitter codes MB rows
        int done[4] = {0, 0, 0, 0};
        while (true) {
            int piece[4], any = 0;
            const uint16_t* pp[4];
            for (int k = 0; k < K; k++) {
                piece[k] = std::min(n[k] - done[k], rnd(3000));
                pp[k] = dp[k] + done[k];
                any |= n[k] - done[k];
            }
            if (!any) break;
            zwh::raw_code_multi(sp, pp, piece, K);
            for (int k = 0; k < K; k++) done[k] += piece[k];
        }
        for (int k = 0; k < K; k++) {
            S[k].flush();
            if (std::vector<uint8_t>(S[k].data(), S[k].data() + S[k].size()) != want[k]) {
                printf("coder MISMATCH trial %d stream %d\n", trial, k);
                return 1;
            }
        }
    }
    // 1b) the 16-lane coder (on a host with AVX-512): 5..16 streams of different
    // lengths, in pieces, against the bit-at-a-time reference
    if (zwh::have_code16()) {
        for (int trial = 0; trial < 20; trial++) {
            const int K = 5 + trial % 12;
            std::vector<uint16_t> arena;
            std::vector<size_t> at(K);
            std::vector<std::vector<uint8_t>> want(K);
            std::vector<int> len(K);
            for (int k = 0; k < K; k++) {
                const int m = rnd(12000);
                zwh::BoolEncoderRef R;
                at[k] = arena.size();
                for (int i = 0; i < m; i++) {
                    const int p = trial % 3 == 0 ? 1 + rnd(255) : (rnd(2) ? 1 + rnd(8) : 247 + rnd(9));
                    int bit = rnd(256) >= p;
                    if (trial % 5 == 1) bit = 1;
                    arena.push_back((uint16_t)(p | bit << 8));
                    R.put(bit, p);
                }
                arena.push_back(0);
                R.flush();
                want[k] = R.buf;
                len[k] = m;
            }
            arena.resize(arena.size() + 32);
            std::vector<zwh::RawBool> S(K);
            std::vector<zwh::RawBool*> sp(K);
            for (int k = 0; k < K; k++) sp[k] = &S[k];
            std::vector<int> done(K, 0);
            while (true) {
                std::vector<const uint16_t*> pp(K);
                std::vector<int> piece(K);
                int any = 0;
                for (int k = 0; k < K; k++) {
                    piece[k] = std::min(len[k] - done[k], rnd(3000));
                    pp[k] = arena.data() + at[k] + done[k];
                    any |= len[k] - done[k];
                }
                if (!any) break;
                zwh::code_streams(sp.data(), arena.data(), pp.data(), piece.data(), K);
                for (int k = 0; k < K; k++) done[k] += piece[k];
            }
            for (int k = 0; k < K; k++) {
                S[k].flush();
                if (std::vector<uint8_t>(S[k].data(), S[k].data() + S[k].size()) != want[k]) {
                    printf("coder16 MISMATCH trial %d stream %d\n", trial, k);
                    return 1;
                }
            }
        }
        printf("16-lane coder checked\n");
    } else {
        printf("(no AVX-512 here: the 16-lane coder not checked)\n");
    }
    // 2) emit_frames (K = 1..16 frames of mixed content) against emit_frame
    for (int trial = 0; trial < 40; trial++) {
        const int K = 1 + trial % 16;
        const int mbw = 1 + rnd(9), mbh = 1 + rnd(7);
        std::vector<ZwFrameParams> P(K);
        std::vector<std::vector<uint8_t>> rec(K);
        static uint8_t upd[16][4][8][3][11];
        bool have[16];
        for (int k = 0; k < K; k++) {
            ZwFrameParams& p = P[k];
            memset(&p, 0, sizeof p);
            p.width = mbw * 16 - rnd(15);
            p.height = mbh * 16 - rnd(15);
            p.mbw = mbw;
            p.mbh = mbh;
            p.seg_enabled = rnd(2);
            p.seg_update_map = p.seg_enabled && rnd(2);
            for (int i = 0; i < 3; i++) p.seg_probs[i] = (uint8_t)(rnd(3) ? 1 + rnd(254) : 255);
            for (int s = 0; s < 4; s++) p.seg[s].quantizer_level = rnd(2) ? rnd(60) - 30 : 0;
            p.base_qi = rnd(128);
            p.filter_level = rnd(64);
            p.skip_prob = 1 + rnd(254);
            have[k] = rnd(2);
            for (size_t i = 0; i < sizeof upd[k]; i++) (&upd[k][0][0][0][0])[i] = (uint8_t)(1 + rnd(255));
            rec[k] = synth_records(mbw, mbh, trial % 3);
        }
        std::vector<uint8_t> got[16], ref;
        std::vector<uint8_t>* gp[16];
        for (int k = 0; k < 16; k++) gp[k] = &got[k];
        const ZwFrameParams* pp[16];
        const uint8_t* rp[16];
        const uint8_t(*up[16])[8][3][11];
        for (int k = 0; k < K; k++) pp[k] = &P[k], rp[k] = rec[k].data(), up[k] = upd[k];
        zwh::emit_frames(gp, pp, rp, K, P[0].width, P[0].height, have, up);
        for (int k = 0; k < K; k++) {
            zwh::emit_frame(ref, P[k], rec[k].data(), P[0].width, P[0].height, have[k], upd[k]);
            if (ref != got[k]) {
                printf("emit MISMATCH trial %d frame %d (%zu vs %zu bytes)\n", trial, k, got[k].size(), ref.size());
                return 1;
            }
        }
    }
    printf("equivalent\n");
    return 0;
}
