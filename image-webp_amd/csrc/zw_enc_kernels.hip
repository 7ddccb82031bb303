// zw_enc_kernels.hip -- device half of the lossy encoder (gfx950).
//
//   k_rgb2yuv     convert_image_yuv / convert_image_y      (decoder/yuv.rs:656, :806)
//   k_analysis    analyze_image per-MB alpha + histogram    (encoder/analysis.rs:964)
//   k_segments    k-means, segment quant, matrices, lambdas (analysis.rs:1029, :1145;
//                 vp8.rs:2278-2388, types.rs:806)
//   k_encode      one encode pass over a batch of frames:   (vp8.rs:1281-1488)
//                 RD mode search (pick_best_intra16/intra4/uv), final transform,
//                 quantization (simple or trellis), recon, error diffusion, skip.
//
// Parallel structure: one workgroup per frame, NW waves.  Macroblock rows are
// dealt to waves round-robin and advance as an x+2y wavefront (a row may work
// on MB x once the row above has finished MB x+1), synchronised through LDS
// progress counters.  Within a macroblock the 64 lanes work block-parallel.
// Pass 1's chroma is a raster chain (left_derr is not reset per row, quirk A5)
// and runs on wave 0 while waves 1..NW-1 do the luma wavefront.
#include "zw_dev.h"

// Waves per workgroup of each encode pass.  Both kernels stay within 168
// VGPRs, so three waves share each SIMD (12 per CU); ZW_NW sets both.
#ifdef ZW_NW
#define ZW_NW1 ZW_NW
#define ZW_NW2 ZW_NW
#endif
#ifndef ZW_NW1
#define ZW_NW1 12
#endif
#ifndef ZW_NW2
#define ZW_NW2 12
#endif
#define NW_MAX (ZW_NW1 > ZW_NW2 ? ZW_NW1 : ZW_NW2)
// Issue priority of a luma wave from its slack to the row above (encode_body):
// slack (MBs) per priority level, 0: off; pass 1's level width and cap.
#ifndef ZW_DYN_PRIO
#define ZW_DYN_PRIO 1
#endif
#ifndef ZW_DYN_PRIO1
#define ZW_DYN_PRIO1 2  // (1: 28.86, 2: 28.74 ms per 256 1080p frames, one-frame kernel)
#endif
#ifndef ZW_P1_LUMA_MAX
#define ZW_P1_LUMA_MAX 3  // (2 kept the luma waves below the chroma chain: 0.7 % slower)
#endif
template <int PASS> struct PassShape {
    static constexpr int NW = PASS == 1 ? ZW_NW1 : ZW_NW2;
    static constexpr int WG = NW * 64;
};

// ---------------------------------------------------------------------------
// RGB(A)/L(A) -> padded YUV420.  One thread per chroma sample; it produces the
// 2x2 luma pixels and the U/V sample.  Padding (x >= w, y >= h) is produced by
// clamping the source coordinate, which equals the reference's edge
// replication (yuv.rs:765-803).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int rgb_y(const uint8_t* p)
{
    return (16839 * p[0] + 33059 * p[1] + 6420 * p[2] + (1 << 15) + (16 << 16)) >> 16;
}
__device__ __forceinline__ int rgb_u(const uint8_t* p) { return -9719 * p[0] - 19081 * p[1] + 28800 * p[2] + (128 << 16); }
__device__ __forceinline__ int rgb_v(const uint8_t* p) { return 28800 * p[0] - 24116 * p[1] - 4684 * p[2] + (128 << 16); }

// chroma sample (cx, cy) of one frame and its 2x2 luma pixels
__device__ __forceinline__ void rgb2yuv_sample(const uint8_t* __restrict__ im, int w, int h, int bpp, int mbw, int cx,
                                               int cy, uint8_t* __restrict__ Yf, uint8_t* __restrict__ Uf,
                                               uint8_t* __restrict__ Vf)
{
    const int cw = mbw * 8, lw = mbw * 16;
    const int acw = (w + 1) / 2, ach = (h + 1) / 2;
    const int scx = cx < acw ? cx : acw - 1, scy = cy < ach ? cy : ach - 1;
    int xs[2] = {min(2 * scx, w - 1), min(2 * scx + 1, w - 1)};
    int ys[2] = {min(2 * scy, h - 1), min(2 * scy + 1, h - 1)};
    // luma: the 2x2 pixels this thread owns in the padded plane
#pragma unroll
    for (int dy = 0; dy < 2; dy++)
#pragma unroll
        for (int dx = 0; dx < 2; dx++) {
            int px = min(2 * cx + dx, w - 1), py = min(2 * cy + dy, h - 1);
            const uint8_t* p = im + ((size_t)py * w + px) * bpp;
            Yf[(size_t)(2 * cy + dy) * lw + 2 * cx + dx] = (uint8_t)(bpp <= 2 ? p[0] : rgb_y(p));
        }
    uint8_t uo = 127, vo = 127;
    if (bpp > 2) {
        int su = 0, sv = 0;
#pragma unroll
        for (int dy = 0; dy < 2; dy++)
#pragma unroll
            for (int dx = 0; dx < 2; dx++) {
                const uint8_t* p = im + ((size_t)ys[dy] * w + xs[dx]) * bpp;
                su += rgb_u(p);
                sv += rgb_v(p);
            }
        uo = (uint8_t)((su + (1 << 17)) >> 18);
        vo = (uint8_t)((sv + (1 << 17)) >> 18);
    }
    Uf[(size_t)cy * cw + cx] = uo;
    Vf[(size_t)cy * cw + cx] = vo;
}

extern "C" __global__ void k_rgb2yuv(const uint8_t* __restrict__ img, int w, int h, int bpp, int mbw, int mbh,
                                     uint8_t* __restrict__ Y, uint8_t* __restrict__ U, uint8_t* __restrict__ V,
                                     size_t img_stride, size_t ysz, size_t csz)
{
    const int cw = mbw * 8, chh = mbh * 8;
    const int f = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= cw * chh) return;
    rgb2yuv_sample(img + (size_t)f * img_stride, w, h, bpp, mbw, idx % cw, idx / cw, Y + (size_t)f * ysz,
                   U + (size_t)f * csz, V + (size_t)f * csz);
}

// Row-coalesced form for 3- and 4-byte pixels: one thread per 8x2 luma pixels
// (4 chroma samples), so a wave reads 64 consecutive 8-pixel runs of two rows
// with 16-byte (RGBA) or 8-byte (RGB) loads and writes 8-byte luma and 4-byte
// chroma words.  Runs that reach the right edge and the padding rows below the
// image take the per-sample path (edge replication).  The host launches it
// only when every run is aligned for those loads.
template <int BPP>
__device__ __forceinline__ void rgb_run8(const uint8_t* __restrict__ row, uint32_t px[8])  // 0x..BBGGRR
{
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    if (BPP == 4) {
        const u32x4 a = __builtin_nontemporal_load((const u32x4*)row);
        const u32x4 b = __builtin_nontemporal_load((const u32x4*)(row + 16));
        px[0] = a.x; px[1] = a.y; px[2] = a.z; px[3] = a.w;
        px[4] = b.x; px[5] = b.y; px[6] = b.z; px[7] = b.w;
    } else {
        const u32x2 a = __builtin_nontemporal_load((const u32x2*)row);
        const u32x2 b = __builtin_nontemporal_load((const u32x2*)(row + 8));
        const u32x2 c = __builtin_nontemporal_load((const u32x2*)(row + 16));
        const uint32_t wd[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
#pragma unroll
        for (int q = 0; q < 2; q++) {  // 4 pixels in 3 words
            const uint32_t w0 = wd[3 * q], w1 = wd[3 * q + 1], w2 = wd[3 * q + 2];
            px[4 * q] = w0;
            px[4 * q + 1] = __builtin_amdgcn_alignbyte(w1, w0, 3);
            px[4 * q + 2] = __builtin_amdgcn_alignbyte(w2, w1, 2);
            px[4 * q + 3] = w2 >> 8;
        }
    }
}

template <int BPP>
__global__ __launch_bounds__(256) void k_rgb2yuv_rows(const uint8_t* __restrict__ img, int w, int h, int mbw, int mbh,
                                                      uint8_t* __restrict__ Y, uint8_t* __restrict__ U,
                                                      uint8_t* __restrict__ V, size_t img_stride, size_t ysz,
                                                      size_t csz)
{
    const int cw = mbw * 8, chh = mbh * 8, lw = mbw * 16, gpr = mbw * 2;  // 4-sample groups per chroma row
    const int f = blockIdx.y;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= gpr * chh) return;
    const int g = idx % gpr, cy = idx / gpr;
    const int cx0 = 4 * g, px0 = 8 * g;
    const uint8_t* im = img + (size_t)f * img_stride;
    uint8_t* Yf = Y + (size_t)f * ysz;
    uint8_t* Uf = U + (size_t)f * csz;
    uint8_t* Vf = V + (size_t)f * csz;
    if (px0 + 8 <= w && cy < (h + 1) / 2) {
        const int r0 = 2 * cy, r1 = min(2 * cy + 1, h - 1);
        uint32_t a[8], b[8];
        rgb_run8<BPP>(im + ((size_t)r0 * w + px0) * BPP, a);
        rgb_run8<BPP>(im + ((size_t)r1 * w + px0) * BPP, b);
        const uint32_t ya[2] = {pk_y4(a[0], a[1], a[2], a[3]), pk_y4(a[4], a[5], a[6], a[7])};
        const uint32_t yb[2] = {pk_y4(b[0], b[1], b[2], b[3]), pk_y4(b[4], b[5], b[6], b[7])};
        uint32_t uw = 0, vw = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int su = pk_u(a[2 * j]) + pk_u(a[2 * j + 1]) + pk_u(b[2 * j]) + pk_u(b[2 * j + 1]) + (512 << 16);
            const int sv = pk_v(a[2 * j]) + pk_v(a[2 * j + 1]) + pk_v(b[2 * j]) + pk_v(b[2 * j + 1]) + (512 << 16);
            uw |= (uint32_t)((su + (1 << 17)) >> 18) << (8 * j);
            vw |= (uint32_t)((sv + (1 << 17)) >> 18) << (8 * j);
        }
        *(uint2*)(Yf + (size_t)(2 * cy) * lw + px0) = make_uint2(ya[0], ya[1]);
        *(uint2*)(Yf + (size_t)(2 * cy + 1) * lw + px0) = make_uint2(yb[0], yb[1]);
        *(uint32_t*)(Uf + (size_t)cy * cw + cx0) = uw;
        *(uint32_t*)(Vf + (size_t)cy * cw + cx0) = vw;
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) rgb2yuv_sample(im, w, h, BPP, mbw, cx0 + j, cy, Yf, Uf, Vf);
    }
}

// ---------------------------------------------------------------------------
// Analysis (analysis.rs:964): one wave per MB.  Lanes 0..31: luma (mode DC/TM
// x 16 blocks), lanes 32..47: chroma (mode x 8 blocks).  Predictors use source
// pixels; on the MB-padded planes libwebp's import/replicate rules reduce to
// direct reads (analysis.rs:520-745).
// ---------------------------------------------------------------------------
// One wave per MB: the MB and its edge pixels staged in LDS.
struct AnalysisTile {
    uint32_t y[16][4];     // luma rows, 4 packed pixels per word
    uint32_t c[2][8][2];   // U, V rows
    uint32_t ytop[4], ctop[2][2];
    uint8_t yleft[16], cleft[2][8];
    uint8_t corner[4];     // Y, U, V
};

#ifndef ZW_AN_MPW
#define ZW_AN_MPW 8
#endif
extern "C" __global__ __launch_bounds__(256) void k_analysis(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U,
                                                             const uint8_t* __restrict__ V, int mbw, int mbh,
                                                             size_t ysz, size_t csz, uint8_t* __restrict__ alpha,
                                                             uint32_t* __restrict__ histo)
{
    __shared__ uint32_t hist[4][4][32];  // [wave][histogram][bin]
    __shared__ AnalysisTile tile[4];
    __shared__ uint32_t ahist[256];      // the workgroup's share of the frame's alpha histogram
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int f = blockIdx.y;
    const int nmb = mbw * mbh;
    ahist[threadIdx.x] = 0;
    __syncthreads();
    const int ys = mbw * 16, cs = mbw * 8;
    const uint8_t* Yf = Y + (size_t)f * ysz;
    const uint8_t* Uf = U + (size_t)f * csz;
    const uint8_t* Vf = V + (size_t)f * csz;
    // This lane's share of an MB and its edges (coalesced u32 loads): y = one
    // luma word; x = a chroma word (lanes < 32), the top row (32..39) or a left
    // pixel (40..63); x2 = the V left pixel (56..63); corner (lanes < 3).
    // Branch-free: every lane issues the same three dword loads at lane-computed
    // addresses (a byte is taken from its aligned dword when the MB is staged; a
    // lane with nothing to fetch reads the frame's first word and discards it),
    // so the next MB's loads stay in flight while this MB is analysed (a
    // lane-divergent if-chain of loads made the compiler wait for each in turn).
    //   y: one luma word;  x: lanes 0..31 chroma words (plane lane >> 4, row
    //   (lane >> 1) & 7), 32..35 the luma top row, 36..39 the chroma top rows,
    //   40..55 the luma left column (bytes), 56..63 the U left column (bytes);
    //   z: lanes 0..2 the Y / U / V corner, 56..63 the V left column (bytes).
    struct AnFetch {
        uint32_t y, xw, zw;
        uint32_t m;  // bits 0..4: x byte shift, 5: x ok, 6: x is a byte; 8..12: z shift, 13: z ok
    };
    auto fetch = [&](int mb) {
        AnFetch r = {0u, 0u, 0u, 0u};
        if (mb >= nmb) return r;
        const int mbx = mb % mbw, mby = mb / mbw;
        const bool ht = mby > 0, hl = mbx > 0;
        r.y = *(const uint32_t*)(Yf + (size_t)(mby * 16 + (lane >> 2)) * ys + mbx * 16 + 4 * (lane & 3));
        const int rr = (lane >> 1) & 7, w = lane & 1, cr = lane - 56;
        const uint8_t* xp;
        size_t xo;
        bool xok = true, xbyte = false;
        if (lane < 32) {
            xp = lane >> 4 ? Vf : Uf;
            xo = (size_t)(mby * 8 + rr) * cs + mbx * 8 + 4 * w;
        } else if (lane < 36) {
            xp = Yf;
            xo = (size_t)(mby * 16 - 1) * ys + mbx * 16 + 4 * (lane - 32);
            xok = ht;
        } else if (lane < 40) {
            xp = ((lane - 36) >> 1) ? Vf : Uf;
            xo = (size_t)(mby * 8 - 1) * cs + mbx * 8 + 4 * w;
            xok = ht;
        } else if (lane < 56) {
            xp = Yf;
            xo = (size_t)(mby * 16 + lane - 40) * ys + mbx * 16 - 1;
            xok = hl;
            xbyte = true;
        } else {
            xp = Uf;
            xo = (size_t)(mby * 8 + cr) * cs + mbx * 8 - 1;
            xok = hl;
            xbyte = true;
        }
        const int zsz = lane == 0 ? 16 : 8, zst = lane == 0 ? ys : cs;
        const uint8_t* zp = lane < 3 ? (lane == 0 ? Yf : (lane == 1 ? Uf : Vf)) : Vf;
        const size_t zo = lane < 3 ? (size_t)(mby * zsz - 1) * zst + mbx * zsz - 1 : (size_t)(mby * 8 + cr) * cs + mbx * 8 - 1;
        const bool zok = lane < 3 ? (ht && hl) : (lane >= 56 && hl);
        xo = xok ? xo : 0;
        const size_t zo2 = zok ? zo : 0;
        r.xw = *(const uint32_t*)((xok ? xp : Yf) + (xo & ~(size_t)3));
        r.zw = *(const uint32_t*)((zok ? zp : Yf) + (zo2 & ~(size_t)3));
        r.m = (uint32_t)(8 * (xo & 3)) | (xok ? 32u : 0u) | (xbyte ? 64u : 0u) | ((uint32_t)(8 * (zo2 & 3)) << 8) |
              (zok ? 0x2000u : 0u);
        return r;
    };
    // ZW_AN_MPW MBs per wave, the workgroup's 4 waves on adjacent MBs; each
    // MB's loads are issued one MB ahead
    AnFetch nx = fetch(blockIdx.x * ZW_AN_MPW * 4 + wv);
    for (int k = 0; k < ZW_AN_MPW; k++) {
    const int mb = (blockIdx.x * ZW_AN_MPW + k) * 4 + wv;
    const AnFetch cur = nx;
    if (k + 1 < ZW_AN_MPW) nx = fetch(mb + 4);
    wsync();
    if (mb < nmb) {
        const int mbx = mb % mbw, mby = mb / mbw;
        // ---- stage the MB and its edges in LDS ----
        // tiles: [plane][row][col] with interior rows 0..15 / 0..7, top row, left column, corner
        AnalysisTile* A = &tile[wv];
        const bool ht = mby > 0, hl = mbx > 0;
        const uint32_t xm = (cur.m & 32u) ? ((cur.m & 64u) ? (cur.xw >> (cur.m & 31u)) & 255u : cur.xw) : 0u;
        const uint8_t zb = (cur.m & 0x2000u) ? (uint8_t)(cur.zw >> ((cur.m >> 8) & 31u)) : (uint8_t)0;
        A->y[lane >> 2][lane & 3] = cur.y;
        if (lane < 32) A->c[lane >> 4][(lane >> 1) & 7][lane & 1] = xm;
        else if (lane < 36) A->ytop[lane - 32] = xm;
        else if (lane < 40) A->ctop[(lane - 36) >> 1][lane & 1] = xm;
        else if (lane < 56) A->yleft[lane - 40] = (uint8_t)xm;
        else {
            A->cleft[0][lane - 56] = (uint8_t)xm;
            A->cleft[1][lane - 56] = zb;
        }
        if (lane < 3) A->corner[lane] = zb;
        wsync();
        uint8_t bins[16];
        uint32_t z = 0;
        int vmax = 0, hidx = 0;
        if (lane < 48) {
            // libwebp analysis predictors on source pixels (analysis.rs:259-490, quirk A21):
            // lane 0..31 luma (mode = lane >> 4: DC, TM; block lane & 15), 32..47 chroma
            // (mode (lane-32) >> 3, block (lane-32) & 7: U 0..3, V 4..7)
            const bool luma = lane < 32;
            const int mode = luma ? (lane >> 4) : ((lane - 32) >> 3);
            const int b = luma ? (lane & 15) : ((lane - 32) & 7);
            const int pl = b >> 2;  // chroma plane
            const int bb = luma ? b : (b & 3);
            const int bx = luma ? (bb & 3) : (bb & 1), by = luma ? (bb >> 2) : (bb >> 1);
            // edge sums (v_sad_u8 over 4 packed bytes)
            uint32_t st = 0, sl = 0;
            if (luma) {
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    st = __builtin_amdgcn_sad_u8(A->ytop[w], 0u, st);
                    sl = __builtin_amdgcn_sad_u8(((const uint32_t*)A->yleft)[w], 0u, sl);
                }
            } else {
#pragma unroll
                for (int w = 0; w < 2; w++) {
                    st = __builtin_amdgcn_sad_u8(A->ctop[pl][w], 0u, st);
                    sl = __builtin_amdgcn_sad_u8(((const uint32_t*)A->cleft[pl])[w], 0u, sl);
                }
            }
            const uint32_t s2 = ht && hl ? st + sl : (ht ? 2 * st : 2 * sl);
            const int dcv = (ht || hl) ? (luma ? (int)((s2 + 16) >> 5) : (int)((s2 + 8) >> 4)) : 0x80;
            const int corner = A->corner[luma ? 0 : 1 + pl];
            int d[16];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int r = by * 4 + i;
                const uint32_t srow = luma ? A->y[r][bx] : A->c[pl][r][bx];
                const int L = luma ? A->yleft[r] : A->cleft[pl][r];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int cidx = bx * 4 + j;
                    const uint32_t tw = luma ? A->ytop[cidx >> 2] : A->ctop[pl][cidx >> 2];
                    const int T = (int)((tw >> (8 * (cidx & 3))) & 255u);
                    const int tm = (ht && hl) ? clamp255(L + T - corner) : (hl ? L : (ht ? T : 129));
                    const int p = mode == 0 ? dcv : tm;
                    d[i * 4 + j] = (int)((srow >> (8 * j)) & 255u) - p;
                }
            }
            // forward_dct_4x4 (analysis.rs:172) == dct4x4 for residuals in [-255, 255]:
            // (X + 1812) >> 9 == (8X + 14500) >> 12 and (X + 937) >> 9 == (8X + 7500) >> 12
            int o[16];
            fdct16_pk(d, o);
            hidx = luma ? mode : 2 + mode;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                bins[k] = (uint8_t)min(iabs(o[k]) >> 3, 31);
                z += bins[k] == 0;
                vmax = max(vmax, (int)bins[k]);
            }
        }
        // Fast path: when bin 0 holds at least half of a histogram's
        // coefficients (256 luma, 128 chroma), no other bin can exceed it, so
        // max_value = that count and last_non_zero = the largest bin index.
        // Sums over the 8-lane groups, then the luma 16-lane groups.
        // (DPP: quad xor 1, quad xor 2, row half mirror give each 8-lane group's
        // total in all its lanes; the row mirror then pairs the row's two groups)
        uint32_t zs = z;
        int vm = vmax;
        zs += (uint32_t)DPP((int)zs, 0xB1);
        vm = max(vm, DPP(vm, 0xB1));
        zs += (uint32_t)DPP((int)zs, 0x4E);
        vm = max(vm, DPP(vm, 0x4E));
        zs += (uint32_t)DPP((int)zs, 0x141);
        vm = max(vm, DPP(vm, 0x141));
        {
            const uint32_t zo = (uint32_t)DPP((int)zs, 0x140);
            const int vo = DPP(vm, 0x140);
            if (lane < 32) {
                zs += zo;
                vm = max(vm, vo);
            }
        }
        const uint32_t ncoef = lane < 32 ? 256u : 128u;
        const bool slow = __ballot(lane < 48 && 2 * zs < ncoef) != 0ull;
        if (slow) {
            // bin 0 holds most coefficients: count it in the lane, add the rest
            // with (far less contended) LDS atomics
            for (int i = lane; i < 128; i += 64) (&hist[wv][0][0])[i] = 0;
            wsync();
            if (lane < 48) {
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (bins[k]) atomicAdd(&hist[wv][hidx][bins[k]], 1u);
                if (z) atomicAdd(&hist[wv][hidx][0], z);
            }
            wsync();
        }
        // per histogram: max count and last non-empty bin (get_alpha,
        // analysis.rs:160), two histograms per pass, lane = (histogram, bin)
        int av[4];
        if (!slow) {
            const int ah = zs > 1 ? (int)(510u * (uint32_t)vm / zs) : 0;
            av[0] = __builtin_amdgcn_readlane(ah, 0);
            av[1] = __builtin_amdgcn_readlane(ah, 16);
            av[2] = __builtin_amdgcn_readlane(ah, 32);
            av[3] = __builtin_amdgcn_readlane(ah, 40);
        } else {
#pragma unroll
            for (int ps = 0; ps < 2; ps++) {
                const uint32_t c = hist[wv][2 * ps + (lane >> 5)][lane & 31];
                uint32_t mx = c;
                mx = max(mx, (uint32_t)DPP((int)mx, 0xB1));
                mx = max(mx, (uint32_t)DPP((int)mx, 0x4E));
                mx = max(mx, (uint32_t)DPP((int)mx, 0x141));
                mx = max(mx, (uint32_t)DPP((int)mx, 0x140));
                mx = max(mx, (uint32_t)__shfl_xor((int)mx, 16));
                const uint32_t half = (uint32_t)(__ballot(c > 0) >> (lane & 32));
                const int lnz = half ? 31 - __clz((int)half) : 1;
                const int ah = mx > 1 ? (int)(510u * (uint32_t)lnz / mx) : 0;
                av[2 * ps] = __builtin_amdgcn_readlane(ah, 0);
                av[2 * ps + 1] = __builtin_amdgcn_readlane(ah, 32);
            }
        }
        const int a0 = av[0], a1 = av[1], a2 = av[2], a3 = av[3];
        if (lane == 0) {
            int best = max(-1, max(a0, a1));
            int buv = max(-1, max(a2, a3));
            int al = (3 * best + buv + 2) >> 2;
            al = 255 - al;
            al = al < 0 ? 0 : (al > 255 ? 255 : al);
            alpha[(size_t)f * nmb + mb] = (uint8_t)al;
            atomicAdd(&ahist[al], 1u);
        }
    }
    }
    __syncthreads();
    const uint32_t c = ahist[threadIdx.x];
    if (c) atomicAdd(&histo[(size_t)f * 256 + threadIdx.x], c);
}

// ---------------------------------------------------------------------------
// The same analysis, four MBs a wave (ZW_AN_FORM 4): 16 lanes an MB, lane j
// working three of the MB's 48 (block, mode) items -- luma block j under DC
// and under TM, chroma block j & 7 (U 0-3, V 4-7) under mode j >> 3 -- so every
// lane has work and the four MBs' chains overlap.  Items, histograms and the
// alpha are those of k_analysis above, computed in the same order.
// ---------------------------------------------------------------------------
// One item: its 16 coefficient bins (min(|c| >> 3, 31)), the count of bin 0 and the largest bin.
DI void an_item(const AnalysisTile* A, bool luma, int mode, int b, bool ht, bool hl, int bins[16], int& z, int& vmax)
{
    const int pl = b >> 2;  // chroma plane
    const int bb = luma ? b : (b & 3);
    const int bx = luma ? (bb & 3) : (bb & 1), by = luma ? (bb >> 2) : (bb >> 1);
    uint32_t st = 0, sl = 0;
    if (luma) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
            st = __builtin_amdgcn_sad_u8(A->ytop[w], 0u, st);
            sl = __builtin_amdgcn_sad_u8(((const uint32_t*)A->yleft)[w], 0u, sl);
        }
    } else {
#pragma unroll
        for (int w = 0; w < 2; w++) {
            st = __builtin_amdgcn_sad_u8(A->ctop[pl][w], 0u, st);
            sl = __builtin_amdgcn_sad_u8(((const uint32_t*)A->cleft[pl])[w], 0u, sl);
        }
    }
    const uint32_t s2 = ht && hl ? st + sl : (ht ? 2 * st : 2 * sl);
    const int dcv = (ht || hl) ? (luma ? (int)((s2 + 16) >> 5) : (int)((s2 + 8) >> 4)) : 0x80;
    const int corner = A->corner[luma ? 0 : 1 + pl];
    int d[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = by * 4 + i;
        const uint32_t srow = luma ? A->y[r][bx] : A->c[pl][r][bx];
        const int L = luma ? A->yleft[r] : A->cleft[pl][r];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int cidx = bx * 4 + j;
            const uint32_t tw = luma ? A->ytop[cidx >> 2] : A->ctop[pl][cidx >> 2];
            const int T = (int)((tw >> (8 * (cidx & 3))) & 255u);
            const int tm = (ht && hl) ? clamp255(L + T - corner) : (hl ? L : (ht ? T : 129));
            const int p = mode == 0 ? dcv : tm;
            d[i * 4 + j] = (int)((srow >> (8 * j)) & 255u) - p;
        }
    }
    int o[16];
    fdct16_pk(d, o);
    z = 0;
    vmax = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        bins[k] = min(iabs(o[k]) >> 3, 31);
        z += bins[k] == 0;
        vmax = max(vmax, bins[k]);
    }
}
DI int max8(int v)  // max within aligned 8-lane groups
{
    v = max(v, DPP(v, 0xB1));
    v = max(v, DPP(v, 0x4E));
    return max(v, DPP(v, 0x141));
}
DI int an_red8(int v)  // sum within aligned 8-lane groups
{
    v += DPP(v, 0xB1);
    v += DPP(v, 0x4E);
    return v + DPP(v, 0x141);
}
DI int max16(int v)
{
    v = max8(v);
    return max(v, DPP(v, 0x140));
}
typedef unsigned an_v4u __attribute__((ext_vector_type(4)));
typedef unsigned an_v2u __attribute__((ext_vector_type(2)));
#ifndef ZW_AN4_GPW
#define ZW_AN4_GPW 1  // 4-MB groups per wave (measured, analysis + segments per 256 1080p frames: 1 1.375, 2 1.47, 4 1.41 ms)
#endif
extern "C" __global__ __launch_bounds__(256) void k_analysis4(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ U,
                                                              const uint8_t* __restrict__ V, int mbw, int mbh,
                                                              size_t ysz, size_t csz, uint8_t* __restrict__ alpha,
                                                              uint32_t* __restrict__ histo)
{
    __shared__ AnalysisTile tile[4][4];   // [wave][MB]
    __shared__ uint32_t hist[4][4][4][32];  // [wave][MB][histogram][bin] (only when some bin 0 is short)
    __shared__ uint32_t ahist[256];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, mi = lane >> 4, j = lane & 15;
    const int f = blockIdx.y;
    const int nmb = mbw * mbh;
    ahist[threadIdx.x] = 0;
    __syncthreads();
    const int ys = mbw * 16, cs = mbw * 8;
    const uint8_t* Yf = Y + (size_t)f * ysz;
    const uint8_t* Uf = U + (size_t)f * csz;
    const uint8_t* Vf = V + (size_t)f * csz;
    AnalysisTile* A = &tile[wv][mi];
#pragma unroll 1
    for (int it = 0; it < ZW_AN4_GPW; it++) {
        const int mb = ((blockIdx.x * ZW_AN4_GPW + it) * 4 + wv) * 4 + mi;
        const bool in = mb < nmb;
        const int mbx = in ? mb % mbw : 0, mby = in ? mb / mbw : 0;
        const bool ht = mby > 0, hl = mbx > 0;
        // ---- stage the MB and its edges (lane j: luma row j, chroma row j & 7 of plane j >> 3)
        {
            const int pl = j >> 3, cr = j & 7;
            const uint8_t* Cf = pl ? Vf : Uf;
            an_v4u yr = {0u, 0u, 0u, 0u};
            an_v2u cw = {0u, 0u};
            uint32_t yl = 0, cl = 0;
            if (in) {
                const uint8_t* yp = Yf + (size_t)(mby * 16 + j) * ys + mbx * 16;
                const uint8_t* cp = Cf + (size_t)(mby * 8 + cr) * cs + mbx * 8;
                yr = *(const an_v4u*)yp;
                cw = *(const an_v2u*)cp;
                if (hl) {
                    yl = yp[-1];
                    cl = cp[-1];
                }
            }
            wsync();  // (the previous group's reads of the tile are done)
            *(an_v4u*)A->y[j] = yr;
            *(an_v2u*)A->c[pl][cr] = cw;
            A->yleft[j] = (uint8_t)yl;
            A->cleft[pl][cr] = (uint8_t)cl;
            if (j < 6) {
                uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
                if (in && ht) {
                    if (j == 0) {
                        const an_v4u t = *(const an_v4u*)(Yf + (size_t)(mby * 16 - 1) * ys + mbx * 16);
                        t0 = t.x; t1 = t.y; t2 = t.z; t3 = t.w;
                    } else if (j < 3) {
                        const an_v2u t = *(const an_v2u*)((j == 1 ? Uf : Vf) + (size_t)(mby * 8 - 1) * cs + mbx * 8);
                        t0 = t.x; t1 = t.y;
                    } else if (hl) {
                        const uint8_t* cp = j == 3 ? Yf + (size_t)(mby * 16 - 1) * ys + mbx * 16 - 1
                                                   : (j == 4 ? Uf : Vf) + (size_t)(mby * 8 - 1) * cs + mbx * 8 - 1;
                        t0 = *cp;
                    }
                }
                if (j == 0) {
                    A->ytop[0] = t0; A->ytop[1] = t1; A->ytop[2] = t2; A->ytop[3] = t3;
                } else if (j < 3) {
                    A->ctop[j - 1][0] = t0;
                    A->ctop[j - 1][1] = t1;
                } else {
                    A->corner[j - 3] = (uint8_t)t0;
                }
            }
            wsync();
        }
        // ---- the three items: luma block j under DC (A) and TM (B), chroma block j & 7 under mode j >> 3 (C)
        int bins[16], zA, vA, zB, vB, zC, vC;
        an_item(A, true, 0, j, ht, hl, bins, zA, vA);
        an_item(A, true, 1, j, ht, hl, bins, zB, vB);
        an_item(A, false, j >> 3, j & 7, ht, hl, bins, zC, vC);
        // per histogram (luma DC, luma TM, chroma DC in lanes j < 8, chroma TM in j >= 8):
        // the bin-0 count and the largest bin
        const int z0 = red16(zA), z1 = red16(zB), z23 = an_red8(zC);
        const int v0 = max16(vA), v1 = max16(vB), v23 = max8(vC);
        // fast path (k_analysis): bin 0 holding at least half of a histogram's
        // coefficients is its largest count, and the last non-empty bin is the largest bin
        const bool ok = 2 * z0 >= 256 && 2 * z1 >= 256 && 2 * z23 >= 128;
        int a0, a1, a23;
        if (__ballot(in && !ok) == 0ull) {
            a0 = z0 > 1 ? (int)(510u * (uint32_t)v0 / (uint32_t)z0) : 0;
            a1 = z1 > 1 ? (int)(510u * (uint32_t)v1 / (uint32_t)z1) : 0;
            a23 = z23 > 1 ? (int)(510u * (uint32_t)v23 / (uint32_t)z23) : 0;
        } else {
            // exact histograms: bin 0 counted in the lane, the other bins by LDS atomics
            uint32_t* H = &hist[wv][mi][0][0];
#pragma unroll
            for (int k = 0; k < 8; k++) (&hist[wv][0][0][0])[64 * k + lane] = 0;
            wsync();
#pragma unroll 1
            for (int t = 0; t < 3; t++) {
                int zz, vv;
                const int h = t < 2 ? t : 2 + (j >> 3);
                an_item(A, t < 2, t < 2 ? t : j >> 3, t < 2 ? j : j & 7, ht, hl, bins, zz, vv);
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (bins[k]) atomicAdd(&H[h * 32 + bins[k]], 1u);
                if (zz) atomicAdd(&H[h * 32], (uint32_t)zz);
            }
            wsync();
            int av[4];
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const uint32_t c0 = H[h * 32 + 2 * j], c1 = H[h * 32 + 2 * j + 1];
                const int mx = max16((int)max(c0, c1));
                const int lnz = max16(c1 ? 2 * j + 1 : (c0 ? 2 * j : -1));
                av[h] = mx > 1 ? (int)(510u * (uint32_t)max(lnz, 0) / (uint32_t)mx) : 0;
            }
            a0 = av[0];
            a1 = av[1];
            a23 = j < 8 ? av[2] : av[3];
        }
        const int a3 = __shfl(a23, (lane & ~15) | 8);  // chroma TM's, from lane 8 of the MB
        if (j == 0 && in) {
            const int best = max(-1, max(a0, a1));
            const int buv = max(-1, max(a23, a3));
            int al = (3 * best + buv + 2) >> 2;
            al = 255 - al;
            al = al < 0 ? 0 : (al > 255 ? 255 : al);
            alpha[(size_t)f * nmb + mb] = (uint8_t)al;
            atomicAdd(&ahist[al], 1u);
        }
    }
    __syncthreads();
    const uint32_t c = ahist[threadIdx.x];
    if (c) atomicAdd(&histo[(size_t)f * 256 + threadIdx.x], c);
}

// ---------------------------------------------------------------------------
// Segments: one thread per frame.  k-means over the alpha histogram
// (assign_segments_kmeans analysis.rs:1029), per-segment quant via the
// reference's f64 fast_math pow (compute_segment_quant :1145; this file is
// built with -ffp-contract=off), matrices/lambdas (Segment::init_matrices
// types.rs:806), segment tree probabilities (vp8.rs:2340-2368).
// ---------------------------------------------------------------------------
__device__ double fm_log2(double x)
{
    unsigned long long bits = __double_as_longlong(x);
    long long e = (long long)((bits >> 52) & 0x7FF) - 1023;
    unsigned long long mb = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
    double m = __longlong_as_double((long long)mb);
    double y = (m - 1.0) / (m + 1.0);
    double y2 = y * y;
    const double C0 = 2.8853900817779268, C1 = 0.9617966939259756, C2 = 0.5770780163555854,
                 C3 = 0.4121985831111324, C4 = 0.3205988987531030;
    double poly = C0 + y2 * (C1 + y2 * (C2 + y2 * (C3 + y2 * C4)));
    return (double)e + y * poly;
}
__device__ double fm_exp2(double x)
{
    if (x < -1022.0) x = -1022.0;
    if (x > 1023.0) x = 1023.0;
    long long xi = x >= 0.0 ? (long long)x : (long long)x - 1;
    double xf = x - (double)xi;
    const double LN2 = 0.6931471805599453;
    const double C1 = LN2, C2 = LN2 * LN2 / 2.0, C3 = LN2 * LN2 * LN2 / 6.0, C4 = LN2 * LN2 * LN2 * LN2 / 24.0,
                 C5 = LN2 * LN2 * LN2 * LN2 * LN2 / 120.0;
    double poly = 1.0 + xf * (C1 + xf * (C2 + xf * (C3 + xf * (C4 + xf * C5))));
    double scale = __longlong_as_double((long long)((unsigned long long)(xi + 1023) << 52));
    return poly * scale;
}
__device__ double fm_pow(double x, double n)
{
    if (x <= 0.0) return 0.0;
    if (x == 1.0 || n == 0.0) return 1.0;
    if (n == 1.0) return x;
    return fm_exp2(n * fm_log2(x));
}
__device__ int segment_quant(int base, int alpha, int sns)
{
    double amp = 0.9 * (double)sns / 100.0 / 128.0;
    double expn = 1.0 - amp * (double)alpha;
    if (expn <= 0.0) return base;
    double cb = 1.0 - ((double)base / 127.0);
    double c = fm_pow(cb, expn);
    int q = (int)(127.0 * (1.0 - c));
    return q < 0 ? 0 : (q > 127 ? 127 : q);
}

__device__ void matrix_init(ZwMatrix& m, int qdc, int qac, int bdc, int bac)
{
    m.q[0] = (uint32_t)qdc;
    m.q[1] = (uint32_t)qac;
    for (int i = 0; i < 2; i++) {
        uint32_t b = i ? bac : bdc;
        m.iq[i] = (1u << 17) / m.q[i];
        m.bias[i] = ((b << 17) + 128) >> 8;
        m.zthresh[i] = ((1u << 17) - 1 - m.bias[i]) / m.iq[i];
    }
}

__device__ void segment_init(ZwSegment& s, int qi, int delta)
{
    int ydc = d_DC_QUANT[qi], yac = d_AC_QUANT[qi];
    int y2dc = d_DC_QUANT[qi] * 2;
    int y2ac = (int)d_AC_QUANT[qi] * 155 / 100;
    if (y2ac < 8) y2ac = 8;
    int uvdc = d_DC_QUANT[qi], uvac = d_AC_QUANT[qi];
    matrix_init(s.y1, ydc, yac, 96, 110);
    matrix_init(s.y2, y2dc, y2ac, 96, 108);
    matrix_init(s.uv, uvdc, uvac, 110, 115);
    for (int i = 0; i < 16; i++) {
        uint32_t q = i == 0 ? (uint32_t)ydc : (uint32_t)yac;
        s.sharpen[i] = (uint16_t)(((uint32_t)d_VP8_FREQ_SHARPENING[i] * q) >> 11);
    }
    uint32_t qi4 = ((uint32_t)ydc + 15u * (uint32_t)yac + 8) >> 4;
    uint32_t qi16 = ((uint32_t)y2dc + 15u * (uint32_t)y2ac + 8) >> 4;
    uint32_t quv = ((uint32_t)uvdc + 15u * (uint32_t)uvac + 8) >> 4;
#define MAX1(v) ((v) ? (v) : 1u)
    s.lt_i4 = MAX1((7 * qi4 * qi4) >> 3);
    s.lt_i16 = MAX1((qi16 * qi16) >> 2);
    s.lt_uv = MAX1((quv * quv) << 1);
    s.l_i4 = MAX1((3 * qi4 * qi4) >> 7);
    s.l_i16 = MAX1(3 * qi16 * qi16);
    s.l_uv = MAX1((3 * quv * quv) >> 6);
    s.l_mode = MAX1((qi4 * qi4) >> 7);
#undef MAX1
    s.tlambda = (50 * qi4) >> 5;
    s.quant_index = qi;
    s.quantizer_level = delta;
}

// Consumes the frame's alpha histogram and clears it for the next launch of
// k_analysis (zeroed once at pipeline creation; no per-launch memset blit).
extern "C" __global__ void k_segments(uint32_t* __restrict__ histo, const ZwFrameParams* __restrict__ tmpl,
                                      ZwFrameParams* __restrict__ params, int nframes)
{
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    ZwFrameParams P = *tmpl;
    const int base = P.base_qi;
    const int nmb = P.mbw * P.mbh;
    for (int i = 0; i < 4; i++) segment_init(P.seg[i], base, 0);
    for (int i = 0; i < 256; i++) P.seg_map_lut[i] = 0;
    P.seg_probs[0] = P.seg_probs[1] = P.seg_probs[2] = 255;
    P.seg_enabled = 0;
    P.seg_update_map = 0;
    if (nmb >= 256) {
        const uint32_t* H = histo + (size_t)f * 256;
        uint8_t centers[4] = {0, 0, 0, 0};
        uint8_t* map = P.seg_map_lut;
        int min_a = 0, max_a = 255;
        for (int n = 0; n < 256; n++)
            if (H[n] > 0) { min_a = n; break; }
        for (int n = 255; n >= min_a; n--)
            if (H[n] > 0) { max_a = n; break; }
        int range = max_a > min_a ? max_a - min_a : 0;
        for (int k = 0; k < 4; k++) centers[k] = (uint8_t)(min_a + ((1 + 2 * k) * range) / 8);
        uint32_t accum[4], dacc[4];
        int wa = 0;
        uint32_t tw = 0;
        for (int it = 0; it < 6; it++) {
            for (int i = 0; i < 4; i++) accum[i] = dacc[i] = 0;
            int cc = 0;
            for (int a = min_a; a <= max_a; a++) {
                if (H[a] > 0) {
                    while (cc + 1 < 4) {
                        int dc = iabs(a - centers[cc]), dn = iabs(a - centers[cc + 1]);
                        if (dn < dc) cc++;
                        else break;
                    }
                    map[a] = (uint8_t)cc;
                    dacc[cc] += (uint32_t)a * H[a];
                    accum[cc] += H[a];
                }
            }
            int displaced = 0;
            wa = 0;
            tw = 0;
            for (int n = 0; n < 4; n++) {
                if (accum[n] > 0) {
                    uint8_t nc = (uint8_t)((dacc[n] + accum[n] / 2) / accum[n]);
                    displaced += iabs(centers[n] - nc);
                    centers[n] = nc;
                    wa += (int)nc * (int)accum[n];
                    tw += accum[n];
                }
            }
            if (displaced < 5) break;
        }
        int mid = tw > 0 ? (wa + (int)tw / 2) / (int)tw : 128;
        int minc = centers[0], maxc = centers[0];
        for (int i = 1; i < 4; i++) {
            minc = min(minc, (int)centers[i]);
            maxc = max(maxc, (int)centers[i]);
        }
        int rng = maxc == minc ? 1 : maxc - minc;
        for (int s = 0; s < 4; s++) {
            int ta = 255 * ((int)centers[s] - mid) / rng;
            ta = ta < -127 ? -127 : (ta > 127 ? 127 : ta);
            int sq = segment_quant(base, ta, 50);
            int delta = (int)(int8_t)((int8_t)sq - (int8_t)base);
            segment_init(P.seg[s], sq, delta);
        }
        uint32_t cnt[4] = {0, 0, 0, 0};
        for (int a = 0; a < 256; a++) cnt[map[a]] += H[a];
        uint32_t t01 = cnt[0] + cnt[1], t23 = cnt[2] + cnt[3];
#define GETP(a, b) ((a) + (b) == 0 ? 255 : (uint8_t)((255 * (a) + ((a) + (b)) / 2) / ((a) + (b))))
        P.seg_probs[0] = GETP(t01, t23);
        P.seg_probs[1] = GETP(cnt[0], cnt[1]);
        P.seg_probs[2] = GETP(cnt[2], cnt[3]);
#undef GETP
        P.seg_update_map = P.seg_probs[0] != 255 || P.seg_probs[1] != 255 || P.seg_probs[2] != 255;
        P.seg_enabled = 1;
    }
    params[f] = P;
    uint4* Hz = (uint4*)(histo + (size_t)f * 256);
    for (int i = 0; i < 64; i++) Hz[i] = make_uint4(0u, 0u, 0u, 0u);
}

// ---------------------------------------------------------------------------
// The encode pass.
// ---------------------------------------------------------------------------
struct EncArgs {
    const uint8_t *Y, *U, *V;
    const uint8_t* alpha;       // per MB (segment lookup)
    const ZwFrameParams* params;
    const ZwLevelCosts* lcost;  // per frame; null in pass 1 (all-zero tables, quirk A2)
    int8_t* derr;               // [nframes][mbw][4] top_derr: pass 1 writes, pass 2 reads
    ZwMbOut* out;
    uint8_t *ry, *ru, *rv;      // reconstruction (pass 2), may be null
    size_t ysz, csz;
    int mbw, mbh, pass;
    int* dbg;                   // optional pass-2 I4 dump (16*34 ints per MB), may be null
    uint8_t* rows;              // row-parallel kernels: zero-filled ZW_ROWS_HDR + nframes * RowsLayout::frame
    uint32_t* sizes;            // pass 2, may be null: per MB its packed record size (zw_pack_kernels.hip)
    int nframes;                // frames of the launch (the frame-pair kernel's last workgroup may hold one)
};

// Per-MB LDS state: what lives from an MB's first search to its stores (the
// staged source, the luma work buffer with the I4 search's reconstruction, the
// levels and sub-modes) and the MB row's left contexts.  A wave working two
// rows at once (the paired kernels) keeps one per row.
struct MbLds {
    uint8_t sy[256], su[64], sv[64];  // source MB (staged per MB)
    uint8_t ws[17 * ZW_BPS];      // luma work buffer (create_border_luma layout)
    uint8_t left_y[20], left_u[12], left_v[12], left_c[12];
    int8_t left_derr[4];
    uint8_t modes[16];
    int16_t lev[25][16];
};

// per-wave LDS scratch
struct WaveLds {
    MbLds mb;                     // the wave's (first) row
    uint8_t cu[9 * ZW_BPS], cv[9 * ZW_BPS];
    uint32_t uvc[64][8];          // pick_uv -> final_chroma, per lane: its coefficients (i16 pairs) + rows' pred
    int dc[64];
    int y2d[64];
    int y2cost[4];
    int V[2][40];                 // I4 value vectors of the (up to) two sub-blocks of a search step
    int nzt[4], nzl[4];
    int misc[16];
    uint32_t pst[2][4];           // paired kernels: per MB {lm | need << 4 | seg << 8, i16 score lo, hi, i4 nz | win << 16}
    // row-parallel kernels: this MB's slice of the row above's state (top_y of
    // the MB and of the MB above-right, top_u/v, top_c, top_derr), pulled from
    // and pushed to global memory around each MB
    uint8_t win_y[32], win_u[8], win_v[8], win_c[12];
    int8_t win_d[4];
#ifdef ZW_PHASE_PROF
    unsigned long long ph[24];
#endif
};


struct Ctx {
    const EncArgs* a;
    const ZwFrameParams* P;
    int method;           // EncoderParams method (wave-uniform, read once)
    const ZwSegment* S;   // the MB's segment, in LDS
    const ZwSegment* Sl;  // the frame's 4 segments, in LDS
    const LdsTables* T;
    WaveLds* W;
    MbLds* M;             // the MB's per-row state (&W->mb, or the paired row's)
    uint8_t *top_y, *top_u, *top_v, *top_c;
    int8_t* top_derr;
    const uint8_t *srcY, *srcU, *srcV;  // MB origin (HBM)
    const uint8_t *sY, *sU, *sV;        // the same MB staged in LDS (strides 16 / 8)
    int ys, cs;
    int mbx, mby, lane, seg;
    int f;                  // frame of the launch
    int oy, oc, ocx, od;    // offsets of this MB in top_y / top_u,v / top_c / top_derr
                            // (mbx*16, *8, *12, *4; 0 in the row-parallel kernels, whose
                            // top_* point at the wave's per-MB window)
};

// create_border_luma (prediction.rs:15) into C.M->ws
// part 0: corner, top and left (everything the I16 search reads: available once
// the MB above is done); part 1: the top-right pixels (row 0 columns 17..31 and
// their copies at rows 4, 8, 12; the I4 search needs the MB above-right);
// part 2: both.
__device__ void build_luma_border(const Ctx& C, int part = 2)
{
    uint8_t* ws = C.M->ws;
    const int l = C.lane;
    const int mbw = C.a->mbw;
    const bool want = part == 2 || (part == 0 ? (l < 17 || l >= 32) : (l >= 17 && l < 32));
    // row 0 entries 0..31
    if (!want) {
    } else if (l < 32) {
        int v;
        if (l == 0) v = C.mby == 0 ? 127 : (C.mbx == 0 ? 129 : C.M->left_y[0]);
        else if (C.mby == 0) v = 127;
        else if (l <= 16) v = C.top_y[C.oy + l - 1];
        else if (C.mbx == mbw - 1) v = C.top_y[C.oy + 15];
        else v = C.top_y[C.oy + l - 1];
        ws[l] = (uint8_t)v;
        if (l >= 17 && l < 21) {
            ws[4 * ZW_BPS + l] = (uint8_t)v;
            ws[8 * ZW_BPS + l] = (uint8_t)v;
            ws[12 * ZW_BPS + l] = (uint8_t)v;
        }
    } else if (l < 48) {
        int i = l - 32;
        ws[(i + 1) * ZW_BPS] = C.mbx == 0 ? 129 : C.M->left_y[1 + i];
    }
    wsync();
}

// create_border_chroma (prediction.rs:85) into cu / cv
__device__ void build_chroma_border(const Ctx& C)
{
    const int l = C.lane;
    if (l < 34) {  // per plane: corner, 8 top, 8 left
        const int pl = l >= 17;
        const int i = pl ? l - 17 : l;
        uint8_t* w = pl ? C.W->cv : C.W->cu;
        const uint8_t* top = pl ? C.top_v : C.top_u;
        const uint8_t* left = pl ? C.M->left_v : C.M->left_u;
        if (i == 0) w[0] = C.mby == 0 ? 127 : (C.mbx == 0 ? 129 : left[0]);
        else if (i <= 8) w[i] = C.mby == 0 ? 127 : top[C.oc + i - 1];
        else w[(i - 8) * ZW_BPS] = C.mbx == 0 ? 129 : left[i - 8];
    }
    wsync();
}

// pick_best_intra16 (vp8.rs:1504-1687).  lane = mode*16 + block.
template <int PASS>
__device__ void pick_i16(const Ctx& C, int& best_mode, unsigned long long& best_score)
{
    const int lane = C.lane, m = lane >> 4, b = lane & 15, bx = b & 3, by = b >> 2;
    const uint8_t* ws = C.M->ws;
    const ZwSegment& S = *C.S;
    const LdsTables* T = C.T;
    const int above = C.mby != 0, left = C.mbx != 0;
    int dcv;
    {  // DC predictor: lanes 0..15 top row, 16..31 left column
        const int top = lane < 16;
        const int v = (int)ws[csel(top, 1 + b, (b + 1) * ZW_BPS)] & -(int)(lane < 32 && (top ? above : left));
        const int sum = red16(v);
        const int s = __builtin_amdgcn_readlane(sum, 0) + __builtin_amdgcn_readlane(sum, 16);
        const int shf = 3 + above + left;
        dcv = (!above && !left) ? 128 : ((s + (1 << (shf - 1))) >> shf);
    }
    int src[16], pr[16], r[16], c[16];
    {
        const int P0 = ws[0];
        int L[4], Tp[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            L[i] = ws[(by * 4 + i + 1) * ZW_BPS];
            Tp[i] = ws[1 + bx * 4 + i];
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t srow = *(const uint32_t*)(C.sY + (by * 4 + i) * 16 + bx * 4);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int p = sel4(m, dcv, Tp[j], L[i], clamp255(L[i] + Tp[j] - P0));
                const int sv = (int)((srow >> (8 * j)) & 255u);
                src[i * 4 + j] = sv;
                pr[i * 4 + j] = p;
                r[i * 4 + j] = sv - p;
            }
        }
    }
    fdct16_pk(r, c);
    int aq[16], dq[16];
    aq[0] = 0;
    int nzac = 0;
#pragma unroll
    for (int k = 1; k < 16; k++) {
        aq[k] = (int)((__umul24((uint32_t)iabs(c[k]), S.y1.iq[1]) + S.y1.bias[1]) >> 17);
        nzac |= aq[k];
        dq[k] = m24(c[k] < 0 ? -aq[k] : aq[k], (int)S.y1.q[1]);
    }
    nzac = nzac != 0;
    int cost = (int)rcost_bf<1, PASS == 2>(aq, 0, 0, T);
    // Y2 in group form: lane (m, b) holds block b's DC under mode m
    int y2cost;
    {
        const int d = wht_g(c[0], b);
        const int t = b > 0;
        const int ay = (int)((__umul24((uint32_t)iabs(d), S.y2.iq[t]) + S.y2.bias[t]) >> 17);
        const int qy = d < 0 ? -ay : ay;
        y2cost = (int)rcost_g<0, PASS == 2>(qy, b, 0, 1, T);  // uniform within the mode's group
        dq[0] = iwht_g(m24(qy, (int)S.y2.q[t]), b);
    }
    idct16(dq);
    int rec[16], sse = 0, flat = 1;
    const int s00 = C.sY[0];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        rec[k] = clamp255(pr[k] + dq[k]);
        const int d = src[k] - rec[k];
        sse += m24(d, d);
        flat &= src[k] == s00;
    }
    int td = iabs(ttransform_diff_pk(rec, src)) >> 5;
    sse = red16(sse);
    td = red16(td);
    cost = red16(cost);
    nzac = red16(nzac);
    flat = red16(flat);
    // per mode (uniform within the 16-lane group), decided on the scalar unit
    const int srcflat = __builtin_amdgcn_readlane(flat, 0) == 16;  // mode-0 group covers all 256 pixels
    cost += y2cost;
    int sd = S.tlambda > 0 ? ((int)S.tlambda * td + 128) >> 8 : 0;
    int dfin = sse;
    if (srcflat && nzac == 0) {
        dfin = sse * 2;
        sd = sd * 2;
    }
    const int mcost = sel4(m, d_FIXED_COSTS_I16[0], d_FIXED_COSTS_I16[1], d_FIXED_COSTS_I16[2], d_FIXED_COSTS_I16[3]) + cost;
    const int dist = dfin + sd;
    long long brd = 0x7fffffffffffffffLL, bfin = 0;
    int bm = 0;
#pragma unroll
    for (int mm = 0; mm < 4; mm++) {
        const long long mc = __builtin_amdgcn_readlane(mcost, mm * 16);
        const long long dd = 256LL * __builtin_amdgcn_readlane(dist, mm * 16);
        const long long r_m = mc * (long long)S.l_i16 + dd;
        const long long f_m = mc * (long long)S.l_mode + dd;
        const int avail = mm == 0 || (mm == 1 && above) || (mm == 2 && left) || (mm == 3 && above && left);
        if (avail && r_m < brd) {
            brd = r_m;
            bfin = f_m;
            bm = mm;
        }
    }
    best_mode = bm;
    best_score = bfin < 0 ? 0ull : (unsigned long long)bfin;
}

#ifdef ZW_PHASE_PROF
// Per-phase cycle counters (profiling builds only): [pass-1][phase].
__device__ unsigned long long zw_phase_cycles_dev[2][24];
__device__ unsigned long long zw_wave_cycles_dev[2][16][24];  // the same per wave index
#define PH_START() long long ph_t_ = clock64()
#define PH_RESET() (ph_t_ = clock64())
#define PH_MARK(k) PH_MARK_L(k, lane, PASS)
// accumulate in the wave's LDS slot; flushed once per kernel (ph_flush)
#define PH_MARK_L(k, ln, ps)                                                        \
    do {                                                                            \
        const long long n_ = clock64();                                             \
        if ((ln) == 0) C.W->ph[k] += (unsigned long long)(n_ - ph_t_);               \
        ph_t_ = n_;                                                                 \
    } while (0)
extern "C" int zw_wave_cycles(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(zw_wave_cycles_dev), sizeof(zw_wave_cycles_dev)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long z[2][16][24];
        if (hipMemcpyToSymbol(HIP_SYMBOL(zw_wave_cycles_dev), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
extern "C" int zw_phase_cycles(unsigned long long* out, int reset)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(zw_phase_cycles_dev), sizeof(zw_phase_cycles_dev)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long z[2][24];
        if (hipMemcpyToSymbol(HIP_SYMBOL(zw_phase_cycles_dev), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#define PH_COUNT(k) \
    do {                \
        if (C.lane == 0) C.W->ph[k] += 1; \
    } while (0)
#elif defined(ZW_ASM_MARKS)
#define PH_COUNT(k) (void)0
// ISA inspection builds: phase boundaries as assembly comments
#define PH_START() asm volatile("; ZWMARK start" ::: "memory")
#define PH_RESET() (void)0
#define PH_MARK(k) asm volatile("; ZWMARK " #k ::: "memory")
#define PH_MARK_L(k, ln, ps) asm volatile("; ZWMARK " #k ::: "memory")
#else
#define PH_COUNT(k) (void)0
#define PH_START() (void)0
#define PH_RESET() (void)0
#define PH_MARK(k) (void)0
#define PH_MARK_L(k, ln, ps) (void)0
#endif

// Fill the I4 value vectors V[h] for the NB sub-blocks (x0[h], y0[h]) of
// C.M->ws (branch-free: every lane reads up to three edge pixels and forms an
// avg2/avg3/copy; the lane -> (edge indices, weights) map is block invariant).
//   V[0..12]  E = [L3 L2 L1 L0 P A0..A7]      V[13..23] avg3(E[k], E[k+1], E[k+2])
//   V[24..35] avg2(E[k], E[k+1])              V[36] avg3(A6,A7,A7)  V[37] avg3(L2,L3,L3)
//   V[38] DC = (4 + L0..L3 + A0..A3) >> 3
template <int NB>
__device__ __forceinline__ void i4_values_n(const Ctx& C, const int* x0, const int* y0)
{
    WaveLds* W = C.W;
    const uint8_t* ws = C.M->ws;
    const int l = C.lane;
    // lane -> (ka, kb, kc) and weights; t: 0 copy, 1 avg3, 2 avg2, 3/4 special avg3
    // (arithmetic only: lane-dependent selects must not become branches)
    const int t = (int)(l >= 13) + (int)(l >= 24) + (int)(l >= 36) + (int)(l >= 37);
    const int k = min(l - 13 * (int)(l >= 13) - 11 * (int)(l >= 24), 12);
    const int t3 = (int)(t == 3), t4 = (int)(t >= 4), t12 = (int)(t == 1 || t == 2);
    const int ka = k + t3 * (11 - k) + t4 * (1 - k);
    const int kb = k + t12 + t3 * (12 - k) - t4 * k;
    const int kc = min(k + 2 * (int)(t == 1), 12);
    // v = (ea + wb*eb + wc*ec + rnd) >> sh
    const int wb = 2 * (int)(t == 1) + (int)(t == 2) + 3 * (t3 + t4);
    const int wc = (int)(t == 1);
    const int sh = (int)(t != 0) + (int)(t != 0 && t != 2);
    const int oa = csel(ka < 4, -ka * ZW_BPS, ka - 4 - 4 * ZW_BPS);  // offsets from rowL = (y0+3)*BPS + x0-1
    const int ob = csel(kb < 4, -kb * ZW_BPS, kb - 4 - 4 * ZW_BPS);
    const int oc = csel(kc < 4, -kc * ZW_BPS, kc - 4 - 4 * ZW_BPS);
    const bool dcl = l < 4 || (l >= 5 && l < 9);
    int v[NB], ea[NB];
#pragma unroll
    for (int h = 0; h < NB; h++) {
        const int rowL = (y0[h] + 3) * ZW_BPS + x0[h] - 1;
        ea[h] = ws[rowL + oa];
        const int eb = ws[rowL + ob], ec = ws[rowL + oc];
        v[h] = (ea[h] + wb * eb + wc * ec + ((1 << sh) >> 1)) >> sh;
    }
#pragma unroll
    for (int h = 0; h < NB; h++) {
        const int dsum = red16(dcl ? ea[h] : 0);
        if (l < 38) W->V[h][l] = v[h];
        if (l == 0) W->V[h][38] = (dsum + 4) >> 3;
    }
    wsync();
}
__device__ __forceinline__ void i4_values(const Ctx& C, int x0, int y0) { i4_values_n<1>(C, &x0, &y0); }

__device__ __forceinline__ int bperm(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }

// V index of pixel p under I4 mode `mode`, with bit 8 set for TrueMotion
// (pred = clamp(V[ia] + V[5 + col] - V[4])).  Sub-block independent.
__device__ __forceinline__ int i4_src_index(const LdsTables* T, int mode, int p)
{
    const int idx = T->i4idx[mode][p];
    const bool tm = idx == 254;
    return csel(tm, 256 + 3 - (p >> 2), csel(idx == 255, 38, idx));
}
__device__ __forceinline__ int i4_pred_at(const int* V, int sidx, int vbc)
{
    const int va = V[sidx & 255];
    return csel(sidx >= 256, clamp255(va + vbc), va);
}

__device__ __forceinline__ unsigned long long rdscore(uint32_t sse, uint32_t rate, uint32_t lambda)
{
    return (unsigned long long)sse * 256ull + (unsigned long long)(uint16_t)rate * lambda;
}

// Running state of the I4 search (pick_best_intra4, vp8.rs:1790-2040).
struct I4State {
    unsigned long long running;  // sum of the chosen blocks' rd scores (+ 211 * lambda_mode)
    uint32_t total_mc;           // header-bit cap accumulator (vp8.rs:1839)
    unsigned long long mpack;    // chosen sub-modes, 4 bits each (raster index)
    uint32_t tnz, lnz;           // nonzero flags of the chosen blocks: bit sbx / bit sby
    uint32_t nzm;                // nonzero flags of the chosen blocks: bit = raster index
};

// Unsigned minimum within aligned 16-lane rows (DPP row rotations), in every lane.
DI uint32_t min16u(uint32_t v)
{
    v = min(v, (uint32_t)DPP((int)v, 0x128));
    v = min(v, (uint32_t)DPP((int)v, 0x124));
    v = min(v, (uint32_t)DPP((int)v, 0x122));
    v = min(v, (uint32_t)DPP((int)v, 0x121));
    return v;
}

// ---------------------------------------------------------------------------
// Chroma in lane-pair form.  A 4x4 chroma block is worked by two lanes, l and
// l ^ 32 (half h = l >> 5): the pixel rows 2h, 2h+1 for prediction, residual,
// the fDCT row pass, the iDCT row pass and the reconstruction, the coefficient
// columns 2h, 2h+1 for the fDCT column pass, quantisation, rate and the iDCT
// column pass.  The halves trade intermediate values with v_permlane32_swap
// (four swaps per transform), so each lane does half of a block's arithmetic
// and the search over 4 modes x 8 blocks fills all 64 lanes.  Pixel rows are
// held as i16 pairs (x0, x1), (x3, x2) (the fdct16_pk layout).
// ---------------------------------------------------------------------------
// Both halves' copies of v: r[0] holds the lower half's value in every lane of
// the upper half, r[1] the upper half's in every lane of the lower half.
__device__ __forceinline__ int hx_partner(int v)
{
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (__lane_id() < 32) ? (int)r[1] : (int)r[0];
}
__device__ __forceinline__ int hx_sum(int v)  // v(l) + v(l ^ 32), in both lanes
{
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (int)r[0] + (int)r[1];
}
DI int lo16(uint32_t v) { return (int)(int16_t)(v & 0xffffu); }
DI int hi16(uint32_t v) { return (int)(int16_t)(v >> 16); }

// The lane's two pixel rows of chroma block (bx, by) under 8x8 mode m (0 DC,
// 1 V, 2 H, 3 TM; predict_dcpred / vpred / hpred / tmpred): pred(i, j) =
// clamp(rowv(i) + colv(j)) with (rowv, colv) = (dc, 0) / (0, T[j]) / (L[i], 0)
// / (L[i] - P, T[j]); source and prediction as i16 pairs.
DI void uv_rows_pk(const uint8_t* w, const uint8_t* sblk, int bx, int by, int h, int m, int dc, uint32_t s01[2],
                   uint32_t s32[2], uint32_t p01[2], uint32_t p32[2])
{
    const int cm = -(int)(m & 1), rm = -(int)(m >= 2);
    const int P = w[0];
    const int ro = csel(m == 0, dc, csel(m == 3, -P, 0));
    const uint8_t* tp = w + 1 + bx * 4;
    const uint32_t c01 = pack_lo(tp[0] & cm, tp[1] & cm), c32 = pack_lo(tp[3] & cm, tp[2] & cm);
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const int y = 2 * h + r;
        const int rv = (w[(by * 4 + y + 1) * ZW_BPS] & rm) + ro;
        const uint32_t rvv = pack_lo(rv, rv);
        p01[r] = clamp_pk(add_pk(c01, rvv));
        p32[r] = clamp_pk(add_pk(c32, rvv));
        const uint32_t sw = *(const uint32_t*)(sblk + y * 8);
        s01[r] = __builtin_amdgcn_perm(0u, sw, 0x0c010c00u);
        s32[r] = __builtin_amdgcn_perm(0u, sw, 0x0c020c03u);
    }
}

// dct4x4 (transform.rs:176) of the pair's block: this lane's coefficients of
// columns 2h, 2h+1, cf[col][row] = coefficient (row, 2h + col).
DI void fdct_pair(const uint32_t s01[2], const uint32_t s32[2], const uint32_t p01[2], const uint32_t p32[2], int h,
                  int cf[2][4])
{
    // row pass (fdct16_pk first stage), outputs of this lane's columns (own*)
    // and of the partner's columns (oth*)
    const zs2 k8p = {8, 8}, k8m = {8, -8}, k1a = {10704, 4434}, k1b = {4434, -10704};
    const uint32_t kA0 = h ? as_zu(k8m) : as_zu(k8p), kA1 = h ? as_zu(k8p) : as_zu(k8m);
    const uint32_t kD0 = h ? as_zu(k1b) : as_zu(k1a), kD1 = h ? as_zu(k1a) : as_zu(k1b);
    const int rD0 = h ? 1875 : 3625, rD1 = h ? 3625 : 1875;
    int own0[2], own1[2], oth0[2], oth1[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t R01 = sub_pk(s01[r], p01[r]), R32 = sub_pk(s32[r], p32[r]);
        const uint32_t A = add_pk(R01, R32), D = sub_pk(R01, R32);
        own0[r] = dot2v(A, kA0, 0);
        oth0[r] = dot2v(A, kA1, 0);
        own1[r] = dot2v(D, kD0, rD0) >> 10;
        oth1[r] = dot2v(D, kD1, rD1) >> 10;
    }
    // the partner's rows of this lane's columns
    const uint32_t g0 = (uint32_t)hx_partner((int)pack_lo(oth0[0], oth0[1]));
    const uint32_t g1 = (uint32_t)hx_partner((int)pack_lo(oth1[0], oth1[1]));
    const zs2 k1p = {1, 1}, k1m = {1, -1}, k2a = {5352, 2217}, k2b = {2217, -5352};
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int* ow = c ? own1 : own0;
        const uint32_t g = c ? g1 : g0;
        // column = rows (0, 1) and (3, 2): own rows are 2h, 2h+1, the partner's the others
        const uint32_t fwd = pack_lo(ow[0], ow[1]), rev = pack_lo(ow[1], ow[0]);
        const uint32_t grev = __builtin_amdgcn_alignbit(g, g, 16);
        const uint32_t X01 = h ? g : fwd, X32 = h ? rev : grev;
        const zs2 A = as_zs2(X01) + as_zs2(X32), D = as_zs2(X01) - as_zs2(X32);
        cf[c][0] = dot2(A, k1p, 7) >> 4;
        cf[c][2] = dot2(A, k1m, 7) >> 4;
        cf[c][1] = (dot2(D, k2a, 12000) >> 16) + ((as_zu(D) & 0xffffu) != 0u ? 1 : 0);
        cf[c][3] = dot2(D, k2b, 51000) >> 16;
    }
}

// idct4x4 (transform.rs:19, i32 form of idct16) of the pair's dequantised
// coefficients dq[col][row] (columns 2h, 2h+1), then the reconstruction
// clamp(pred + residual) of this lane's two rows as i16 pairs (x0,x1),(x3,x2).
DI void idct_recon_pair(const int dq[2][4], const uint32_t p01[2], const uint32_t p32[2], int h, uint32_t r01[2],
                        uint32_t r32[2])
{
    uint32_t lo[2], hi[2];  // vertical pass of this lane's columns: rows (0,1), (2,3)
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int x0 = dq[c][0], x1 = dq[c][1], x2 = dq[c][2], x3 = dq[c][3];
        const int a1 = x0 + x2, b1 = x0 - x2;
        const int c1 = (m24(x1, 35468) >> 16) - (x3 + (m24(x3, 20091) >> 16));
        const int d1 = (x1 + (m24(x1, 20091) >> 16)) + (m24(x3, 35468) >> 16);
        lo[c] = pack_lo(a1 + d1, b1 + c1);
        hi[c] = pack_lo(b1 - c1, a1 - d1);
    }
    // the partner needs these columns at its rows, this lane the partner's columns at its own
    const uint32_t g0 = (uint32_t)hx_partner((int)(h ? lo[0] : hi[0]));
    const uint32_t g1 = (uint32_t)hx_partner((int)(h ? lo[1] : hi[1]));
    const uint32_t m0 = h ? hi[0] : lo[0], m1 = h ? hi[1] : lo[1];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        // values of row 2h + r at columns 0..3
        const int e0 = r ? hi16(m0) : lo16(m0), e1 = r ? hi16(m1) : lo16(m1);
        const int f0 = r ? hi16(g0) : lo16(g0), f1 = r ? hi16(g1) : lo16(g1);
        const int y0 = h ? f0 : e0, y1 = h ? f1 : e1, y2 = h ? e0 : f0, y3 = h ? e1 : f1;
        const int a1 = y0 + y2, b1 = y0 - y2;
        const int c1 = (m24(y1, 35468) >> 16) - (y3 + (m24(y3, 20091) >> 16));
        const int d1 = (y1 + (m24(y1, 20091) >> 16)) + (m24(y3, 35468) >> 16);
        const int o0 = (a1 + d1 + 4) >> 3, o1 = (b1 + c1 + 4) >> 3, o2 = (b1 - c1 + 4) >> 3, o3 = (a1 - d1 + 4) >> 3;
        r01[r] = clamp_pk(add_pk(pack_lo(o0, o1), p01[r]));
        r32[r] = clamp_pk(add_pk(pack_lo(o3, o2), p32[r]));
    }
}

// get_residual_cost (cost.rs:1670, quirk A1: positions are natural indices) of
// a lane pair's block, first position 0: av[col][row] = |level| at natural
// index n = 4 row + 2h + col.  Returns the block's rate in 1/256 bits, uniform
// in the pair.  LC = false: the LevelCosts tables are zero (pass 1, quirk A2)
// and lfc[0] == 0, so positions past the last nonzero level add nothing.
template <bool LC>
DI int rcost_pair(const int av[2][4], int h, int ctx0, int ctype, const LdsTables* T, int& last_o)
{
    unsigned nzbits = 0, big = 0;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int n = 4 * r + 2 * h + c;
            nzbits |= (unsigned)min(av[c][r], 1) << n;
            big |= (unsigned)(av[c][r] >= 2) << n;
        }
    nzbits |= (unsigned)hx_partner((int)nzbits);
    big |= (unsigned)hx_partner((int)big);
    const int last = 31 - __clz((int)nzbits);
    last_o = last;
    int part = 0;
    if (LC) {
        // predecessor contexts from the partner's second column (2(1-h)+1), 2 bits per row
        unsigned sc = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) sc |= (unsigned)min(av[1][r], 2) << (2 * r);
        const unsigned rc = (unsigned)hx_partner((int)sc);
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int n = 4 * r + 2 * h + c;
                int ctx;
                if (c == 1) ctx = min(av[0][r], 2);
                else if (r == 0) ctx = h ? (int)(rc & 3u) : ctx0;  // n = 2: column 1 of row 0; n = 0: ctx0
                else ctx = h ? (int)((rc >> (2 * r)) & 3u) : (int)((rc >> (2 * r - 2)) & 3u);
                const int a = av[c][r];
                const int tl = T->lfc[min(a, 2047)] + T->lc[ctype][band_of(n)][ctx][min(a, 67)];
                part += tl & -(int)(n <= last);
            }
    } else {
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int r = 0; r < 4; r++) part += T->lfc[min(av[c][r], 2047)];
    }
    const int sum = hx_sum(part);
    const int ctx_t = ((big >> max(last, 0)) & 1u) ? 2 : 1;
    const int tail = (int)T->beob[ctype][band_of(min(last + 1, 15))][ctx_t] & -(int)(last < 15);
    const int head = (int)T->binit[ctype][0][ctx0] & -(int)(ctx0 == 0);
    return csel(last < 0, (int)T->beob[ctype][0][ctx0], head + sum + tail);  // (no divergent branch)
}

// Chroma DC predictors of both planes (uniform values): lanes 0..15 sum U,
// 16..31 V; lane i < 8 reads left pixel i, i >= 8 top pixel i - 8.
__device__ __forceinline__ void uv_dc_preds(const Ctx& C, int& dcU, int& dcV)
{
    const int l = C.lane, pl = (l >> 4) & 1, i = l & 15;
    const uint8_t* w = pl ? C.W->cv : C.W->cu;
    const int above = C.mby != 0, left = C.mbx != 0;
    const int v = (int)w[csel(i < 8, (i + 1) * ZW_BPS, i - 7)] & -(int)(i < 8 ? left : above);
    const int sum = red16(v);
    const int su = __builtin_amdgcn_readlane(sum, 0), sv = __builtin_amdgcn_readlane(sum, 16);
    const int shf = 2 + left + above;
    dcU = (above | left) ? (su + (1 << (shf - 1))) >> shf : 128;
    dcV = (above | left) ? (sv + (1 << (shf - 1))) >> shf : 128;
}

// pick_best_uv (vp8.rs:2050-2200): lane pair (l, l ^ 32) = mode * 8 + block
// (U blocks 0..3, V 4..7).  Each lane leaves its coefficients (i16 pairs) and
// its rows' prediction in W->uvc[lane], so final_chroma starts from the chosen
// mode's transform instead of recomputing it.
template <int PASS>
__device__ int pick_uv(const Ctx& C)
{
    const ZwSegment& S = *C.S;
    const LdsTables* T = C.T;
    WaveLds* W = C.W;
    const int l = C.lane;
    const int above = C.mby != 0, left = C.mbx != 0;
    int dcU, dcV;
    uv_dc_preds(C, dcU, dcV);
    const int h = l >> 5, q = l & 31, m = q >> 3, b = q & 7;
    const int pl = b >> 2, bx = b & 1, by = (b >> 1) & 1;
    uint32_t s01[2], s32[2], p01[2], p32[2];
    uv_rows_pk(pl ? W->cv : W->cu, (pl ? C.sV : C.sU) + by * 32 + bx * 4, bx, by, h, m, pl ? dcV : dcU, s01, s32, p01,
               p32);
    int cf[2][4];
    fdct_pair(s01, s32, p01, p32, h, cf);
    {
        uint32_t* e = W->uvc[l];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            e[2 * c] = pack_lo(cf[c][0], cf[c][1]);
            e[2 * c + 1] = pack_lo(cf[c][2], cf[c][3]);
        }
        e[4] = p01[0];
        e[5] = p32[0];
        e[6] = p01[1];
        e[7] = p32[1];
    }
    // quantize_coeff (no sharpening, cost.rs:457); natural index n = 4 row + 2h + col
    int dq[2][4], av[2][4];
    int nzac = 0;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool dcs = c == 0 && r == 0;  // natural index 2h: the DC when h == 0
            const int t = dcs ? (int)(h != 0) : 1;
            const uint32_t iq = dcs ? (h ? S.uv.iq[1] : S.uv.iq[0]) : S.uv.iq[1];
            const uint32_t bias = dcs ? (h ? S.uv.bias[1] : S.uv.bias[0]) : S.uv.bias[1];
            const int q_ = dcs ? (int)(h ? S.uv.q[1] : S.uv.q[0]) : (int)S.uv.q[1];
            const int v = cf[c][r];
            const int a = (int)((__umul24((uint32_t)iabs(v), iq) + bias) >> 17);
            av[c][r] = a;
            dq[c][r] = m24(v < 0 ? -a : a, q_);
            nzac += t ? min(a, 1) : 0;
        }
    // get_residual_cost (cost.rs:1670), ctype 2, first 0, ctx0 0
    int last_;
    int cost = rcost_pair<PASS == 2>(av, h, 0, 2, T, last_);
    // reconstruction and SSE of this lane's rows
    uint32_t r01[2], r32[2];
    idct_recon_pair(dq, p01, p32, h, r01, r32);
    int sse = 0;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t d01 = sub_pk(s01[r], r01[r]), d32 = sub_pk(s32[r], r32[r]);
        sse = dot2v(d01, d01, sse);
        sse = dot2v(d32, d32, sse);
    }
    sse = red8(hx_sum(sse));
    cost = red8(cost);
    nzac = red8(hx_sum(nzac));
    const int fixed = sel4(m, d_FIXED_COSTS_UV[0], d_FIXED_COSTS_UV[1], d_FIXED_COSTS_UV[2], d_FIXED_COSTS_UV[3]);
    const int pen = (m > 0 && nzac <= 2) ? 140 * 8 : 0;
    const int csum = fixed + cost + pen;
    // per-mode RD on the scalar unit: rd = (fixed + cost + pen) * lambda_uv + 256 * sse
    long long brd = 0x7fffffffffffffffLL;
    int bm = 0;
#pragma unroll
    for (int mm = 0; mm < 4; mm++) {
        const long long r_m = (long long)__builtin_amdgcn_readlane(csum, mm * 8) * (long long)S.l_uv +
                              256LL * (long long)__builtin_amdgcn_readlane(sse, mm * 8);
        const int avail = mm == 0 || (mm == 1 && above) || (mm == 2 && left) || (mm == 3 && above && left);
        if (avail && r_m < brd) {
            brd = r_m;
            bm = mm;
        }
    }
    return bm;
}

// ---------------------------------------------------------------------------
// I4 search (pick_best_intra4, vp8.rs:1790-2040) in lane-pair form.
// Sub-blocks are visited along x+2y anti-diagonals (10 steps, 6 of them with
// two independent blocks).  One step evaluates ALL ten modes of both blocks at
// once: lane l = 32 hf + 16 slot + mode (modes 10..15 idle), the pair (l,
// l ^ 32) working one (block, mode) in the chroma pair layout (rows 2hf,
// 2hf+1 / columns 2hf, 2hf+1).  The reference's candidate set -- the K modes
// of smallest prediction SSE, in that order (K = 3 / 4 / 10 by method) -- is
// applied afterwards as an eligibility mask: the chosen mode is the eligible
// one of smallest RD score, ties to the smaller (sse, mode) key, which is the
// reference's first strict minimum in candidate order.  The full RD of the
// non-candidates costs nothing extra (the lanes would idle) and the ranking no
// longer sits in front of the transforms.
// ---------------------------------------------------------------------------
// Per-lane constants of the search (fixed for an MB).
struct I4Lane {
    uint32_t ia, ib;  // bperm byte addresses (4 x V index) of the lane's pixels in rows 2hf, 2hf+1, one per byte
    uint32_t psel;    // v_perm selector taking the lane's slot half of two gathered words
    int tm;           // mode is TrueMotion
};

// Value vectors of the step's (up to) two sub-blocks, slot 0 in the low and
// slot 1 in the high 16 bits: lane v < 39 holds V[v] (see i4_values_n).
template <int NB>
__device__ __forceinline__ uint32_t i4_values_pk(const Ctx& C, const int* x0, const int* y0)
{
    const uint8_t* ws = C.M->ws;
    const int l = C.lane;
    const int t = (int)(l >= 13) + (int)(l >= 24) + (int)(l >= 36) + (int)(l >= 37);
    const int k = min(l - 13 * (int)(l >= 13) - 11 * (int)(l >= 24), 12);
    const int t3 = (int)(t == 3), t4 = (int)(t >= 4), t12 = (int)(t == 1 || t == 2);
    const int ka = k + t3 * (11 - k) + t4 * (1 - k);
    const int kb = k + t12 + t3 * (12 - k) - t4 * k;
    const int kc = min(k + 2 * (int)(t == 1), 12);
    const int wb = 2 * (int)(t == 1) + (int)(t == 2) + 3 * (t3 + t4);
    const int wc = (int)(t == 1);
    const int sh = (int)(t != 0) + (int)(t != 0 && t != 2);
    const int oa = csel(ka < 4, -ka * ZW_BPS, ka - 4 - 4 * ZW_BPS);
    const int ob = csel(kb < 4, -kb * ZW_BPS, kb - 4 - 4 * ZW_BPS);
    const int oc = csel(kc < 4, -kc * ZW_BPS, kc - 4 - 4 * ZW_BPS);
    const bool dcl = l < 4 || (l >= 5 && l < 9);
    uint32_t v = 0, ea = 0;
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int hh = NB == 2 ? h : 0;
        const int rowL = (y0[hh] + 3) * ZW_BPS + x0[hh] - 1;
        const int a = ws[rowL + oa], eb = ws[rowL + ob], ec = ws[rowL + oc];
        v |= (uint32_t)((a + wb * eb + wc * ec + ((1 << sh) >> 1)) >> sh) << (16 * h);
        ea |= (uint32_t)a << (16 * h);
    }
    // DC = (4 + L0..L3 + A0..A3) >> 3 of both slots at once (sums < 2^16)
    const uint32_t ds = (uint32_t)__builtin_amdgcn_readfirstlane(red16((int)(dcl ? ea : 0u)));
    const uint32_t dcv = (((ds & 0xffffu) + 4) >> 3) | ((((ds >> 16) + 4) >> 3) << 16);
    return l == 38 ? dcv : v;
}

DI void i4_lane_init(const Ctx& C, I4Lane& L)
{
    const int l = C.lane, hf = l >> 5, m = l & 15, mv = m < 10 ? m : 0;
    L.ia = L.ib = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int sa = i4_src_index(C.T, mv, 8 * hf + j) & 255, sb = i4_src_index(C.T, mv, 8 * hf + 4 + j) & 255;
        L.ia |= (uint32_t)(4 * sa) << (8 * j);
        L.ib |= (uint32_t)(4 * sb) << (8 * j);
    }
    L.psel = (l & 16) ? 0x0c060c02u : 0x0c040c00u;
    L.tm = mv == 1;
}

DI int quad_or(int v)
{
    v |= DPP(v, 0xB1);
    return v | DPP(v, 0x4E);
}
DI int quad_sum(int v)
{
    v += DPP(v, 0xB1);
    return v + DPP(v, 0x4E);
}

// get_residual_cost (cost.rs:1670, quirk A1) of a quad's block, first position
// 0: lane q holds column q, av[r] = |level| at natural index n = 4 r + q.
// Uniform in the quad.  LC = false: pass 1 (zero LevelCosts, quirk A2).
template <bool LC>
DI int rcost_quad(const int av[4], int q, int ctx0, int ctype, const LdsTables* T, int& last_o, int head_none[2])
{
    unsigned nz = 0, big = 0, sc = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int n = 4 * r + q;
        nz |= (unsigned)min(av[r], 1) << n;
        big |= (unsigned)(av[r] >= 2) << n;
        sc |= (unsigned)min(av[r], 2) << (2 * r);
    }
    // every table read of the block issued before any is used (one LDS round
    // trip): the level costs, then the end-of-block cost at last + 1
    int tl[4];
    if (LC) {
        // the context of position n is min(|level[n - 1]|, 2): lane q - 1 of the
        // same row, for q = 0 lane 3 of the row above (ctx0 at n = 0)
        const unsigned pv = (unsigned)DPP((int)sc, 0x93);  // quad_perm [3, 0, 1, 2]
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int n = 4 * r + q;
            const int c_same = (int)((pv >> (2 * r)) & 3u);
            const int c_q0 = r == 0 ? ctx0 : (int)((pv >> (2 * r - 2)) & 3u);
            const int ctx = csel(q == 0, c_q0, c_same);
            const int a = av[r];
            tl[r] = T->lfc[min(a, 2047)] + T->lc[ctype][band_of(n)][ctx][min(a, 67)];
        }
    } else {
#pragma unroll
        for (int r = 0; r < 4; r++) tl[r] = T->lfc[min(av[r], 2047)];
    }
    nz = (unsigned)quad_or((int)nz);
    big = (unsigned)quad_or((int)big);
    const int last = 31 - __clz((int)nz);
    last_o = last;
    const int ctx_t = ((big >> max(last, 0)) & 1u) ? 2 : 1;
    const int tail = (int)T->beob[ctype][band_of(min(last + 1, 15))][ctx_t] & -(int)(last < 15);
    int part = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) part += LC ? tl[r] & -(int)(4 * r + q <= last) : tl[r];
    const int sum = quad_sum(part);
    return csel(last < 0, head_none[1], head_none[0] + sum + tail);  // (no divergent branch)
}

// Candidate evaluation of an I4 step in quad form (K <= 4: methods 0-4).  The
// step's candidate set -- the K modes of smallest prediction SSE per block,
// `rank` from the pair layout -- is evaluated with four lanes per (block,
// candidate): lane = 16 slot + 4 k + q, q = pixel row / coefficient column,
// k = the candidate's rank.  A lane does a quarter of a block's arithmetic
// (the quad transforms of the chroma chain), and only the K candidates are
// transformed instead of all ten modes.  The winner is the smallest (score,
// rank) of each slot's row: the reference's first strict minimum over its
// candidates in SSE order.
template <int PASS, int NB>
DI void i4_cand_quad(const Ctx& C, const int* sbx, const int* sby, const int* x0, const int* y0, const int* tctx,
                     const int* lctx, const int* nzc, int K, int rank, uint32_t vp, uint32_t ap01, uint32_t ap32,
                     I4State& st, bool keep)
{
    PH_START();
    const ZwSegment& S = *C.S;
    const LdsTables* T = C.T;
    const int l = C.lane, m = l & 15, hf = l >> 5;
    // candidate modes: k-th of each slot from the pair layout's ranks (lane
    // 16 slot + mode of the lower half), four bits each, slot 1 at bit 16
    uint32_t modes = 0;
    for (int k = 0; k < K; k++) {
        const unsigned long long b = __ballot(hf == 0 && m < 10 && rank == k);
        const uint32_t lo = (uint32_t)b & 0xffffu, hi = ((uint32_t)b >> 16) & 0xffffu;
        modes |= (uint32_t)__builtin_ctz(lo | 0x10000u) << (4 * k);
        if (NB == 2) modes |= (uint32_t)__builtin_ctz(hi | 0x10000u) << (16 + 4 * k);
    }
    const int slot = NB == 2 ? (l >> 4) & 1 : 0, k = (l >> 2) & 3, q = l & 3;
    const int mq = (int)((modes >> (16 * slot + 4 * k)) & 15u);
    const int mv = k < K ? mq : 0;  // (k >= K: a valid mode, never eligible)
    const int sl = NB == 2 ? 1 : 0;
    const int bx = csel(slot, sbx[sl], sbx[0]), by = csel(slot, sby[sl], sby[0]);
    const int ctx0 = csel(slot, nzc[sl], nzc[0]);
    const int mcost = T->fci4[csel(slot, tctx[sl], tctx[0])][csel(slot, lctx[sl], lctx[0])][mv];
    // read up front, off the transform's chain: the quantiser of this lane's
    // coefficients and the block's costs that depend only on ctx0 (the first
    // coefficient's "more tokens" bit, and the empty block's end of block)
    const uint32_t iq0 = q ? S.y1.iq[1] : S.y1.iq[0], bs0 = q ? S.y1.bias[1] : S.y1.bias[0];
    const uint32_t iq1 = S.y1.iq[1], bs1 = S.y1.bias[1];
    const int q0 = q ? (int)S.y1.q[1] : (int)S.y1.q[0], qa = (int)S.y1.q[1];
    int hn[2];
    hn[0] = (int)T->binit[3][0][ctx0] & -(int)(ctx0 == 0);
    hn[1] = (int)T->beob[3][0][ctx0];
    // prediction of row q: V indices of its four pixels (254: TrueMotion,
    // V[3 - q] + the top offsets; 255: the DC entry V[38])
    uint32_t p01, p32;
    {
        // bpermute byte addresses of the row's four pixels (T->i4qa: 4 x V index)
        const uint32_t iw = *(const uint32_t*)&T->i4qa[mv][4 * q];
        const uint32_t psel = (l & 16) ? 0x0c060c02u : 0x0c040c00u;
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            v[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((iw >> (8 * j)) & 255u), (int)vp);
        const uint32_t q01 = __builtin_amdgcn_perm(v[1], v[0], psel), q32 = __builtin_amdgcn_perm(v[2], v[3], psel);
        const bool tm = mv == 1;
        p01 = tm ? clamp_pk(add_pk(q01, ap01)) : q01;
        p32 = tm ? clamp_pk(add_pk(q32, ap32)) : q32;
    }
    uint32_t s01, s32;
    {
        const uint32_t sw = *(const uint32_t*)(C.sY + (by * 4 + q) * 16 + bx * 4);
        s01 = __builtin_amdgcn_perm(0u, sw, 0x0c010c00u);
        s32 = __builtin_amdgcn_perm(0u, sw, 0x0c020c03u);
    }
    PH_MARK_L(22, l, 0);
    const uint32_t R01 = sub_pk(s01, p01), R32 = sub_pk(s32, p32);
    int cf[4];
    uvq_fdct(add_pk(R01, R32), sub_pk(R01, R32), q, cf);
    int av[4], dq[4], lv[4];
    {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool dcs = r == 0;  // (0, q): the DC for q = 0
            const int v = cf[r];
            const int a = (int)((__umul24((uint32_t)iabs(v), dcs ? iq0 : iq1) + (dcs ? bs0 : bs1)) >> 17);
            av[r] = a;
            lv[r] = v < 0 ? -a : a;
            dq[r] = m24(lv[r], dcs ? q0 : qa);
        }
    }
    int last;
    const int cost = rcost_quad<PASS == 2>(av, q, ctx0, 3, T, last, hn);  // get_cost_luma4 (ctype 3, first 0)
    PH_MARK_L(23, l, 0);
    uint32_t r01, r32;
    uvq_idct_recon(dq, p01, p32, q, r01, r32);
    int sse = 0;
    {
        const uint32_t d01 = sub_pk(s01, r01), d32 = sub_pk(s32, r32);
        sse = dot2v(d01, d01, sse);
        sse = dot2v(d32, d32, sse);
    }
    sse = quad_sum(sse);
    const uint32_t rate = (uint32_t)(mcost + cost);
    // rd_score (cost.rs): sse * 256 + u16(rate) * lambda_i4 < 2^29
    const uint32_t score = (uint32_t)sse * 256u + (rate & 0xffffu) * S.l_i4;
    const uint32_t key2 = k < K ? (score << 2) | (uint32_t)k : 0xffffffffu;
    const uint32_t kmin = min16u(key2);
    const unsigned long long win = __ballot(key2 == kmin);
    PH_MARK_L(12, l, 0);
    int bk[NB];
#pragma unroll
    for (int h = 0; h < NB; h++) {
        bk[h] = __builtin_ctz((uint32_t)(win >> (16 * h)) & 0xffffu) >> 2;
        const int bmode = (int)((modes >> (16 * h + 4 * bk[h])) & 15u);
        const int wl = 16 * h + 4 * bk[h];
        const uint32_t bsse = (uint32_t)__builtin_amdgcn_readlane(sse, wl);
        const uint32_t brate = (uint32_t)__builtin_amdgcn_readlane((int)rate, wl);
        const int bnz = __builtin_amdgcn_readlane((int)(last >= 0), wl);
        const int i = sby[h] * 4 + sbx[h];
        st.tnz = (st.tnz & ~(1u << sbx[h])) | ((uint32_t)bnz << sbx[h]);
        st.lnz = (st.lnz & ~(1u << sby[h])) | ((uint32_t)bnz << sby[h]);
        st.nzm |= (uint32_t)bnz << i;
        // the winner's mode cost is its lane's mcost (= fci4[tctx][lctx][bmode]): no LDS round trip on the step chain
        st.total_mc += (uint32_t)__builtin_amdgcn_readlane(mcost, wl);
        st.running += rdscore(bsse, brate, S.l_mode);
        st.mpack |= (unsigned long long)bmode << (4 * i);
        if (l == h) C.M->modes[i] = (uint8_t)bmode;
    }
    // the winners' quads write their rows of the reconstruction (and, when the
    // final pass reuses them, their columns of levels in zigzag order)
    const int bks = csel(slot, bk[sl], bk[0]);
    if (k == bks && l < 16 * NB) {
        const int xo = csel(slot, x0[sl], x0[0]), yo = csel(slot, y0[sl], y0[0]);
        const uint32_t wd = __builtin_amdgcn_perm(r32, r01, 0x04060200u);
        uint8_t* p = C.M->ws + (yo + q) * ZW_BPS + xo;
#pragma unroll
        for (int j = 0; j < 4; j++) p[j] = (uint8_t)(wd >> (8 * j));
        if (keep) {
            int16_t* lvp = C.M->lev[by * 4 + bx];
#pragma unroll
            for (int r = 0; r < 4; r++) lvp[izz_of(4 * r + q)] = (int16_t)lv[r];
        }
    }
    wsync();
    PH_MARK_L(13, l, 0);
}

template <int PASS, int NB>
__device__ __forceinline__ void i4_step(const Ctx& C, const int* sbx, const int* sby, int K, const I4Lane& LC,
                                        I4State& st, bool keep)
{
    const ZwSegment& S = *C.S;
    const LdsTables* T = C.T;
    const int l = C.lane, hf = l >> 5, m = l & 15;
    const int slot = NB == 2 ? (l >> 4) & 1 : 0;
    int x0[NB], y0[NB], tctx[NB], lctx[NB], nzc[NB];
#pragma unroll
    for (int h = 0; h < NB; h++) {
        const int i = sby[h] * 4 + sbx[h];
        x0[h] = sbx[h] * 4 + 1;
        y0[h] = sby[h] * 4 + 1;
        tctx[h] = sby[h] == 0 ? 0 : (int)((st.mpack >> (4 * (i - 4))) & 15);
        lctx[h] = sbx[h] == 0 ? 0 : (int)((st.mpack >> (4 * (i - 1))) & 15);
        nzc[h] = (sby[h] == 0 ? 0 : (int)((st.tnz >> sbx[h]) & 1)) + (sbx[h] == 0 ? 0 : (int)((st.lnz >> sby[h]) & 1));
    }
    const int sl = NB == 2 ? 1 : 0;
    const int bx = csel(slot, sbx[sl], sbx[0]), by = csel(slot, sby[sl], sby[0]);
    const int ctx0 = csel(slot, nzc[sl], nzc[0]);
    const int mcost = T->fci4[csel(slot, tctx[sl], tctx[0])][csel(slot, lctx[sl], lctx[0])][m < 10 ? m : 0];
    PH_START();
    const uint32_t vp = i4_values_pk<NB>(C, x0, y0);
    PH_MARK_L(10, l, 0);
    // TrueMotion offsets V[5 + j] - V[4] of both slots, as (x0, x1), (x3, x2) pairs
    uint32_t ap01, ap32;
    {
        const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)vp, 4);
        uint32_t a[4];
#pragma unroll
        for (int j = 0; j < 4; j++) a[j] = (uint32_t)__builtin_amdgcn_readlane((int)vp, 5 + j);
        const int sh = 16 * slot;
        const int p_ = (int)((P >> sh) & 255u);
        const int d0 = (int)((a[0] >> sh) & 255u) - p_, d1 = (int)((a[1] >> sh) & 255u) - p_;
        const int d2 = (int)((a[2] >> sh) & 255u) - p_, d3 = (int)((a[3] >> sh) & 255u) - p_;
        ap01 = pack_lo(d0, d1);
        ap32 = pack_lo(d3, d2);
    }
    // this lane's predictions (rows 2hf, 2hf+1) gathered from the value vectors
    uint32_t p01[2], p32[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t ix = r ? LC.ib : LC.ia;
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ix & 255u), (int)vp);
        const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ix >> 8) & 255u), (int)vp);
        const uint32_t v2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ix >> 16) & 255u), (int)vp);
        const uint32_t v3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ix >> 24), (int)vp);
        const uint32_t q01 = __builtin_amdgcn_perm(v1, v0, LC.psel), q32 = __builtin_amdgcn_perm(v2, v3, LC.psel);
        p01[r] = LC.tm ? clamp_pk(add_pk(q01, ap01)) : q01;
        p32[r] = LC.tm ? clamp_pk(add_pk(q32, ap32)) : q32;
    }
    // source rows
    uint32_t s01[2], s32[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t sw = *(const uint32_t*)(C.sY + (by * 4 + 2 * hf + r) * 16 + bx * 4);
        s01[r] = __builtin_amdgcn_perm(0u, sw, 0x0c010c00u);
        s32[r] = __builtin_amdgcn_perm(0u, sw, 0x0c020c03u);
    }
    // prediction SSE and the candidate set: rank of key = sse * 16 + mode among
    // the slot's ten modes (the reference's stable ascending sort, quirk A12)
    int pse = 0;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t d01 = sub_pk(s01[r], p01[r]), d32 = sub_pk(s32[r], p32[r]);
        pse = dot2v(d01, d01, pse);
        pse = dot2v(d32, d32, pse);
    }
    pse = hx_sum(pse);
    const int key = m < 10 ? (pse << 4) | m : 0x7fffffff;
    // rank = #{lanes of the 16-lane row with a smaller key}: per rotation the
    // borrow of a DPP subtraction (keys are in [0, 2^31), so the borrow is
    // rot(key) < key) into VCC, then an add-with-carry
    int rank = 0, scratch_;
#define ZW_RANK_STEP(R) "v_sub_co_u32_dpp %1, vcc, %2, %2 row_ror:" #R " row_mask:0xf bank_mask:0xf\n" \
                        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
    asm volatile("s_nop 1\n" ZW_RANK_STEP(1) ZW_RANK_STEP(2) ZW_RANK_STEP(3) ZW_RANK_STEP(4) ZW_RANK_STEP(5)
                     ZW_RANK_STEP(6) ZW_RANK_STEP(7) ZW_RANK_STEP(8) ZW_RANK_STEP(9) ZW_RANK_STEP(10)
                         ZW_RANK_STEP(11) ZW_RANK_STEP(12) ZW_RANK_STEP(13) ZW_RANK_STEP(14) ZW_RANK_STEP(15)
                 : "+v"(rank), "=&v"(scratch_)
                 : "v"(key)
                 : "vcc");
#undef ZW_RANK_STEP
    PH_MARK_L(11, l, 0);
#ifndef ZW_I4_QUAD
#define ZW_I4_QUAD 1
#endif
    if (ZW_I4_QUAD && K <= 4) {
        i4_cand_quad<PASS, NB>(C, sbx, sby, x0, y0, tctx, lctx, nzc, K, rank, vp, ap01, ap32, st, keep);
        return;
    }
    // transform, quantiser, rate, reconstruction and distortion of every
    // (block, mode): natural coefficient index n = 4 row + 2 hf + col, the DC
    // (n = 0) in the lower half's column 0
    int cf[2][4];
    fdct_pair(s01, s32, p01, p32, hf, cf);
    int av[2][4], dq[2][4];
    unsigned sgn = 0;
    {
        const uint32_t iq0 = hf ? S.y1.iq[1] : S.y1.iq[0], bs0 = hf ? S.y1.bias[1] : S.y1.bias[0];
        const int q0 = hf ? (int)S.y1.q[1] : (int)S.y1.q[0];
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const bool dcs = c == 0 && r == 0;
                const int v = cf[c][r];
                const int a = (int)((__umul24((uint32_t)iabs(v), dcs ? iq0 : S.y1.iq[1]) + (dcs ? bs0 : S.y1.bias[1])) >> 17);
                av[c][r] = a;
                dq[c][r] = m24(v < 0 ? -a : a, dcs ? q0 : (int)S.y1.q[1]);
                sgn |= (unsigned)(v < 0) << (4 * c + r);
            }
    }
    int last;
    const int cost = rcost_pair<PASS == 2>(av, hf, ctx0, 3, T, last);  // get_cost_luma4 (ctype 3, first 0)
    uint32_t r01[2], r32[2];
    idct_recon_pair(dq, p01, p32, hf, r01, r32);
    int sse = 0;
#pragma unroll
    for (int r = 0; r < 2; r++) {
        const uint32_t d01 = sub_pk(s01[r], r01[r]), d32 = sub_pk(s32[r], r32[r]);
        sse = dot2v(d01, d01, sse);
        sse = dot2v(d32, d32, sse);
    }
    sse = hx_sum(sse);
    const uint32_t rate = (uint32_t)(mcost + cost);
    // rd_score (cost.rs): sse * 256 + u16(rate) * lambda_i4 < 2^29 (see above)
    const uint32_t score = (uint32_t)sse * 256u + (rate & 0xffffu) * S.l_i4;
    const bool elig = m < 10 && rank < K;
    // the eligible lane of smallest (score, rank) in each slot's row: the
    // reference's first strict minimum over its candidates in SSE order
    unsigned long long win;
    if (K <= 4) {
        const uint32_t key2 = elig ? (score << 2) | (uint32_t)rank : 0xffffffffu;
        const uint32_t kmin = min16u(key2);
        win = __ballot(key2 == kmin);
    } else {
        // (DPP reads other lanes: every min16u runs with the whole wave active)
        const uint32_t sk = elig ? score : 0xffffffffu;
        const uint32_t smin = min16u(sk);
        const uint32_t rk = sk == smin ? (uint32_t)rank : 0xffffffffu;
        const uint32_t rmin = min16u(rk);
        win = __ballot(rk == rmin && sk == smin);
    }
    PH_MARK_L(12, l, 0);
    int bmode[NB];
#pragma unroll
    for (int h = 0; h < NB; h++) {
        bmode[h] = __builtin_ctz((uint32_t)(win >> (16 * h)) & 0xffffu);
        const int wl = 16 * h + bmode[h];
        const uint32_t bsse = (uint32_t)__builtin_amdgcn_readlane(sse, wl);
        const uint32_t brate = (uint32_t)__builtin_amdgcn_readlane((int)rate, wl);
        const int bnz = __builtin_amdgcn_readlane((int)(last >= 0), wl);
        const int i = sby[h] * 4 + sbx[h];
        st.tnz = (st.tnz & ~(1u << sbx[h])) | ((uint32_t)bnz << sbx[h]);
        st.lnz = (st.lnz & ~(1u << sby[h])) | ((uint32_t)bnz << sby[h]);
        st.nzm |= (uint32_t)bnz << i;
        st.total_mc += (uint32_t)__builtin_amdgcn_readlane(mcost, wl);  // (lane wl's mode is bmode[h])
        st.running += rdscore(bsse, brate, S.l_mode);
        st.mpack |= (unsigned long long)bmode[h] << (4 * i);
        if (l == h) C.M->modes[i] = (uint8_t)bmode[h];
    }
    // the winners' two lanes write their rows of the reconstruction (and, when
    // the final pass reuses them, the levels in zigzag order)
    const int bms = csel(slot, bmode[sl], bmode[0]);
    if (m == bms && (NB == 2 || slot == 0)) {
        const int xo = csel(slot, x0[sl], x0[0]), yo = csel(slot, y0[sl], y0[0]);
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t wd = __builtin_amdgcn_perm(r32[r], r01[r], 0x04060200u);
            uint8_t* p = C.M->ws + (yo + 2 * hf + r) * ZW_BPS + xo;
#pragma unroll
            for (int j = 0; j < 4; j++) p[j] = (uint8_t)(wd >> (8 * j));
        }
        if (keep) {
            int16_t* lv = C.M->lev[by * 4 + bx];
#pragma unroll
            for (int c = 0; c < 2; c++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int a = av[c][r];
                    lv[izz_of(4 * r + 2 * hf + c)] = (int16_t)(((sgn >> (4 * c + r)) & 1u) ? -a : a);
                }
        }
    }
    wsync();
    PH_MARK_L(13, l, 0);
}

// pick_best_intra4 (vp8.rs:1790-2040).  Returns true when I4 wins; modes in C.M->modes.
// Each block's choice depends only on its left / top / top-right neighbours,
// which every earlier anti-diagonal holds, so every choice equals the
// raster-order one.  The reference's early exits (running score >= the I16
// score, vp8.rs:2018; mode cost cap, :1839) test sums of non-negative terms,
// which grow with every block: "some raster prefix crossed the bound" is "the
// sum over every block crossed it", so testing the sum of the blocks searched
// so far after each step decides exactly as the reference does.
template <int PASS>
__device__ bool pick_i4(const Ctx& C, unsigned long long i16_score, bool keep, uint32_t& nzm)
{
    const ZwSegment& S = *C.S;
    const int K = C.method <= 3 ? 3 : (C.method == 4 ? 4 : 10);
    I4State st;
    st.running = 211ull * S.l_mode;
    st.total_mc = 0;
    st.mpack = 0;
    st.tnz = st.lnz = st.nzm = 0;
    I4Lane LC;
    i4_lane_init(C, LC);
    PH_COUNT(20);
    for (int s = 0; s < 10; s++) {
        PH_COUNT(19);
        // anti-diagonal s: A = (sbx, sby) with the smallest sby, B = (sbx - 2, sby + 1)
        const int sbyA = s < 4 ? 0 : (s - 2) >> 1;
        const int sbxA = s - 2 * sbyA;
        if (s >= 2 && s <= 7) {
            const int bx[2] = {sbxA, sbxA - 2}, by[2] = {sbyA, sbyA + 1};
            i4_step<PASS, 2>(C, bx, by, K, LC, st, keep);
        } else {
            i4_step<PASS, 1>(C, &sbxA, &sbyA, K, LC, st, keep);
        }
        if (st.running >= i16_score) return false;
        if (st.total_mc > 256u * 16u * 16u / 4u) return false;
    }
    nzm = st.nzm;
    return true;
}

// ---------------------------------------------------------------------------
// Paired I4 search: one wave searches the MBs of two rows at once.  The paired
// kernels give a wave two MB rows, y and y + 1, the second two columns behind
// (the x + 2y wavefront's lag), so MB A = (x, y) and MB B = (x - 2, y + 1) reach
// their I4 searches together; both visit the same anti-diagonal steps.  Lanes
// 0..31 work A and lanes 32..63 work B (hm = lane >> 5): the candidate phase
// keeps the quad form (lane = 32 hm + 16 slot + 4 k + q), the ranking works
// all four rows of a (slot, mode) in one lane (lane = 32 hm + 16 slot + mode).
// The value vectors of the four (MB, slot) blocks are packed one byte each
// (byte 2 hm + slot) in lanes 0..38.  Every per-MB decision (winners, early
// exits, running scores) is the single search's, per MB: a search that ends
// early leaves its lanes computing on, with their stores masked.
// ---------------------------------------------------------------------------
struct I4PLane {
    uint32_t ix[4];  // bperm byte addresses (4 x V index) of the lane's pixels in rows 0..3, one per byte
    uint32_t psel;   // v_perm selector taking the lane's (MB, slot) byte of two gathered words
    int tm;          // mode is TrueMotion
    // the candidate step's quantiser of the lane's coefficient column q (its MB's
    // segment, fixed for the search): read once instead of every step
    uint32_t iq0, bs0, iq1, bs1;
    int q0, qa;
    uint32_t l_i4;
};

DI uint32_t i4p_psel(int hm, int slot)
{
    const uint32_t b = (uint32_t)(2 * hm + slot);
    return 0x0c000c00u | ((4u + b) << 16) | b;
}

DI void i4p_lane_init(const Ctx& C, const Ctx& CB, I4PLane& L)
{
    const int l = C.lane, m = l & 15, mv = m < 10 ? m : 0;
    {
        const ZwSegment* Sh = (l >> 5) ? CB.S : C.S;
        const int q = l & 3;
        L.iq0 = q ? Sh->y1.iq[1] : Sh->y1.iq[0];
        L.bs0 = q ? Sh->y1.bias[1] : Sh->y1.bias[0];
        L.iq1 = Sh->y1.iq[1];
        L.bs1 = Sh->y1.bias[1];
        L.q0 = q ? (int)Sh->y1.q[1] : (int)Sh->y1.q[0];
        L.qa = (int)Sh->y1.q[1];
        L.l_i4 = Sh->l_i4;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) w |= (uint32_t)(4 * (i4_src_index(C.T, mv, 4 * r + j) & 255)) << (8 * j);
        L.ix[r] = w;
    }
    L.psel = i4p_psel(l >> 5, (l >> 4) & 1);
    L.tm = mv == 1;
}

// Value vectors (see i4_values_pk) of both MBs' step blocks: lane v < 39 holds
// V[v] of (A slot 0, A slot 1, B slot 0, B slot 1) in bytes 0..3.
template <int NB>
DI uint32_t i4p_values(const Ctx& CA, const Ctx& CB, const int* x0, const int* y0)
{
    const int l = CA.lane;
    const int t = (int)(l >= 13) + (int)(l >= 24) + (int)(l >= 36) + (int)(l >= 37);
    const int k = min(l - 13 * (int)(l >= 13) - 11 * (int)(l >= 24), 12);
    const int t3 = (int)(t == 3), t4 = (int)(t >= 4), t12 = (int)(t == 1 || t == 2);
    const int ka = k + t3 * (11 - k) + t4 * (1 - k);
    const int kb = k + t12 + t3 * (12 - k) - t4 * k;
    const int kc = min(k + 2 * (int)(t == 1), 12);
    const int wb = 2 * (int)(t == 1) + (int)(t == 2) + 3 * (t3 + t4);
    const int wc = (int)(t == 1);
    const int sh = (int)(t != 0) + (int)(t != 0 && t != 2);
    const int oa = csel(ka < 4, -ka * ZW_BPS, ka - 4 - 4 * ZW_BPS);
    const int ob = csel(kb < 4, -kb * ZW_BPS, kb - 4 - 4 * ZW_BPS);
    const int oc = csel(kc < 4, -kc * ZW_BPS, kc - 4 - 4 * ZW_BPS);
    const bool dcl = l < 4 || (l >= 5 && l < 9);
    uint32_t v[2], ea[2];
#pragma unroll
    for (int mb = 0; mb < 2; mb++) {
        const uint8_t* ws = (mb ? CB : CA).M->ws;
        v[mb] = ea[mb] = 0;
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int hh = NB == 2 ? h : 0;
            const int rowL = (y0[hh] + 3) * ZW_BPS + x0[hh] - 1;
            const int a = ws[rowL + oa], eb = ws[rowL + ob], ec = ws[rowL + oc];
            v[mb] |= (uint32_t)((a + wb * eb + wc * ec + ((1 << sh) >> 1)) >> sh) << (16 * h);
            ea[mb] |= (uint32_t)a << (16 * h);
        }
    }
    // the DCs of the four blocks (sums < 2^16 per slot)
    const uint32_t da = (uint32_t)__builtin_amdgcn_readfirstlane(red16((int)(dcl ? ea[0] : 0u)));
    const uint32_t db = (uint32_t)__builtin_amdgcn_readfirstlane(red16((int)(dcl ? ea[1] : 0u)));
    const uint32_t dcv = (((da & 0xffffu) + 4) >> 3) | ((((da >> 16) + 4) >> 3) << 8) |
                         ((((db & 0xffffu) + 4) >> 3) << 16) | ((((db >> 16) + 4) >> 3) << 24);
    return l == 38 ? dcv : __builtin_amdgcn_perm(v[1], v[0], 0x06040200u);
}

template <int PASS, int NB>
DI void i4p_step(const Ctx& CA, const Ctx& CB, const int* sbx, const int* sby, int K, const I4PLane& LC,
                 I4State st[2], const bool act[2], bool keep)
{
    [[maybe_unused]] const Ctx& C = CA;  // (the phase counters)
    const int l = CA.lane, m = l & 15, hm = l >> 5;
    const int slot = NB == 2 ? (l >> 4) & 1 : 0;
    const int sl = NB == 2 ? 1 : 0;
    // per (MB, slot) contexts, wave-uniform, then the lane's
    int x0[NB], y0[NB], tc[2][NB], lc[2][NB], nc[2][NB];
#pragma unroll
    for (int h = 0; h < NB; h++) {
        const int i = sby[h] * 4 + sbx[h];
        x0[h] = sbx[h] * 4 + 1;
        y0[h] = sby[h] * 4 + 1;
#pragma unroll
        for (int mb = 0; mb < 2; mb++) {
            tc[mb][h] = sby[h] == 0 ? 0 : (int)((st[mb].mpack >> (4 * (i - 4))) & 15);
            lc[mb][h] = sbx[h] == 0 ? 0 : (int)((st[mb].mpack >> (4 * (i - 1))) & 15);
            nc[mb][h] = (sby[h] == 0 ? 0 : (int)((st[mb].tnz >> sbx[h]) & 1)) +
                        (sbx[h] == 0 ? 0 : (int)((st[mb].lnz >> sby[h]) & 1));
        }
    }
    auto pick = [&](const int (&v)[2][NB]) {
        const int a = csel(slot, v[0][sl], v[0][0]), b = csel(slot, v[1][sl], v[1][0]);
        return csel(hm, b, a);
    };
    const int tctx = pick(tc), lctx = pick(lc), ctx0 = pick(nc);
    const int bx = csel(slot, sbx[sl], sbx[0]), by = csel(slot, sby[sl], sby[0]);
    const uint8_t* sYh = hm ? CB.sY : CA.sY;
    const LdsTables* Th = hm ? CB.T : CA.T;  // the lane's frame's tables (costs, probabilities)
    PH_START();
    const uint32_t vp = i4p_values<NB>(CA, CB, x0, y0);
    // TrueMotion offsets V[5 + j] - V[4] of the lane's (MB, slot), as (x0, x1), (x3, x2) pairs
    uint32_t ap01, ap32;
    {
        const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)vp, 4);
        uint32_t a[4];
#pragma unroll
        for (int j = 0; j < 4; j++) a[j] = (uint32_t)__builtin_amdgcn_readlane((int)vp, 5 + j);
        const int sh = 8 * (2 * hm + slot);
        const int p_ = (int)((P >> sh) & 255u);
        const int d0 = (int)((a[0] >> sh) & 255u) - p_, d1 = (int)((a[1] >> sh) & 255u) - p_;
        const int d2 = (int)((a[2] >> sh) & 255u) - p_, d3 = (int)((a[3] >> sh) & 255u) - p_;
        ap01 = pack_lo(d0, d1);
        ap32 = pack_lo(d3, d2);
    }
    PH_MARK_L(10, l, 0);
    // ranking: the four rows of (MB, slot, mode) in one lane
    int pse = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t ix = LC.ix[r];
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ix & 255u), (int)vp);
        const uint32_t v1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ix >> 8) & 255u), (int)vp);
        const uint32_t v2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ix >> 16) & 255u), (int)vp);
        const uint32_t v3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ix >> 24), (int)vp);
        const uint32_t q01 = __builtin_amdgcn_perm(v1, v0, LC.psel), q32 = __builtin_amdgcn_perm(v2, v3, LC.psel);
        const uint32_t p01 = LC.tm ? clamp_pk(add_pk(q01, ap01)) : q01;
        const uint32_t p32 = LC.tm ? clamp_pk(add_pk(q32, ap32)) : q32;
        const uint32_t sw = *(const uint32_t*)(sYh + (by * 4 + r) * 16 + bx * 4);
        const uint32_t d01 = sub_pk(__builtin_amdgcn_perm(0u, sw, 0x0c010c00u), p01);
        const uint32_t d32 = sub_pk(__builtin_amdgcn_perm(0u, sw, 0x0c020c03u), p32);
        pse = dot2v(d01, d01, pse);
        pse = dot2v(d32, d32, pse);
    }
    const int key = m < 10 ? (pse << 4) | m : 0x7fffffff;
    int rank = 0, scratch_;
#define ZW_RANK_STEP(R) "v_sub_co_u32_dpp %1, vcc, %2, %2 row_ror:" #R " row_mask:0xf bank_mask:0xf\n" \
                        "v_addc_co_u32_e32 %0, vcc, 0, %0, vcc\n"
    asm volatile("s_nop 1\n" ZW_RANK_STEP(1) ZW_RANK_STEP(2) ZW_RANK_STEP(3) ZW_RANK_STEP(4) ZW_RANK_STEP(5)
                     ZW_RANK_STEP(6) ZW_RANK_STEP(7) ZW_RANK_STEP(8) ZW_RANK_STEP(9) ZW_RANK_STEP(10)
                         ZW_RANK_STEP(11) ZW_RANK_STEP(12) ZW_RANK_STEP(13) ZW_RANK_STEP(14) ZW_RANK_STEP(15)
                 : "+v"(rank), "=&v"(scratch_)
                 : "v"(key)
                 : "vcc");
#undef ZW_RANK_STEP
    PH_MARK_L(11, l, 0);
    // candidate modes: k-th of each (MB, slot) group, four bits each, group g at bit 16 g
    unsigned long long modes = 0;
    for (int k = 0; k < K; k++) {
        const unsigned long long b = __ballot(m < 10 && rank == k);
#pragma unroll
        for (int g = 0; g < 4; g++)
            modes |= (unsigned long long)__builtin_ctz((uint32_t)(b >> (16 * g)) | 0x10000u) << (16 * g + 4 * k);
    }
    const int k = (l >> 2) & 3, q = l & 3;
    const int g = 2 * hm + slot;
    const int mq = (int)((modes >> (16 * g + 4 * k)) & 15ull);
    const int mv = k < K ? mq : 0;  // (k >= K: a valid mode, never eligible)
    const int mcost = Th->fci4[tctx][lctx][mv];
    const uint32_t iq0 = LC.iq0, bs0 = LC.bs0, iq1 = LC.iq1, bs1 = LC.bs1;
    const int q0 = LC.q0, qa = LC.qa;
    int hn[2];
    hn[0] = (int)Th->binit[3][0][ctx0] & -(int)(ctx0 == 0);
    hn[1] = (int)Th->beob[3][0][ctx0];
    uint32_t p01, p32;
    {
        const uint32_t iw = *(const uint32_t*)&Th->i4qa[mv][4 * q];
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++)
            v[j] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((iw >> (8 * j)) & 255u), (int)vp);
        const uint32_t q01 = __builtin_amdgcn_perm(v[1], v[0], LC.psel), q32 = __builtin_amdgcn_perm(v[2], v[3], LC.psel);
        const bool tm = mv == 1;
        p01 = tm ? clamp_pk(add_pk(q01, ap01)) : q01;
        p32 = tm ? clamp_pk(add_pk(q32, ap32)) : q32;
    }
    uint32_t s01, s32;
    {
        const uint32_t sw = *(const uint32_t*)(sYh + (by * 4 + q) * 16 + bx * 4);
        s01 = __builtin_amdgcn_perm(0u, sw, 0x0c010c00u);
        s32 = __builtin_amdgcn_perm(0u, sw, 0x0c020c03u);
    }
    PH_MARK_L(22, l, 0);
    const uint32_t R01 = sub_pk(s01, p01), R32 = sub_pk(s32, p32);
    int cf[4];
    uvq_fdct(add_pk(R01, R32), sub_pk(R01, R32), q, cf);
    int av[4], dq[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool dcs = r == 0;  // (0, q): the DC for q = 0
        const int v = cf[r];
        const int a = (int)((__umul24((uint32_t)iabs(v), dcs ? iq0 : iq1) + (dcs ? bs0 : bs1)) >> 17);
        av[r] = a;
        lv[r] = v < 0 ? -a : a;
        dq[r] = m24(lv[r], dcs ? q0 : qa);
    }
    int last;
    const int cost = rcost_quad<PASS == 2>(av, q, ctx0, 3, Th, last, hn);
    PH_MARK_L(23, l, 0);
    uint32_t r01, r32;
    uvq_idct_recon(dq, p01, p32, q, r01, r32);
    int sse = 0;
    {
        const uint32_t d01 = sub_pk(s01, r01), d32 = sub_pk(s32, r32);
        sse = dot2v(d01, d01, sse);
        sse = dot2v(d32, d32, sse);
    }
    sse = quad_sum(sse);
    const uint32_t rate = (uint32_t)(mcost + cost);
    const uint32_t score = (uint32_t)sse * 256u + (rate & 0xffffu) * LC.l_i4;
    const uint32_t key2 = k < K ? (score << 2) | (uint32_t)k : 0xffffffffu;
    const uint32_t kmin = min16u(key2);
    const unsigned long long win = __ballot(key2 == kmin);
    // the winner's u16 rate, mode cost (< 2^15) and nonzero flag in one word: one
    // readlane for them instead of three
    const uint32_t pk = (rate & 0xffffu) | ((uint32_t)mcost << 16) | ((uint32_t)(last >= 0) << 31);
    PH_MARK_L(12, l, 0);
#pragma unroll
    for (int mb = 0; mb < 2; mb++) {
        const ZwSegment& S = *(mb ? CB : CA).S;
        MbLds* M = (mb ? CB : CA).M;
#pragma unroll
        for (int h = 0; h < NB; h++) {
            const int gg = 2 * mb + h;
            const int bk = __builtin_ctz((uint32_t)(win >> (16 * gg)) & 0xffffu) >> 2;
            const int bmode = (int)((modes >> (16 * gg + 4 * bk)) & 15ull);
            const int wl = 16 * gg + 4 * bk;
            const uint32_t bsse = (uint32_t)__builtin_amdgcn_readlane(sse, wl);
            const uint32_t bpk = (uint32_t)__builtin_amdgcn_readlane((int)pk, wl);
            const uint32_t brate = bpk & 0xffffu;
            const int bnz = (int)(bpk >> 31);
            const int i = sby[h] * 4 + sbx[h];
            I4State& s = st[mb];
            s.tnz = (s.tnz & ~(1u << sbx[h])) | ((uint32_t)bnz << sbx[h]);
            s.lnz = (s.lnz & ~(1u << sby[h])) | ((uint32_t)bnz << sby[h]);
            s.nzm |= (uint32_t)bnz << i;
            s.total_mc += (bpk >> 16) & 0x7fffu;
            s.running += rdscore(bsse, brate, S.l_mode);
            s.mpack |= (unsigned long long)bmode << (4 * i);
            if (act[mb] && l == gg) M->modes[i] = (uint8_t)bmode;
        }
    }
    // the winners' quads write their rows of the reconstruction (and levels)
    const int bks = __builtin_ctz((uint32_t)(win >> (16 * g)) & 0xffffu) >> 2;
    if (k == bks && ((l >> 4) & 1) < NB && (hm ? act[1] : act[0])) {
        MbLds* M = hm ? CB.M : CA.M;
        const int xo = csel(slot, x0[sl], x0[0]), yo = csel(slot, y0[sl], y0[0]);
        const uint32_t wd = __builtin_amdgcn_perm(r32, r01, 0x04060200u);
        uint8_t* p = M->ws + (yo + q) * ZW_BPS + xo;
#pragma unroll
        for (int j = 0; j < 4; j++) p[j] = (uint8_t)(wd >> (8 * j));
        if (keep) {
            int16_t* lvp = M->lev[by * 4 + bx];
#pragma unroll
            for (int r = 0; r < 4; r++) lvp[izz_of(4 * r + q)] = (int16_t)lv[r];
        }
    }
    wsync();
    PH_MARK_L(13, l, 0);
}

// pick_best_intra4 (vp8.rs:1790-2040) of two MBs at once (K <= 4): bit mb of
// the result is set when I4 wins MB mb (A, B); each MB's early exits are the
// single search's (pick_i4).  An MB with act* false is not searched (its
// lanes compute on its work buffer with every store masked).
template <int PASS>
__device__ uint32_t pick_i4_pair(const Ctx& CA, const Ctx& CB, unsigned long long i16A, unsigned long long i16B,
                                 bool actA, bool actB, bool keep, uint32_t& nzA, uint32_t& nzB)
{
    const int K = CA.method <= 3 ? 3 : 4;
    I4State st[2];
    st[0].running = 211ull * CA.S->l_mode;
    st[1].running = 211ull * CB.S->l_mode;
#pragma unroll
    for (int mb = 0; mb < 2; mb++) {
        st[mb].total_mc = 0;
        st[mb].mpack = 0;
        st[mb].tnz = st[mb].lnz = st[mb].nzm = 0;
    }
    bool act[2] = {actA, actB};  // (an MB without a search: its lanes run masked)
    const unsigned long long lim[2] = {i16A, i16B};
    I4PLane LC;
    i4p_lane_init(CA, CB, LC);
    for (int s = 0; s < 10; s++) {
        const int sbyA = s < 4 ? 0 : (s - 2) >> 1;
        const int sbxA = s - 2 * sbyA;
        if (s >= 2 && s <= 7) {
            const int bx[2] = {sbxA, sbxA - 2}, by[2] = {sbyA, sbyA + 1};
            i4p_step<PASS, 2>(CA, CB, bx, by, K, LC, st, act, keep);
        } else {
            i4p_step<PASS, 1>(CA, CB, &sbxA, &sbyA, K, LC, st, act, keep);
        }
#pragma unroll
        for (int mb = 0; mb < 2; mb++)
            if (st[mb].running >= lim[mb] || st[mb].total_mc > 256u * 16u * 16u / 4u) act[mb] = false;
        if (!act[0] && !act[1]) return 0;
    }
    nzA = st[0].nzm;
    nzB = st[1].nzm;
    return (uint32_t)act[0] | ((uint32_t)act[1] << 1);
}

// Final luma transform (transform_luma_block vp8.rs:2647 / _4x4 :2785).
// Writes zigzag levels to C.M->lev[0..16], recon into C.M->ws.  Returns the
// simple-quant "any nonzero" flag for skip detection (check_all_coeffs_zero).
__device__ int final_luma(const Ctx& C, int mode, bool trel, int y_nz_out[16], int i4_nzm)
{
    WaveLds* W = C.W;
    const ZwSegment& S = *C.S;
    const int l = C.lane;
    int anynz = 0;
    PH_START();
    if (mode == 4 && i4_nzm >= 0) {
        // simple quantisation: the search's winners are the final blocks (same
        // prediction, transform and quantize_coeff); their levels are in
        // C.M->lev, their reconstruction in C.M->ws
#pragma unroll
        for (int i = 0; i < 16; i++) y_nz_out[i] = (i4_nzm >> i) & 1;
        if (l < 16) C.M->lev[16][l] = 0;
        wsync();
        PH_MARK_L(15, l, 0);
        PH_COUNT(7);
        return i4_nzm != 0;
    }
    if (mode != 4) {
        build_luma_border(C);
        const uint8_t* ws = C.M->ws;
        const int above = C.mby != 0, left = C.mbx != 0;
        const int b = l & 15, bx = b & 3, by = b >> 2;
        int dcv;
        {  // DC predictor: lanes 0..15 top row, 16..31 left column
            const int top = l < 16;
            const int v = (int)ws[csel(top, 1 + b, (b + 1) * ZW_BPS)] & -(int)(l < 32 && (top ? above : left));
            const int sum = red16(v);
            const int su = __builtin_amdgcn_readlane(sum, 0) + __builtin_amdgcn_readlane(sum, 16);
            const int shf = 3 + above + left;
            dcv = (!above && !left) ? 128 : ((su + (1 << (shf - 1))) >> shf);
        }
        int c[16], pr[16];
        {
            // every 16-lane group computes its block's coefficients (lanes 16..47
            // feed the ctx-parallel trellis)
            const int P0 = ws[0];
            int L[4], Tp[4], r[16];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                L[i] = ws[(by * 4 + i + 1) * ZW_BPS];
                Tp[i] = ws[1 + bx * 4 + i];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t srow = *(const uint32_t*)(C.sY + (by * 4 + i) * 16 + bx * 4);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int p = sel4(mode, dcv, Tp[j], L[i], clamp255(L[i] + Tp[j] - P0));
                    pr[i * 4 + j] = p;
                    r[i * 4 + j] = (int)((srow >> (8 * j)) & 255u) - p;
                }
            }
            fdct16_pk(r, c);
        }
        // Y2 (the 16 DCs) in group form: lane b holds block b's DC
        int y2dq;
        {
            const int d = wht_g(c[0], b);
            const int t = b > 0;
            const int y2q = quantz(d, S.y2.iq[t], S.y2.bias[t]);
            if (l < 16) C.M->lev[16][izz_of(b)] = (int16_t)y2q;
            if (gmask(y2q != 0)) anynz = 1;
            y2dq = iwht_g(m24(y2q, (int)S.y2.q[t]), b);
        }
        PH_MARK_L(16, l, 0);
        int dq[16], lv[16];
        int nzb = 0;
        {
            // simple-quant check on the AC coefficients (check_all_coeffs_zero)
            int snz = 0;
            if (l < 16) {
#pragma unroll
                for (int k = 1; k < 16; k++) snz |= quantz(c[k], S.y1.iq[1], S.y1.bias[1]) != 0;
            }
            anynz |= __any(snz) ? 1 : 0;
        }
        if (trel) {
            // Trellis for every block under all three contexts at once (lane =
            // ctx0*16 + block), then resolve the raster-order nz context chain
            // (left / top neighbours) on the scalar unit and pick each block's result.
            int tnz = 0;
            if (l < 48) {
#pragma unroll
                for (int k = 0; k < 16; k++) dq[k] = c[k];
                tnz = trellis<1, true>(dq, lv, S.y1, S.sharpen, S.lt_i16, C.T, 0, l >> 4);
            }
            PH_MARK_L(17, l, 0);
            const unsigned long long nzm = __ballot(l < 48 && tnz);
            int nt[4], nl[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                nt[q] = __builtin_amdgcn_readfirstlane(C.top_c[C.ocx + 1 + q]);
                nl[q] = __builtin_amdgcn_readfirstlane(C.M->left_c[1 + q]);
            }
            unsigned code = 0, nzbits = 0;
#pragma unroll
            for (int bb = 0; bb < 16; bb++) {
                const int cx = min(nl[bb >> 2] + nt[bb & 3], 2);
                const int z = (int)((nzm >> (cx * 16 + bb)) & 1ull);
                nt[bb & 3] = z;
                nl[bb >> 2] = z;
                code |= (unsigned)cx << (2 * bb);
                nzbits |= (unsigned)z << bb;
            }
            const int srcl = (int)((code >> (2 * b)) & 3u) * 16 + b;
            // gather the chosen context's levels as i16 pairs (|level| <= 2047)
            // and dequantise them again (the trellis leaves level * q at the AC
            // positions; the DC position is replaced by the Y2 output below)
            lv[0] = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t w = (uint32_t)__shfl((int)pack_lo(lv[2 * i], lv[2 * i + 1]), srcl);
                lv[2 * i] = lo16(w);
                lv[2 * i + 1] = hi16(w);
            }
#pragma unroll
            for (int n = 1; n < 16; n++) dq[kZZ(n)] = m24(lv[n], (int)S.y1.q[1]);
            nzb = (nzbits >> b) & 1u;
            PH_MARK_L(18, l, 0);
        } else if (l < 16) {
#pragma unroll
            for (int n = 1; n < 16; n++) {
                const int j = kZZ(n);
                lv[n] = quantz(c[j], S.y1.iq[1], S.y1.bias[1]);
                nzb |= lv[n] != 0;
            }
            dq[0] = 0;
#pragma unroll
            for (int n = 1; n < 16; n++) dq[kZZ(n)] = m24(lv[n], (int)S.y1.q[1]);
        }
        wsync();
        if (l < 16) {
            lv[0] = 0;
#pragma unroll
            for (int n = 0; n < 16; n++) C.M->lev[b][n] = (int16_t)lv[n];
            dq[0] = y2dq;
            idct16(dq);
            uint8_t* wsp = C.M->ws;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int y = by * 4 + (k >> 2), x = bx * 4 + (k & 3);
                wsp[(y + 1) * ZW_BPS + 1 + x] = (uint8_t)clamp255(pr[k] + dq[k]);
            }
        }
        const unsigned nzmask = (unsigned)__ballot(l < 16 && nzb);  // block b's flag at bit b
        for (int k = 0; k < 16; k++) y_nz_out[k] = (int)((nzmask >> k) & 1u);
        wsync();
        PH_MARK_L(14, l, 0);
    } else {
        build_luma_border(C);
        int top_nz[4], left_nz[4];
        for (int k = 0; k < 4; k++) {
            top_nz[k] = C.top_c[C.ocx + 1 + k];
            left_nz[k] = C.M->left_c[1 + k];
        }
        for (int i = 0; i < 16; i++) {
            const int sby = i >> 2, sbx = i & 3, x0 = sbx * 4 + 1, y0 = sby * 4 + 1;
            const int bm = C.M->modes[i];
            i4_values(C, x0, y0);
            // 16-lane group form: every group computes the same block; group 0 stores
            const int k = l & 15;
            const int pk = i4_pred_at(W->V[0], i4_src_index(C.T, bm, k), W->V[0][5 + (k & 3)] - W->V[0][4]);
            const int svk = C.sY[(sby * 4 + (k >> 2)) * 16 + sbx * 4 + (k & 3)];
            const int ck = fdct_g(svk - pk, k);
            const int ctx0 = min(left_nz[sby] + top_nz[sbx], 2);
            if (C.a->dbg && C.a->pass == 2 && l < 16) {
                int* d = C.a->dbg + (((size_t)C.f * C.a->mbw * C.a->mbh + (size_t)C.mby * C.a->mbw + C.mbx) * 16 + i) * 34;
                d[k] = ck;
                d[16 + k] = pk;
                if (k == 0) {
                    d[32] = ctx0;
                    d[33] = bm;
                }
            }
            const int qs = quantz(ck, S.y1.iq[k > 0], S.y1.bias[k > 0]);
            const int snz = gmask(qs != 0) != 0;
            int dqk, nzq;
            if (trel) {
                // lane-parallel trellis: lane n = zigzag position n
                const int cn = gget(ck, zz_of(k));
                int lvn;
                nzq = trellis_g<0>(cn, k, S.y1, S.sharpen, S.lt_i4, C.T, 3, ctx0, lvn);
                if (l < 16) C.M->lev[i][k] = (int16_t)lvn;
                dqk = m24(gget(lvn, izz_of(k)), (int)S.y1.q[k > 0]);
            } else {
                if (l < 16) C.M->lev[i][izz_of(k)] = (int16_t)qs;
                nzq = snz;
                dqk = m24(qs, (int)S.y1.q[k > 0]);
            }
            const int rk = idct_g(dqk, k);
            if (l < 16) C.M->ws[(y0 + (k >> 2)) * ZW_BPS + x0 + (k & 3)] = (uint8_t)clamp255(pk + rk);
            wsync();
            if (l == 0) {
                W->misc[1] = nzq;
                W->misc[2] = snz;
            }
            wsync();
            const int nz = W->misc[1];
            anynz |= W->misc[2];
            top_nz[sbx] = nz;
            left_nz[sby] = nz;
            y_nz_out[i] = nz;
            wsync();
        }
        if (l < 16) C.M->lev[16][l] = 0;
        wsync();
        PH_MARK_L(15, l, 0);
        PH_COUNT(7);
    }
    return anynz;
}

// Final chroma transform with error diffusion (transform_chroma_blocks
// vp8.rs:3039, apply_chroma_error_diffusion :572), lane-pair form: lanes b and
// 32 + b work block b (U 0..3, V 4..7) from the coefficients pick_uv left for
// the chosen mode.  Levels to C.M->lev[17..24], recon into cu / cv.  Returns the
// simple-quant "any nonzero" flag; uv_nz[8] receives per-block has-coefficients.
__device__ int final_chroma(const Ctx& C, int mode, int8_t* top_derr, int uv_nz[8])
{
    WaveLds* W = C.W;
    const ZwSegment& S = *C.S;
    const int l = C.lane;
    const int h = l >> 5, b = l & 7, pl = b >> 2, bx = b & 1, by = (b >> 1) & 1;
    const bool act = (l & 31) < 8;
    int cf[2][4];
    uint32_t p01[2], p32[2];
    {
        const uint32_t* e = W->uvc[h * 32 + mode * 8 + b];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            cf[c][0] = lo16(e[2 * c]);
            cf[c][1] = hi16(e[2 * c]);
            cf[c][2] = lo16(e[2 * c + 1]);
            cf[c][3] = hi16(e[2 * c + 1]);
        }
        p01[0] = e[4];
        p32[0] = e[5];
        p01[1] = e[6];
        p32[1] = e[7];
    }
    // DC error diffusion (vp8.rs chroma quirk, per plane: blocks 0,1,2,3 in
    // order), on the scalar unit; block k's DC is cf[0][0] of lane k.
    {
        const int q = (int)S.uv.q[0];
        const uint32_t iq = S.uv.iq[0], bias = S.uv.bias[0];
        const uint32_t zt = S.uv.zthresh[0];  // ((1 << 17) - 1 - bias) / iq, matrix_init
        int dcs[8];
#pragma unroll
        for (int k = 0; k < 8; k++) dcs[k] = __builtin_amdgcn_readlane(cf[0][0], k);
        auto diffuse = [&](int& dc, int te, int le) -> int {
            dc += (7 * te + 8 * le) >> 3;
            const int sign = dc < 0;
            const uint32_t a = (uint32_t)(sign ? -dc : dc);
            const int level = a > zt ? (int)((a * iq + bias) >> 17) : 0;
            const int err = (int)a - level * q;
            const int se = sign ? -err : err;
            const int v = se >> 1;
            return (int)(int8_t)(v < -127 ? -127 : (v > 127 ? 127 : v));
        };
#pragma unroll
        for (int ch = 0; ch < 2; ch++) {
            int8_t* top = top_derr + ch * 2;
            int8_t* lft = C.M->left_derr + ch * 2;
            const int t0 = __builtin_amdgcn_readfirstlane((int)top[0]), t1 = __builtin_amdgcn_readfirstlane((int)top[1]);
            const int l0 = __builtin_amdgcn_readfirstlane((int)lft[0]), l1 = __builtin_amdgcn_readfirstlane((int)lft[1]);
            int* d = dcs + ch * 4;
            const int e0 = diffuse(d[0], t0, l0);
            const int e1 = diffuse(d[1], t1, e0);
            const int e2 = diffuse(d[2], e0, l1);
            const int e3 = diffuse(d[3], e1, e2);
            const int nl1 = (int)(int8_t)((3 * e3) >> 2);
            wsync();
            if (l == 0) {
                lft[0] = (int8_t)e1;
                lft[1] = (int8_t)nl1;
                top[0] = (int8_t)e2;
                top[1] = (int8_t)(e3 - nl1);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(cf[0][0]) : "s"(__builtin_amdgcn_readfirstlane(dcs[k])), "i"(k));
    }
    // quantize_coeff of this lane's 8 coefficients (natural index n = 4 row + 2h + col)
    int dq[2][4];
    int nz = 0;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool dcs = c == 0 && r == 0;
            const uint32_t iq = dcs ? (h ? S.uv.iq[1] : S.uv.iq[0]) : S.uv.iq[1];
            const uint32_t bias = dcs ? (h ? S.uv.bias[1] : S.uv.bias[0]) : S.uv.bias[1];
            const int q_ = dcs ? (int)(h ? S.uv.q[1] : S.uv.q[0]) : (int)S.uv.q[1];
            const int lv = quantz(cf[c][r], iq, bias);
            nz |= lv;
            if (act) C.M->lev[17 + b][izz_of(4 * r + 2 * h + c)] = (int16_t)lv;
            dq[c][r] = m24(lv, q_);
        }
    uint32_t r01[2], r32[2];
    idct_recon_pair(dq, p01, p32, h, r01, r32);
    if (act) {
        uint8_t* w = pl ? W->cv : W->cu;
#pragma unroll
        for (int r = 0; r < 2; r++) {
            uint8_t* row = w + (by * 4 + 2 * h + r + 1) * ZW_BPS + 1 + bx * 4;
            row[0] = (uint8_t)(r01[r] & 255u);
            row[1] = (uint8_t)(r01[r] >> 16);
            row[2] = (uint8_t)(r32[r] >> 16);
            row[3] = (uint8_t)(r32[r] & 255u);
        }
    }
    const int nzb = (nz | hx_partner(nz)) != 0;
    int any = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uv_nz[k] = __builtin_amdgcn_readlane(nzb, k);
        any |= uv_nz[k];
    }
    wsync();
    return any;
}

// Publish borders for the next MBs (vp8.rs:2771-2777, :3101-3118).
__device__ void store_luma_borders(const Ctx& C)
{
    const int l = C.lane;
    if (l < 17) C.M->left_y[l] = C.M->ws[l * ZW_BPS + 16];
    else if (l < 33) C.top_y[C.oy + (l - 17)] = C.M->ws[16 * ZW_BPS + (l - 17) + 1];
    if (C.a->ry && l < 64) {
        uint8_t* ry = C.a->ry + (size_t)C.f * C.a->ysz + (size_t)C.mby * 16 * C.ys + C.mbx * 16;
        for (int k = l; k < 256; k += 64) ry[(size_t)(k >> 4) * C.ys + (k & 15)] = C.M->ws[((k >> 4) + 1) * ZW_BPS + 1 + (k & 15)];
    }
    wsync();
}
__device__ void store_chroma_borders(const Ctx& C)
{
    const int l = C.lane;
    WaveLds* W = C.W;
    if (l < 9) {
        C.M->left_u[l] = W->cu[l * ZW_BPS + 8];
        C.M->left_v[l] = W->cv[l * ZW_BPS + 8];
    } else if (l < 17) {
        C.top_u[C.oc + (l - 9)] = W->cu[8 * ZW_BPS + (l - 9) + 1];
        C.top_v[C.oc + (l - 9)] = W->cv[8 * ZW_BPS + (l - 9) + 1];
    }
    if (C.a->ru) {
        uint8_t* ru = C.a->ru + (size_t)C.f * C.a->csz + (size_t)C.mby * 8 * C.cs + C.mbx * 8;
        uint8_t* rv = C.a->rv + (size_t)C.f * C.a->csz + (size_t)C.mby * 8 * C.cs + C.mbx * 8;
        const int k = l;
        ru[(size_t)(k >> 3) * C.cs + (k & 7)] = W->cu[((k >> 3) + 1) * ZW_BPS + 1 + (k & 7)];
        rv[(size_t)(k >> 3) * C.cs + (k & 7)] = W->cv[((k >> 3) + 1) * ZW_BPS + 1 + (k & 7)];
    }
    wsync();
}

__device__ void write_levels(const Ctx& C, int first_blk, int nblk, bool zero)
{
    ZwMbOut* o = C.a->out + (size_t)C.f * C.a->mbw * C.a->mbh + (size_t)C.mby * C.a->mbw + C.mbx;
    // as words (ZwMbOut records and the LDS levels are 4-byte aligned)
    uint32_t* dst = (uint32_t*)&o->levels[first_blk][0];
    const uint32_t* srcl = (const uint32_t*)&C.M->lev[first_blk][0];
    for (int k = C.lane; k < nblk * 8; k += 64) dst[k] = zero ? 0u : srcl[k];
}

// ---------------------------------------------------------------------------
// Pass-1 chroma chain in quad form, one wave per plane (chain wave 0: U,
// chain wave 1: V).  Lane l = 16 m + 4 b + q works mode m (0 DC, 1 V, 2 H,
// 3 TM) of 4x4 block b (bx = b & 1, by = b >> 1): pixel row q for the
// prediction, residual, row transform input and reconstruction; coefficient
// column q for the column transform, quantisation and rate.  A quad gathers
// its rows' row-transform inputs with DPP broadcasts and each lane forms its
// own column, so a lane does a quarter block and the plane's 4 modes x 4
// blocks fill one wave.  The arithmetic (packing points, rounding) is the pair
// form's (fdct_pair / idct_recon_pair), so the results are identical.  Only the
// mode decision couples the planes -- one RD over U + V (pick_best_uv,
// vp8.rs:2050-2200) -- and the waves trade their per-mode (rate, SSE, AC
// nonzeros) through LDS; the DC error diffusion (vp8.rs:572-647) runs per
// channel, so each wave keeps its own.  Halving the chain's instruction stream
// shortens pass 1, which the chain bounds for single frames (quirk A5 makes it
// serial across rows) and nearly bounds in batches.
// ---------------------------------------------------------------------------
struct UvQ {
    int pl;             // 0 U, 1 V
    uint8_t* w;         // the plane's work buffer (create_border_chroma layout, stride ZW_BPS)
    const uint8_t* sp;  // the MB's staged source plane (8x8, stride 8)
    uint8_t* top;       // frame-wide top row of the plane
    uint8_t* left;      // the wave's left column (corner + 8 rows)
};

// create_border_chroma (prediction.rs:85) of one plane
DI void uvq_border(const Ctx& C, const UvQ& U)
{
    const int l = C.lane;
    if (l < 17) {
        if (l == 0) U.w[0] = C.mby == 0 ? 127 : (C.mbx == 0 ? 129 : U.left[0]);
        else if (l <= 8) U.w[l] = C.mby == 0 ? 127 : U.top[C.mbx * 8 + l - 1];
        else U.w[(l - 8) * ZW_BPS] = C.mbx == 0 ? 129 : U.left[l - 8];
    }
    wsync();
}

// get_residual_cost (cost.rs:1670; ctype 2, first 0, ctx0 0; pass 1: the
// LevelCosts tables are zero, quirk A2) of the quad's block, av[r] = |level|
// at natural index 4 r + q.  Uniform in the quad.
DI int uvq_rcost(const int av[4], int q, const LdsTables* T)
{
    unsigned nz = 0, big = 0;
    int part = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int n = 4 * r + q;
        nz |= (unsigned)min(av[r], 1) << n;
        big |= (unsigned)(av[r] >= 2) << n;
        part += T->lfc[min(av[r], 2047)];
    }
    nz = (unsigned)quad_or((int)nz);
    big = (unsigned)quad_or((int)big);
    const int sum = quad_sum(part);
    const int last = 31 - __clz((int)nz);
    const int ctx_t = ((big >> max(last, 0)) & 1u) ? 2 : 1;
    const int tail = (int)T->beob[2][band_of(min(last + 1, 15))][ctx_t] & -(int)(last < 15);
    const int head = (int)T->binit[2][0][0];
    return csel(last < 0, (int)T->beob[2][0][0], head + sum + tail);  // (no divergent branch)
}

// pick_best_uv (vp8.rs:2050-2200) with the partner plane's wave: returns the
// chroma mode.  Leaves each lane's coefficients and prediction row in
// W->uvc[lane] for uvq_final.  xch: [plane][2][12] exchange words, xflag[2].
DI int uvq_pick(const Ctx& C, const UvQ& U, int* xch, int* xflag, int seq)
{
    const ZwSegment& S = *C.S;
    const LdsTables* T = C.T;
    WaveLds* W = C.W;
    const int l = C.lane, m = l >> 4, b = (l >> 2) & 3, q = l & 3, bx = b & 1, by = b >> 1;
    const int above = C.mby != 0, left = C.mbx != 0;
    // DC predictor (lanes 0..15: i < 8 left pixel i, i >= 8 top pixel i - 8)
    int dc;
    {
        const int i = l & 15;
        const int v = (int)U.w[csel(i < 8, (i + 1) * ZW_BPS, i - 7)] & -(int)(i < 8 ? left : above);
        const int su = __builtin_amdgcn_readlane(red16(v), 0);
        const int shf = 2 + left + above;
        dc = (above | left) ? (su + (1 << (shf - 1))) >> shf : 128;
    }
    // prediction and source of row y = 4 by + q (uv_rows_pk)
    uint32_t p01, p32, s01, s32;
    {
        const int cm = -(int)(m & 1), rm = -(int)(m >= 2);
        const int P = U.w[0];
        const int ro = csel(m == 0, dc, csel(m == 3, -P, 0));
        const uint8_t* tp = U.w + 1 + bx * 4;
        const uint32_t c01 = pack_lo(tp[0] & cm, tp[1] & cm), c32 = pack_lo(tp[3] & cm, tp[2] & cm);
        const int y = by * 4 + q;
        const int rv = (U.w[(y + 1) * ZW_BPS] & rm) + ro;
        const uint32_t rvv = pack_lo(rv, rv);
        p01 = clamp_pk(add_pk(c01, rvv));
        p32 = clamp_pk(add_pk(c32, rvv));
        const uint32_t sw = *(const uint32_t*)(U.sp + y * 8 + bx * 4);
        s01 = __builtin_amdgcn_perm(0u, sw, 0x0c010c00u);
        s32 = __builtin_amdgcn_perm(0u, sw, 0x0c020c03u);
    }
    const uint32_t R01 = sub_pk(s01, p01), R32 = sub_pk(s32, p32);
    int cf[4];
    uvq_fdct(add_pk(R01, R32), sub_pk(R01, R32), q, cf);
    {
        uint32_t* e = W->uvc[l];
        e[0] = pack_lo(cf[0], cf[1]);
        e[1] = pack_lo(cf[2], cf[3]);
        e[2] = p01;
        e[3] = p32;
    }
    // quantize_coeff (no sharpening, cost.rs:457): the DC is (r, q) = (0, 0)
    int av[4], dq[4], nzac = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool dcs = r == 0 && q == 0;
        const uint32_t iq = dcs ? S.uv.iq[0] : S.uv.iq[1];
        const uint32_t bias = dcs ? S.uv.bias[0] : S.uv.bias[1];
        const int q_ = dcs ? (int)S.uv.q[0] : (int)S.uv.q[1];
        const int v = cf[r];
        const int a = (int)((__umul24((uint32_t)iabs(v), iq) + bias) >> 17);
        av[r] = a;
        dq[r] = m24(v < 0 ? -a : a, q_);
        nzac += dcs ? 0 : min(a, 1);
    }
    const int cost = uvq_rcost(av, q, T);
    uint32_t r01, r32;
    uvq_idct_recon(dq, p01, p32, q, r01, r32);
    int sse = 0;
    {
        const uint32_t d01 = sub_pk(s01, r01), d32 = sub_pk(s32, r32);
        sse = dot2v(d01, d01, sse);
        sse = dot2v(d32, d32, sse);
    }
    // per-mode plane totals (a block's rate once, from its quad's lane 0)
    const int ct = red16(q == 0 ? cost : 0), st = red16(sse), nt = red16(nzac);
    int* mine = xch + (U.pl * 2 + (seq & 1)) * 12;
    const int* theirs = xch + ((1 - U.pl) * 2 + (seq & 1)) * 12;
    if ((l & 15) == 0) {
        mine[m * 3 + 0] = ct;
        mine[m * 3 + 1] = st;
        mine[m * 3 + 2] = nt;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (l == 0) __hip_atomic_store(&xflag[U.pl], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
    while (__hip_atomic_load(&xflag[1 - U.pl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < seq)
        __builtin_amdgcn_s_sleep(1);
    // the same decision in both waves: rd = (fixed + rate + pen) * lambda_uv + 256 * sse
    long long brd = 0x7fffffffffffffffLL;
    int bm = 0;
#pragma unroll
    for (int mm = 0; mm < 4; mm++) {
        const int c_o = __builtin_amdgcn_readfirstlane(theirs[mm * 3 + 0]);
        const int s_o = __builtin_amdgcn_readfirstlane(theirs[mm * 3 + 1]);
        const int n_o = __builtin_amdgcn_readfirstlane(theirs[mm * 3 + 2]);
        const int c_m = __builtin_amdgcn_readlane(ct, mm * 16), s_m = __builtin_amdgcn_readlane(st, mm * 16);
        const int n_m = __builtin_amdgcn_readlane(nt, mm * 16);
        const int fixed = sel4(mm, d_FIXED_COSTS_UV[0], d_FIXED_COSTS_UV[1], d_FIXED_COSTS_UV[2], d_FIXED_COSTS_UV[3]);
        const int pen = (mm > 0 && n_m + n_o <= 2) ? 140 * 8 : 0;
        const long long r_m = (long long)(fixed + c_m + c_o + pen) * (long long)S.l_uv + 256LL * (long long)(s_m + s_o);
        const int avail = mm == 0 || (mm == 1 && above) || (mm == 2 && left) || (mm == 3 && above && left);
        if (avail && r_m < brd) {
            brd = r_m;
            bm = mm;
        }
    }
    return bm;
}

// transform_chroma_blocks (vp8.rs:3039-3121) of one plane under mode cm:
// the DC error diffusion of channel U.pl (vp8.rs:572-647), quantisation,
// levels into C.M->lev[17 + 4 pl + b], reconstruction into the work buffer.
DI void uvq_final(const Ctx& C, const UvQ& U, int cm, int8_t* top_derr)
{
    WaveLds* W = C.W;
    const ZwSegment& S = *C.S;
    const int l = C.lane, b = (l >> 2) & 3, q = l & 3, bx = b & 1, by = b >> 1;
    const bool act = l < 16;
    int cf[4];
    uint32_t p01, p32;
    {
        const uint32_t* e = W->uvc[cm * 16 + (l & 15)];
        cf[0] = lo16(e[0]);
        cf[1] = hi16(e[0]);
        cf[2] = lo16(e[1]);
        cf[3] = hi16(e[1]);
        p01 = e[2];
        p32 = e[3];
    }
    {
        const int qd = (int)S.uv.q[0];
        const uint32_t iq = S.uv.iq[0], bias = S.uv.bias[0];
        const uint32_t zt = S.uv.zthresh[0];  // ((1 << 17) - 1 - bias) / iq, matrix_init
        int d[4];
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = __builtin_amdgcn_readlane(cf[0], 4 * k);
        auto diffuse = [&](int& dc, int te, int le) -> int {
            dc += (7 * te + 8 * le) >> 3;
            const int sign = dc < 0;
            const uint32_t a = (uint32_t)(sign ? -dc : dc);
            const int level = a > zt ? (int)((a * iq + bias) >> 17) : 0;
            const int err = (int)a - level * qd;
            const int se = sign ? -err : err;
            const int v = se >> 1;
            return (int)(int8_t)(v < -127 ? -127 : (v > 127 ? 127 : v));
        };
        int8_t* top = top_derr + U.pl * 2;
        int8_t* lft = C.M->left_derr;
        const int t0 = __builtin_amdgcn_readfirstlane((int)top[0]), t1 = __builtin_amdgcn_readfirstlane((int)top[1]);
        const int l0 = __builtin_amdgcn_readfirstlane((int)lft[0]), l1 = __builtin_amdgcn_readfirstlane((int)lft[1]);
        const int e0 = diffuse(d[0], t0, l0);
        const int e1 = diffuse(d[1], t1, e0);
        const int e2 = diffuse(d[2], e0, l1);
        const int e3 = diffuse(d[3], e1, e2);
        const int nl1 = (int)(int8_t)((3 * e3) >> 2);
        wsync();
        if (l == 0) {
            lft[0] = (int8_t)e1;
            lft[1] = (int8_t)nl1;
            top[0] = (int8_t)e2;
            top[1] = (int8_t)(e3 - nl1);
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            asm volatile("v_writelane_b32 %0, %1, %2"
                         : "+v"(cf[0])
                         : "s"(__builtin_amdgcn_readfirstlane(d[k])), "i"(4 * k));
    }
    int dq[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const bool dcs = r == 0 && q == 0;
        const int lv = quantz(cf[r], dcs ? S.uv.iq[0] : S.uv.iq[1], dcs ? S.uv.bias[0] : S.uv.bias[1]);
        if (act) C.M->lev[17 + 4 * U.pl + b][izz_of(4 * r + q)] = (int16_t)lv;
        dq[r] = m24(lv, dcs ? (int)S.uv.q[0] : (int)S.uv.q[1]);
    }
    uint32_t r01, r32;
    uvq_idct_recon(dq, p01, p32, q, r01, r32);
    if (act) {
        uint8_t* row = U.w + (by * 4 + q + 1) * ZW_BPS + 1 + bx * 4;
        row[0] = (uint8_t)(r01 & 255u);
        row[1] = (uint8_t)(r01 >> 16);
        row[2] = (uint8_t)(r32 >> 16);
        row[3] = (uint8_t)(r32 & 255u);
    }
    wsync();
}

// Borders of one plane for the next MBs (vp8.rs:3101-3118), and its debug
// reconstruction when asked for.
DI void uvq_store_borders(const Ctx& C, const UvQ& U)
{
    const int l = C.lane;
    if (l < 9) U.left[l] = U.w[l * ZW_BPS + 8];
    else if (l < 17) U.top[C.mbx * 8 + (l - 9)] = U.w[8 * ZW_BPS + (l - 9) + 1];
    uint8_t* rp = U.pl ? C.a->rv : C.a->ru;
    if (rp) {
        rp += (size_t)C.f * C.a->csz + (size_t)C.mby * 8 * C.cs + C.mbx * 8;
        rp[(size_t)(l >> 3) * C.cs + (l & 7)] = U.w[((l >> 3) + 1) * ZW_BPS + 1 + (l & 7)];
    }
    wsync();
}

// What an MB needs from global memory, fetched one MB ahead (the loads are in
// flight while the previous MB is encoded): the lane's word of the source MB
// (luma: row lane>>2, word lane&3; chroma lanes < 32: plane lane>>4, row
// (lane>>1)&7, word lane&1) and the MB's alpha (segment lookup).
struct MbFetch {
    uint32_t y, c;
    int alpha;
};
__device__ __forceinline__ MbFetch fetch_mb(const EncArgs* a, int f, int lane, int mbx, int mby)
{
    const int ys = a->mbw * 16, cs = a->mbw * 8;
    const uint8_t* sy = a->Y + (size_t)f * a->ysz + (size_t)mby * 16 * ys + mbx * 16;
    MbFetch r;
    r.y = *(const uint32_t*)(sy + (size_t)(lane >> 2) * ys + (lane & 3) * 4);
    r.c = 0;
    if (lane < 32) {
        const int pl = lane >> 4, k = lane & 15;
        const uint8_t* sp = (pl ? a->V : a->U) + (size_t)f * a->csz + (size_t)mby * 8 * cs + mbx * 8;
        r.c = *(const uint32_t*)(sp + (size_t)(k >> 1) * cs + (k & 1) * 4);
    }
    r.alpha = a->alpha[(size_t)f * a->mbw * a->mbh + (size_t)mby * a->mbw + mbx];
    return r;
}

__device__ void setup_ctx(Ctx& C, const EncArgs* a, const uint8_t* seg_lut, WaveLds* W, int mbx, int mby,
                          const MbFetch& m)
{
    C.mbx = mbx;
    C.mby = mby;
    const int f = C.f;
    C.ys = a->mbw * 16;
    C.cs = a->mbw * 8;
    C.srcY = a->Y + (size_t)f * a->ysz + (size_t)mby * 16 * C.ys + mbx * 16;
    C.srcU = a->U + (size_t)f * a->csz + (size_t)mby * 8 * C.cs + mbx * 8;
    C.srcV = a->V + (size_t)f * a->csz + (size_t)mby * 8 * C.cs + mbx * 8;
    // stage the source MB in LDS: 64 lanes x 4 B luma, 32 lanes x 4 B chroma
    {
        const int l = C.lane;
        ((uint32_t*)C.M->sy)[l] = m.y;
        if (l < 32) ((uint32_t*)((l >> 4) ? C.M->sv : C.M->su))[l & 15] = m.c;
        C.sY = C.M->sy;
        C.sU = C.M->su;
        C.sV = C.M->sv;
    }
    wsync();
    // wave-uniform: the segment's matrices / lambdas / sharpening come from LDS;
    // seg_lut is the k-means alpha -> segment map (all zero without segments)
    const int seg = __builtin_amdgcn_readfirstlane((int)seg_lut[m.alpha]);
    C.seg = seg;
    C.S = C.Sl + seg;
}

__device__ void wait_row(const int* progress, int wave_of_prev, int need)
{
    while (__hip_atomic_load(&progress[wave_of_prev], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
        __builtin_amdgcn_s_sleep(1);
}
// s_setprio with a wave-uniform level
DI void set_prio(int p)
{
    if (p >= 3) __builtin_amdgcn_s_setprio(3);
    else if (p == 2) __builtin_amdgcn_s_setprio(2);
    else if (p == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
__device__ void publish(int* progress, int wave, int val)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(&progress[wave], val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_wave_barrier();
}


// The lane id as a value the compiler cannot prove loop-invariant.  Taken at
// the top of every MB iteration, it keeps lane-derived constants (per-lane
// offsets, 64-bit source pointers, table indices) from being hoisted out of
// the MB loops and held -- or spilled -- across them: they are cheap to
// recompute and the registers go to the search stages.
__device__ __forceinline__ int opaque_lane(int lane)
{
    asm volatile("" : "+v"(lane));
    return lane;
}

// ---------------------------------------------------------------------------
// Row-parallel encode (small batches, single frames): one wave per workgroup,
// MB rows handed out by a per-frame ticket, the row-to-row state (top_y, and in
// pass 2 top_u/v, top_c, top_derr) and the progress counters in global memory.
// A wave only waits for a row whose ticket an already running wave holds, so
// the grid cannot deadlock whatever the residency.  Hand-off: every byte of the
// row state is stored sc1 (write-through) and drained (vmcnt(0)) before the
// sc1 progress store; the consumer polls progress with sc1 loads and reads the
// bytes with sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility).
// Pass 1's chroma raster chain (quirk A5) runs in workgroup 0 of each frame,
// with its top_u/v/derr in its own LDS, as in the batch kernels.
// ---------------------------------------------------------------------------
struct RowsLayout {
    size_t sync, ty, tu, tv, tc, td, frame;
    __host__ __device__ RowsLayout(int mbw, int mbh)
    {
        auto a16 = [](size_t v) { return (v + 15) & ~(size_t)15; };
        sync = 0;                                  // int [4 + mbh]: ticket, pad x3, done MBs per row
        ty = a16(4 * (4 + (size_t)mbh));
        tu = ty + a16((size_t)mbw * 16 + 16);
        tv = tu + a16((size_t)mbw * 8);
        tc = tv + a16((size_t)mbw * 8);
        td = tc + a16((size_t)mbw * 12);
        frame = td + a16((size_t)mbw * 4);
    }
};
#define ZW_ROWS_HDR 256  // launch header: [0] error word (a wave gave up waiting)
#define ZW_ENC_SPIN_MAX (1 << 22)
DI uint32_t ld_sc1(const void* p) { return __hip_atomic_load((const uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DI void st_sc1(void* p, uint32_t v) { __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DI int row_ticket(int* ticket)
{
    int t = 0;
    if ((threadIdx.x & 63) == 0) t = atomicAdd(ticket, 1);
    return __builtin_amdgcn_readfirstlane(__shfl(t, 0));
}
// Wait until *prog >= need; seen caches the last value read (the row above
// usually runs ahead, so most waits cost no memory round trip).  After
// ZW_ENC_SPIN_MAX polls, or once another wave gave up, report through *err.
DI void row_wait(const int* prog, int need, int* err, int& seen)
{
    if (seen >= need) return;
    int it = 0;
    for (;;) {
        seen = __builtin_amdgcn_readfirstlane((int)ld_sc1(prog));
        if (seen >= need) break;
        __builtin_amdgcn_s_sleep(1);
        if (++it > ZW_ENC_SPIN_MAX || ((it & 1023) == 0 && ld_sc1(err))) {
            if ((threadIdx.x & 63) == 0) atomicOr(err, 1);
            seen = 1 << 30;
            break;
        }
    }
    // pairs with row_publish's release: the row state loads below may not be
    // hoisted above the poll (C++ memory model, not only GFX9's in-order returns)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
DI void row_publish(int* prog, int val)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are out
    if ((threadIdx.x & 63) == 0)
        __hip_atomic_store((uint32_t*)prog, (uint32_t)val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_wave_barrier();
}

// Pass 1's chroma chain: one wave (pair form) or two (quad form, one wave per
// plane).  The row-parallel kernels take the two-wave chain: it bounds their
// pass 1 (one 1080p frame: 27.7 -> 22.1 ms), and their pass-1 workgroups then
// run two waves (the chain's two planes; two luma rows elsewhere).  The batch
// kernels keep one chain wave: there a second one costs a luma wave and
// measured slower (34.4 -> 35.0 ms per 256 1080p frames).
#ifndef ZW_UVQ_CHAIN_ROWS
#define ZW_UVQ_CHAIN_ROWS 1
#endif
#ifndef ZW_UVQ_CHAIN_BATCH
#define ZW_UVQ_CHAIN_BATCH 0
#endif
template <bool ROWS> struct ChainShape {
    static constexpr int NCH = (ROWS ? ZW_UVQ_CHAIN_ROWS : ZW_UVQ_CHAIN_BATCH) ? 2 : 1;
};
// the per-MB stage loops of the frame-pair kernel: ZW_PAIR_UNROLL 1 emits
// each stage twice (constant frame index), 0 once (a two-trip loop); measured
// per 256 1080p frames: pass 2 29.80 vs 30.26 ms, pass 1 the same
#ifndef ZW_PAIR_UNROLL
#define ZW_PAIR_UNROLL 1
#endif
#if ZW_PAIR_UNROLL
#define ZW_PAIR_LOOP _Pragma("unroll")
#else
#define ZW_PAIR_LOOP _Pragma("nounroll")
#endif
template <int PASS> struct RowsShape {
    static constexpr int NW = PASS == 1 ? ChainShape<true>::NCH : 1;
};

// Bytes of the frame-wide row arrays a workgroup keeps in LDS: top_y, top_u,
// top_v, top_c, top_derr.  The batch kernels (one workgroup per frame) keep all
// of them; in the row-parallel kernels the luma waves work from per-MB windows
// of the global row state, and only pass 1's chroma chain keeps top_u / top_v /
// top_derr, so their LDS no longer grows with the width (which is what bounded
// the encodable width: 1 568 MBs with the batch shapes, any u16 width here).
struct TopLds {
    size_t y, u, v, c, d;
    __host__ __device__ TopLds(int mbw, bool rows, int pass)
    {
        const bool all = !rows, chain = rows && pass == 1;
        y = all ? (((size_t)mbw * 16 + 48 + 15) & ~(size_t)15) : 0;
        u = v = all || chain ? (((size_t)mbw * 8 + 48 + 15) & ~(size_t)15) : 0;
        c = all ? (((size_t)mbw * 12 + 15) & ~(size_t)15) : 0;
        d = all || chain ? (((size_t)mbw * 4 + 15) & ~(size_t)15) : 0;
    }
};

template <int PASS, bool ROWS, int FP = 1>
__device__ __forceinline__ void encode_body(const EncArgs& a)
{
    constexpr int NW = ROWS ? RowsShape<PASS>::NW : PassShape<PASS>::NW, WG = NW * 64;
    constexpr int NCH = PASS == 1 ? ChainShape<ROWS>::NCH : 0;  // chain waves (pass 1)
    constexpr bool PAIR = FP == 2;  // frame pairs: the workgroup encodes frames f and f + 1
    static_assert(FP == 1 || (FP == 2 && !ROWS), "frame pairs: the batch kernels");
    // pass 1's chroma chain waves: in frame pairs one per frame (the one-wave
    // form), else NCH (the quad form's two waves in the row kernels)
    constexpr int NCW = PASS == 1 ? (PAIR ? 2 : NCH) : 0;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int f = ROWS ? blockIdx.y : blockIdx.x * FP;
    const int nf = PAIR ? min(2, a.nframes - f) : 1;  // frames of this workgroup
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int mbw = a.mbw, mbh = a.mbh;
    const ZwFrameParams* P = a.params + f;
    // carve LDS
    size_t off = 0;
    // (per frame of the workgroup: the tables, segments, alpha map and the top rows)
    constexpr size_t sT = (sizeof(LdsTables) + 15) & ~(size_t)15, sS = (4 * sizeof(ZwSegment) + 15) & ~(size_t)15;
    LdsTables* T = (LdsTables*)(smem + off);
    off += sT * FP;
    ZwSegment* Sl = (ZwSegment*)(smem + off);  // the frame's 4 segments (matrices, lambdas, sharpening)
    off += sS * FP;
    uint8_t* seg_lut = smem + off;  // alpha -> segment (zeros when segmentation is off)
    off += 256 * FP;
    WaveLds* Wall = (WaveLds*)(smem + off);
    off += ((sizeof(WaveLds) + 15) & ~(size_t)15) * NW;
    MbLds* Mall2 = (MbLds*)(smem + off);  // frame pairs: the second frame's per-MB state
    off += PAIR ? ((sizeof(MbLds) + 15) & ~(size_t)15) * NW : 0;
    int* progress = (int*)(smem + off);
    off += 64;
    int* xch = (int*)(smem + off);  // two-wave chroma chain: [plane][2][12] exchange words, then 2 flags
    int* xflag = xch + 48;
    off += 256;
    const TopLds TS(mbw, ROWS, PASS);
    uint8_t* top_y = smem + off;
    off += TS.y * FP;
    uint8_t* top_u = smem + off;
    off += TS.u * FP;
    uint8_t* top_v = smem + off;
    off += TS.v * FP;
    uint8_t* top_c = smem + off;  // [mbw][12]: y2, y[4], u[2], v[2]
    off += TS.c * FP;
    int8_t* top_derr = (int8_t*)(smem + off);  // [mbw][4]
    WaveLds* W = (WaveLds*)((uint8_t*)Wall + ((sizeof(WaveLds) + 15) & ~(size_t)15) * wv);
    // row-parallel: is this workgroup pass 1's chroma chain (it keeps the
    // frame-wide top_u/v/derr in LDS), and the frame's global row state
    const bool chain_wg = PASS == 1 && (ROWS ? blockIdx.x == 0 : wv < NCW);
    const RowsLayout RL(mbw, mbh);
    uint8_t* rb = ROWS ? a.rows + ZW_ROWS_HDR + (size_t)f * RL.frame : nullptr;
    int* rerr = ROWS ? (int*)a.rows : nullptr;
    int* rsync = (int*)rb;

    // init shared state (each frame of the workgroup)
#pragma unroll
    for (int fr = 0; fr < FP; fr++) {
        if (fr >= nf) break;
        const int ff = f + fr;
        const ZwFrameParams* Pf = a.params + ff;
        LdsTables* Tf = (LdsTables*)((uint8_t*)T + sT * fr);
        ZwSegment* Sf = (ZwSegment*)((uint8_t*)Sl + sS * fr);
        uint8_t* lut = seg_lut + 256 * fr;
        for (int i = threadIdx.x; i < (int)(sizeof(Tf->lc) / 2); i += WG)
            (&Tf->lc[0][0][0][0])[i] = a.lcost ? (&a.lcost[ff].lc[0][0][0][0])[i] : 0;
        for (int i = threadIdx.x; i < 96; i += WG) {
            (&Tf->eob[0][0][0])[i] = a.lcost ? (&a.lcost[ff].eob[0][0][0])[i] : 0;
            (&Tf->init[0][0][0])[i] = a.lcost ? (&a.lcost[ff].init[0][0][0])[i] : 0;
        }
        for (int i = threadIdx.x; i < 4 * 8 * 3 * 11; i += WG) (&Tf->probs[0][0][0][0])[i] = (&Pf->probs[0][0][0][0])[i];
        static_assert(sizeof(ZwSegment) % 4 == 0, "segment copy by dwords");
        for (int i = threadIdx.x; i < (int)(4 * sizeof(ZwSegment) / 4); i += WG)
            ((uint32_t*)Sf)[i] = ((const uint32_t*)Pf->seg)[i];
        for (int i = threadIdx.x; i < 256; i += WG) lut[i] = Pf->seg_enabled ? Pf->seg_map_lut[i] : 0;
        load_static_tables(Tf, threadIdx.x, WG, &Pf->probs[0][0][0][0]);
        if (!ROWS || chain_wg) {
            uint8_t* ty = top_y + TS.y * fr;
            uint8_t* tu = top_u + TS.u * fr;
            uint8_t* tv = top_v + TS.v * fr;
            uint8_t* tcx = top_c + TS.c * fr;
            int8_t* td = top_derr + TS.d * fr;
            if (!ROWS) {
                for (int i = threadIdx.x; i < mbw * 16 + 48; i += WG) ty[i] = 127;
                for (int i = threadIdx.x; i < mbw * 12; i += WG) tcx[i] = 0;
            }
            for (int i = threadIdx.x; i < mbw * 8 + 48; i += WG) {
                tu[i] = 127;
                tv[i] = 127;
            }
            for (int i = threadIdx.x; i < mbw * 4; i += WG) td[i] = PASS == 2 ? a.derr[(size_t)ff * mbw * 4 + i] : 0;
        }
    }
    if (threadIdx.x < NW) progress[threadIdx.x] = -1;
    if (threadIdx.x < 2) xflag[threadIdx.x] = 0;
    if (ROWS && lane < 12) W->win_c[lane] = 0;  // pass 1: the complexity contexts stay zero
    __syncthreads();

    Ctx C;
    C.a = &a;
    C.P = P;
    C.T = T;
    C.W = W;
    C.M = &W->mb;
    C.lane = lane;
    C.f = f;
    C.Sl = Sl;
    C.method = __builtin_amdgcn_readfirstlane(P->method);
    C.top_y = top_y;
    C.top_u = top_u;
    C.top_v = top_v;
    C.top_c = top_c;
    C.top_derr = top_derr;
    C.oy = C.oc = C.ocx = C.od = 0;
    const bool trel = PASS == 2 && __builtin_amdgcn_readfirstlane(P->do_trellis);
    // without trellis (and without the pass-2 I4 dump) the final I4 blocks are
    // the search's winners, which the search leaves in C.M->lev / C.M->ws
    const bool keep_i4 = !trel && (PASS == 1 || a.dbg == nullptr);
    const size_t nmb = (size_t)mbw * mbh;
#ifdef ZW_PHASE_PROF
    if (lane < 24) W->ph[lane] = 0;
    wsync();
    auto ph_flush = [&]() {
        if (lane < 24) atomicAdd(&zw_phase_cycles_dev[PASS - 1][lane], W->ph[lane]);
        if (lane < 24) atomicAdd(&zw_wave_cycles_dev[PASS - 1][wv][lane], W->ph[lane]);
    };
#else
    auto ph_flush = []() {};
#endif

    if (chain_wg) {
        // ---- pass-1 chroma raster chain ----
        // the chain is pass 1's critical path: it takes issue priority over the
        // luma waves sharing its SIMD (measured: 47.6 -> 44.3 ms per 256 1080p
        // frames against luma-first priority at 12 waves)
#ifndef ZW_CHAIN_PRIO
#define ZW_CHAIN_PRIO 3
#endif
        __builtin_amdgcn_s_setprio(ZW_CHAIN_PRIO);
        // frame pairs: chain wave k works frame f + k
        const int cfr = PAIR ? wv : 0;
        if (PAIR && cfr >= nf) {
            ph_flush();
            return;
        }
        const int fc = f + cfr;
        const uint8_t* const lutc = seg_lut + 256 * cfr;
        int8_t* const tdc = top_derr + TS.d * cfr;
        if (PAIR) {
            C.f = fc;
            C.P = a.params + fc;
            C.T = (const LdsTables*)((const uint8_t*)T + sT * cfr);
            C.Sl = (const ZwSegment*)((const uint8_t*)Sl + sS * cfr);
            C.top_u = top_u + TS.u * cfr;
            C.top_v = top_v + TS.v * cfr;
            C.top_derr = tdc;
            C.method = __builtin_amdgcn_readfirstlane(C.P->method);
        }
        if (lane < 4) C.M->left_derr[lane] = 0;
        if (NCH == 2 && !PAIR) {
            // quad form: wave 0 the U plane, wave 1 the V plane
            const int pl = wv;
            UvQ U;
            U.pl = pl;
            U.w = W->cu;
            U.sp = C.M->su;
            U.top = pl ? top_v : top_u;
            U.left = C.M->left_u;
            const uint8_t* const P0 = (pl ? a.V : a.U) + (size_t)f * a.csz;
            const int cs = mbw * 8;
            auto fetch_uv = [&](int mbx, int mby) {
                MbFetch r;
                r.y = lane < 16 ? *(const uint32_t*)(P0 + (size_t)(mby * 8 + (lane >> 1)) * cs + mbx * 8 + (lane & 1) * 4)
                                : 0u;
                r.c = 0;
                r.alpha = a.alpha[(size_t)f * nmb + (size_t)mby * mbw + mbx];
                return r;
            };
            C.ys = mbw * 16;
            C.cs = cs;
            MbFetch nx = fetch_uv(0, 0);
            int seq = 0;
            for (int mby = 0; mby < mbh; mby++) {
                if (lane < 12) C.M->left_u[lane] = 129;
                wsync();
                for (int mbx = 0; mbx < mbw; mbx++) {
                    PH_START();
                    const int lane = opaque_lane(threadIdx.x & 63);
                    C.lane = lane;
                    const MbFetch cur = nx;
                    if (mbx + 1 < mbw) nx = fetch_uv(mbx + 1, mby);
                    else if (mby + 1 < mbh) nx = fetch_uv(0, mby + 1);
                    C.mbx = mbx;
                    C.mby = mby;
                    if (lane < 16) ((uint32_t*)C.M->su)[lane] = cur.y;
                    wsync();
                    const int seg = __builtin_amdgcn_readfirstlane((int)seg_lut[cur.alpha]);
                    C.seg = seg;
                    C.S = C.Sl + seg;
                    uvq_border(C, U);
                    const int cm = uvq_pick(C, U, xch, xflag, ++seq);
                    PH_MARK(8);
                    uvq_final(C, U, cm, top_derr + mbx * 4);
                    PH_MARK(9);
                    uvq_store_borders(C, U);
                    ZwMbOut* o = a.out + (size_t)f * nmb + (size_t)mby * mbw + mbx;
                    if (pl == 0 && lane == 0) o->chroma_mode = (uint8_t)cm;
                    write_levels(C, 17 + 4 * pl, 4, false);
                    wsync();
                }
            }
            for (int i = lane; i < mbw * 2; i += 64) {
                const int j = (i >> 1) * 4 + pl * 2 + (i & 1);
                a.derr[(size_t)f * mbw * 4 + j] = top_derr[j];
            }
            ph_flush();
            return;
        }
        MbFetch nx = fetch_mb(&a, fc, lane, 0, 0);
        for (int mby = 0; mby < mbh; mby++) {
            if (lane < 12) {
                C.M->left_u[lane] = 129;
                C.M->left_v[lane] = 129;
            }
            wsync();
            for (int mbx = 0; mbx < mbw; mbx++) {
                PH_START();
                const int lane = opaque_lane(threadIdx.x & 63);
                C.lane = lane;
                const MbFetch cur = nx;
                if (mbx + 1 < mbw) nx = fetch_mb(&a, fc, lane, mbx + 1, mby);
                else if (mby + 1 < mbh) nx = fetch_mb(&a, fc, lane, 0, mby + 1);
                setup_ctx(C, &a, lutc, W, mbx, mby, cur);
                C.oc = mbx * 8;
                C.ocx = mbx * 12;
                build_chroma_border(C);
                const int cm = pick_uv<PASS>(C);
                PH_MARK(8);
                int uvnz[8];
                final_chroma(C, cm, tdc + mbx * 4, uvnz);
                PH_MARK(9);
                store_chroma_borders(C);
                ZwMbOut* o = a.out + (size_t)fc * nmb + (size_t)mby * mbw + mbx;
                if (lane == 0) o->chroma_mode = (uint8_t)cm;
                write_levels(C, 17, 8, false);
                wsync();
            }
        }
        for (int i = lane; i < mbw * 4; i += 64) a.derr[(size_t)fc * mbw * 4 + i] = tdc[i];
        ph_flush();
        return;
    }

    // Pass 1 luma waves: below the chroma chain (ZW_CHAIN_PRIO), which sets the
    // pass's length once 11 waves share the luma wavefront.
#ifndef ZW_LUMA_PRIO
#define ZW_LUMA_PRIO 0
#endif
    if (PASS == 1) __builtin_amdgcn_s_setprio(ZW_LUMA_PRIO);
    const int nrw = PASS == 1 ? NW - NCH : NW;  // waves on the luma wavefront
    // Row k of each round of nrw rows goes to wave luma_wave(k).  In pass 1 the
    // luma waves that share SIMD 0 with the chroma chain (issue priority 3)
    // run slowest, and every later row of a round waits on a slow row: they
    // take the last rows of each round, which only the next round's first
    // row follows, with a round of slack.
#ifndef ZW_P1_ORDER
#define ZW_P1_ORDER 1
#endif
    auto p1_before = [](int v, int w) {  // wave v takes its row of a round before wave w
        const bool sv = (v & 3) < NCH, sw = (w & 3) < NCH;
        return (ZW_P1_ORDER && sv != sw) ? sw : v < w;
    };
    auto luma_rank = [&](int w) {
        if (PASS == 2) return w;
        int r = 0;
        for (int v = NCH; v < NW; v++) r += (int)p1_before(v, w);
        return r;
    };
    auto luma_wave = [&](int k) {
        if (PASS == 2) return k;
        int w = NCH;
        for (int v = NCH; v < NW; v++)
            if (luma_rank(v) == k) w = v;
        return w;
    };
    // ZW_P1_SLOWSKIP (pass 1, batch shape): the luma waves on SIMD 0 (beside
    // the chain) take fewer rows.  Rows go out in rounds: the nfast rows of the
    // other SIMDs' waves, then the round's share of SIMD-0 rows (the SIMD-0
    // waves in turn), ZW_P1_SLOW_NUM SIMD-0 rows per ZW_P1_SLOW_DEN rounds.  So
    // SIMD 0 carries the chain plus fewer luma rows, and its rows keep pace
    // with the rest instead of throttling every row behind them.
#ifndef ZW_P1_SLOWSKIP
#define ZW_P1_SLOWSKIP 1
#endif
#ifndef ZW_P1_SLOW_NUM
#define ZW_P1_SLOW_NUM 1  // re-tuned in round 4 (1080p, 256 frames, one lane): 1/1 28.2-28.3 ms, 3/2 28.8-29.0,
#endif                    // 2/3 29.0-29.1, 1/2 29.2, 4/3 29.8, 0/1 29.9, 2/1 31.7
#ifndef ZW_P1_SLOW_DEN
#define ZW_P1_SLOW_DEN 1
#endif
    constexpr bool skip_mode = ZW_P1_SLOWSKIP && PASS == 1 && !ROWS && NCH == 1 && NW > 4;
    constexpr int nslow = (NW - 1) / 4 > 0 ? (NW - 1) / 4 : 1;  // luma waves on SIMD 0: 4, 8, ..
    constexpr int nfast = NW - NCH - (NW - 1) / 4;             // luma waves on SIMDs 1..3
    auto fast_wave = [](int i) { return i + 1 + i / 3; };
    auto wave_of_row = [&](int y) {
        if (!skip_mode) return luma_wave(y % (nrw > 0 ? nrw : 1));
        constexpr int L = ZW_P1_SLOW_DEN * nfast + ZW_P1_SLOW_NUM;
        int r = y % L, before = (y / L) * ZW_P1_SLOW_NUM;
        for (int k = 0; k < ZW_P1_SLOW_DEN; k++) {
            const int sk = ((k + 1) * ZW_P1_SLOW_NUM) / ZW_P1_SLOW_DEN - (k * ZW_P1_SLOW_NUM) / ZW_P1_SLOW_DEN;
            if (r < nfast) return fast_wave(r);
            r -= nfast;
            if (r < sk) return 4 * (1 + (before + r) % nslow);
            r -= sk;
            before += sk;
        }
        return 0;  // unreachable
    };
    // skip mode: the wave's next row after `y`
    auto next_row = [&](int y) {
        for (y++; y < mbh; y++)
            if (wave_of_row(y) == wv) break;
        return y;
    };
    const int rw = ROWS ? 0 : (skip_mode ? next_row(-1) : luma_rank(wv));
    if (ROWS) {
        // the wave's window stands in for the frame-wide top arrays (offsets 0)
        C.top_y = W->win_y;
        C.top_u = W->win_u;
        C.top_v = W->win_v;
        C.top_c = W->win_c;
        C.top_derr = W->win_d;
    }
    // everything of an MB after its searches: the final transforms, the
    // complexity contexts (pass 2), the levels, the MB record and the borders
    auto mb_store = [&](Ctx& C, int lm, int cm, bool i4reuse, uint32_t i4nz, bool trel) __attribute__((always_inline)) {
        const int lane = C.lane;
        PH_START();
        int ynz[16];
        const int lnz = final_luma(C, lm, trel, ynz, i4reuse ? (int)i4nz : -1);
        PH_MARK(4);
        int uvnz[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int cnz = 0;
        if (PASS == 2) cnz = final_chroma(C, cm, C.top_derr + C.od, uvnz);
        PH_MARK(5);
        ZwMbOut* o = a.out + (size_t)C.f * nmb + (size_t)C.mby * mbw + C.mbx;
        if (PASS == 2) {
            const int skip = !(lnz | cnz);
            // complexity (encode_residual_data semantics / skip clearing)
            if (lane == 0) {
                uint8_t* tc = C.top_c + C.ocx;
                uint8_t* lc = C.M->left_c;
                if (skip) {
                    for (int k = 1; k < 9; k++) tc[k] = lc[k] = 0;
                    if (lm != 4) tc[0] = lc[0] = 0;
                } else {
                    if (lm != 4) {
                        int y2nz = 0;
                        for (int n = 0; n < 16; n++) y2nz |= C.M->lev[16][n] != 0;
                        tc[0] = lc[0] = (uint8_t)y2nz;
                    }
                    for (int x = 0; x < 4; x++) tc[1 + x] = (uint8_t)ynz[12 + x];
                    for (int y = 0; y < 4; y++) lc[1 + y] = (uint8_t)ynz[y * 4 + 3];
                    tc[5] = (uint8_t)uvnz[2];
                    tc[6] = (uint8_t)uvnz[3];
                    lc[5] = (uint8_t)uvnz[1];
                    lc[6] = (uint8_t)uvnz[3];
                    tc[7] = (uint8_t)uvnz[6];
                    tc[8] = (uint8_t)uvnz[7];
                    lc[7] = (uint8_t)uvnz[5];
                    lc[8] = (uint8_t)uvnz[7];
                }
                o->skip = (uint8_t)skip;
                o->chroma_mode = (uint8_t)cm;
            }
            store_chroma_borders(C);
            write_levels(C, 0, 25, skip);
            if (a.sizes) {
                // the packed record size k_pack_size would compute from these
                // levels: header, eob bytes and every block's levels up to its eob
                int e = 0;
                if (lane < 25 && !skip) {
                    const uint32_t* lw = (const uint32_t*)C.M->lev[lane];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const uint32_t v = lw[q];
                        e = (v >> 16) ? 2 * q + 2 : ((v & 0xffffu) ? 2 * q + 1 : e);
                    }
                }
                // lanes 0..24 hold the eobs: DPP sums per 16-lane row, rows 0 and 1 added
                const int r16 = red16(e);
                const int es = __builtin_amdgcn_readlane(r16, 0) + __builtin_amdgcn_readlane(r16, 16);
                if (lane == 0)
                    a.sizes[(size_t)C.f * nmb + (size_t)C.mby * mbw + C.mbx] = (uint32_t)(1 + (lm == 4 ? 8 : 0) + 25 + 2 * es);
            }
        } else {
            write_levels(C, 0, 17, false);
            if (lane == 0) o->skip = 0;  // pass-1 skip is decided on the host from the levels
        }
        if (lane == 0) {
            o->luma_mode = (uint8_t)lm;
            o->segment = (uint8_t)C.seg;
        }
        if (lane < 16) o->bpred[lane] = lm == 4 ? C.M->modes[lane] : 0;
        store_luma_borders(C);
    };
    if constexpr (PAIR) {
        // ---- frame pairs: every wave works MB row y of both frames of the
        // workgroup (the rows of a frame go to the waves as in the one-frame
        // kernel), MB (x, y) of frame 0 and of frame 1 per iteration.  Both
        // frames' rows advance together, so one progress word per wave serves
        // both.  The two MBs' I4 searches run in one wave (pick_i4_pair): lanes
        // 0..31 frame 0, lanes 32..63 frame 1.  The other per-MB stages run in
        // loops over the frames (not unrolled: one copy of their code), and what
        // an MB's stages hand on goes through LDS (W->pst), not registers.
        MbLds* const Mp[2] = {&W->mb, Mall2 + wv};
        const int meth0 = C.method;
        const int K = C.method <= 3 ? 3 : (C.method == 4 ? 4 : 10);
        // per-frame encoder settings (a launch's frames normally share them)
        const int meth1 = nf == 2 ? __builtin_amdgcn_readfirstlane(a.params[f + 1].method) : C.method;
        const bool trel1 = PASS == 2 && nf == 2 && __builtin_amdgcn_readfirstlane(a.params[f + 1].do_trellis);
        const bool keep1 = !trel1 && (PASS == 1 || a.dbg == nullptr);
        // the luma waves (pass 1: after the chain waves) take the rows in turn
        constexpr int NL = NW - NCW;
        const bool same_k = nf == 1 || (meth1 == C.method && trel1 == trel);
        for (int it = 0;; it++) {
            const int mby = (wv - NCW) + it * NL;
            if (mby >= mbh) break;
#pragma unroll
            for (int fr = 0; fr < 2; fr++) {
                MbLds* M = Mp[fr];
                if (lane < 20) M->left_y[lane] = 129;
                if (lane < 12) {
                    M->left_u[lane] = M->left_v[lane] = 129;
                    M->left_c[lane] = 0;
                }
                if (lane < 4) M->left_derr[lane] = 0;
            }
            wsync();
            const int prevw = mby > 0 ? NCW + (mby - 1) % NL : 0;
            auto wait_above = [&](int need) {
                if (mby > 0) wait_row(progress, prevw, (mby - 1) * 65536 + need);
            };
            for (int mbx = 0; mbx < mbw; mbx++) {
                PH_START();
                const int lane = opaque_lane(threadIdx.x & 63);
                C.lane = lane;
                // point C at frame fr's MB (x, y)
                auto enter = [&](int fr) {
                    // a fresh opaque lane per MB stage: lane-derived constants are
                    // recomputed, not held across the other frame's stages
                    C.lane = opaque_lane(threadIdx.x & 63);
                    C.f = f + fr;
                    C.P = a.params + C.f;
                    C.T = (const LdsTables*)((const uint8_t*)T + sT * fr);
                    C.Sl = (const ZwSegment*)((const uint8_t*)Sl + sS * fr);
                    C.top_y = top_y + TS.y * fr;
                    C.top_u = top_u + TS.u * fr;
                    C.top_v = top_v + TS.v * fr;
                    C.top_c = top_c + TS.c * fr;
                    C.top_derr = top_derr + TS.d * fr;
                    C.M = fr ? Mp[1] : Mp[0];
                    C.method = fr ? meth1 : meth0;
                    C.mbx = mbx;
                    C.mby = mby;
                    C.oy = mbx * 16;
                    C.oc = mbx * 8;
                    C.ocx = mbx * 12;
                    C.od = mbx * 4;
                    C.sY = C.M->sy;
                    C.sU = C.M->su;
                    C.sV = C.M->sv;
                };
                auto pst = [&](int fr, int k) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)W->pst[fr][k]); };
                wait_above(min(mbx + 1, mbw));
#if ZW_DYN_PRIO > 0
                {
                    int slack = mbw;
                    if (mby > 0) {
                        const int v = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(&progress[prevw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                        if ((v >> 16) == mby - 1) slack = (v & 0xffff) - mbx - 1;
                    }
                    constexpr int dp = PASS == 1 ? ZW_DYN_PRIO1 : ZW_DYN_PRIO;
                    const int pr_ = slack >= dp * 3 ? 3 : (slack >= dp * 2 ? 2 : (slack >= dp ? 1 : 0));
                    set_prio(PASS == 1 ? min(pr_, ZW_P1_LUMA_MAX) : pr_);
                }
#endif
                PH_MARK(0);
ZW_PAIR_LOOP
                for (int fr = 0; fr < 2; fr++) {
                    if (fr >= nf) {
                        if (lane == 0) W->pst[fr][0] = 0;  // (no frame 1: no search)
                        continue;
                    }
                    enter(fr);
                    const MbFetch fm = fetch_mb(&a, C.f, lane, mbx, mby);
                    setup_ctx(C, &a, seg_lut + 256 * fr, W, mbx, mby, fm);
                    build_luma_border(C, 0);
                    int l_;
                    unsigned long long s_;
                    pick_i16<PASS>(C, l_, s_);
                    const bool n_ = C.method > 1 && (C.method >= 5 || s_ > 211ull * C.S->l_mode || l_ != 0);
                    if (lane == 0) {
                        W->pst[fr][0] = (uint32_t)l_ | ((uint32_t)n_ << 4) | ((uint32_t)C.seg << 8);
                        W->pst[fr][1] = (uint32_t)s_;
                        W->pst[fr][2] = (uint32_t)(s_ >> 32);
                        W->pst[fr][3] = 0;
                    }
                    wsync();
                }
                wsync();
                PH_MARK(1);
                const uint32_t s0 = pst(0, 0), s1 = pst(1, 0);
                const bool n0 = (s0 >> 4) & 1u, n1 = (s1 >> 4) & 1u;
                if (n0 || n1) wait_above(min(mbx + 2, mbw));
ZW_PAIR_LOOP
                for (int fr = 0; fr < 2; fr++) {
                    if (!((pst(fr, 0) >> 4) & 1u)) continue;
                    enter(fr);
                    build_luma_border(C, 1);
                }
                PH_MARK(21);
                if (K <= 4 && same_k && (n0 || n1)) {
                    Ctx CA = C, CB = C;
                    CA.lane = CB.lane = opaque_lane(threadIdx.x & 63);
                    CA.T = T;
                    CB.T = (const LdsTables*)((const uint8_t*)T + sT);
                    CA.M = Mp[0];
                    CB.M = Mp[1];
                    CA.S = Sl + (s0 >> 8);
                    CB.S = (const ZwSegment*)((const uint8_t*)Sl + sS) + (s1 >> 8);
                    CA.sY = Mp[0]->sy;
                    CB.sY = Mp[1]->sy;
                    const unsigned long long i0 = pst(0, 1) | ((unsigned long long)pst(0, 2) << 32);
                    const unsigned long long i1 = pst(1, 1) | ((unsigned long long)pst(1, 2) << 32);
                    uint32_t z0 = 0, z1 = 0;
                    const uint32_t r = pick_i4_pair<PASS>(CA, CB, i0, i1, n0, n1, keep_i4, z0, z1);
                    if (lane == 0) {
                        W->pst[0][3] = (r & 1u) ? (z0 | 0x10000u) : 0u;
                        W->pst[1][3] = (r & 2u) ? (z1 | 0x10000u) : 0u;
                    }
                } else if (n0 || n1) {
ZW_PAIR_LOOP
                    for (int fr = 0; fr < 2; fr++) {
                        const uint32_t sm = pst(fr, 0);
                        if (!((sm >> 4) & 1u)) continue;
                        enter(fr);
                        C.seg = (int)(sm >> 8);
                        C.S = C.Sl + C.seg;
                        uint32_t z = 0;
                        const bool w4 = pick_i4<PASS>(C, pst(fr, 1) | ((unsigned long long)pst(fr, 2) << 32),
                                                      fr ? keep1 : keep_i4, z);
                        if (lane == 0) W->pst[fr][3] = w4 ? (z | 0x10000u) : 0u;
                    }
                }
                wsync();
                PH_MARK(2);
ZW_PAIR_LOOP
                for (int fr = 0; fr < 2; fr++) {
                    if (fr >= nf) continue;
                    enter(fr);
                    const uint32_t sm = pst(fr, 0), r4 = pst(fr, 3);
                    C.seg = (int)(sm >> 8);
                    C.S = C.Sl + C.seg;
                    int cm = 0;  // (pass 1: the chain waves work the chroma)
                    if (PASS == 2) {
                        build_chroma_border(C);
                        cm = pick_uv<PASS>(C);
                    }
                    PH_MARK(3);
                    const bool w4 = (r4 >> 16) & 1u;
                    mb_store(C, w4 ? 4 : (int)(sm & 15u), cm, w4 && (fr ? keep1 : keep_i4), r4 & 0xffffu,
                             fr ? trel1 : trel);
                    PH_RESET();
                }
                publish(progress, wv, mby * 65536 + mbx + 1);
                PH_MARK(6);
            }
        }
        ph_flush();
        return;
    }
    uint8_t* const gty = ROWS ? rb + RL.ty : nullptr;
    uint8_t* const gtu = ROWS ? rb + RL.tu : nullptr;
    uint8_t* const gtv = ROWS ? rb + RL.tv : nullptr;
    uint8_t* const gtc = ROWS ? rb + RL.tc : nullptr;
    uint8_t* const gtd = ROWS ? rb + RL.td : nullptr;
    for (int it = 0, yk = rw;; it++) {
        const int mby = ROWS ? row_ticket(&rsync[0]) : (skip_mode ? yk : rw + it * nrw);
        if (skip_mode) yk = next_row(yk);
        if (mby >= mbh) break;
        if (lane < 20) C.M->left_y[lane] = 129;
        if (lane < 12) {
            C.M->left_u[lane] = 129;
            C.M->left_v[lane] = 129;
            C.M->left_c[lane] = 0;
        }
        if (lane < 4) C.M->left_derr[lane] = 0;
        wsync();
        const int prevw = (!ROWS && mby > 0) ? wave_of_row(mby - 1) : 0;
        int seen = -1;  // ROWS: last progress value read of the row above
        int* const prog_above = ROWS ? rsync + 4 + (mby > 0 ? mby - 1 : 0) : nullptr;
        // the row above has finished `need` MBs
        auto wait_above = [&](int need) {
            if (mby == 0) return;
            if (ROWS) row_wait(prog_above, need, rerr, seen);
            else wait_row(progress, prevw, (mby - 1) * 65536 + need);
        };
#ifndef ZW_FETCH_AHEAD
#define ZW_FETCH_AHEAD (PASS == 2)
#endif
        // Pass 1 loads the MB's source words and alpha at the top of its
        // iteration, in flight during the wait for the row above; pass 2 fetches
        // them one MB ahead.  (Fetched ahead, the words do not stay in registers:
        // each is spilled to scratch right after its load, so the three loads
        // run one after another, each also waiting for the previous MB's stores
        // -- vmcnt counts stores.  Measured per 256 1080p frames: pass 1 29.12 ->
        // 28.98 ms loading at the top, pass 2 37.38 -> 37.64 ms.)
        MbFetch nx;
        if (ZW_FETCH_AHEAD) nx = fetch_mb(&a, f, lane, 0, mby);
        for (int mbx = 0; mbx < mbw; mbx++) {
            PH_START();
            const int lane = opaque_lane(threadIdx.x & 63);
            C.lane = lane;
            MbFetch cur;
            if (ZW_FETCH_AHEAD) {
                cur = nx;
                if (mbx + 1 < mbw) nx = fetch_mb(&a, f, lane, mbx + 1, mby);
            } else {
                cur = fetch_mb(&a, f, lane, mbx, mby);
            }
            // the I16 and chroma searches need only the MB above (x, y-1); the
            // I4 search also reads the above-right MB's bottom row: wait for
            // (x+1, y-1) only then, so the wait overlaps the first searches
            wait_above(min(mbx + 1, mbw));
            if (ROWS) {
                // pull this MB's slice of the row above's state into the window
                if (mby > 0) {
                    uint32_t v = 0;
                    if (lane < 4) v = ld_sc1(gty + mbx * 16 + 4 * lane);
                    else if (PASS == 2 && lane < 6) v = ld_sc1(gtu + mbx * 8 + 4 * (lane - 4));
                    else if (PASS == 2 && lane < 8) v = ld_sc1(gtv + mbx * 8 + 4 * (lane - 6));
                    else if (PASS == 2 && lane < 11) v = ld_sc1(gtc + mbx * 12 + 4 * (lane - 8));
                    else if (PASS == 2 && lane < 12) v = ld_sc1(gtd + mbx * 4);
                    if (lane < 4) ((uint32_t*)W->win_y)[lane] = v;
                    else if (PASS == 2 && lane < 6) ((uint32_t*)W->win_u)[lane - 4] = v;
                    else if (PASS == 2 && lane < 8) ((uint32_t*)W->win_v)[lane - 6] = v;
                    else if (PASS == 2 && lane < 11) ((uint32_t*)W->win_c)[lane - 8] = v;
                    else if (PASS == 2 && lane < 12) ((uint32_t*)W->win_d)[0] = v;
                } else if (PASS == 2) {
                    // row 0: zero contexts; top_derr from pass 1 (quirk A6)
                    if (lane < 3) ((uint32_t*)W->win_c)[lane] = 0;
                    else if (lane == 3)
                        ((uint32_t*)W->win_d)[0] = *(const uint32_t*)(a.derr + (size_t)f * mbw * 4 + mbx * 4);
                }
                wsync();
            } else {
                C.oy = mbx * 16;
                C.oc = mbx * 8;
                C.ocx = mbx * 12;
                C.od = mbx * 4;
            }
#if ZW_DYN_PRIO > 0
            if (!ROWS) {
                // Issue priority from the slack to the row above.  VALU issue is
                // arbitrated by priority, then wave age: at equal priority the
                // youngest waves of each SIMD run slowest and every row behind
                // theirs waits on them (35 % of the oldest waves' time).  A row
                // that trails the row above by more than the two-MB minimum is
                // the one later rows wait for, so it issues first.
                int slack = mbw;
                if (mby > 0) {
                    const int v = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&progress[prevw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    if ((v >> 16) == mby - 1) slack = (v & 0xffff) - mbx - 1;
                }
                constexpr int dp = PASS == 1 ? ZW_DYN_PRIO1 : ZW_DYN_PRIO;
                const int p = slack >= dp * 3 ? 3 : (slack >= dp * 2 ? 2 : (slack >= dp ? 1 : 0));
                set_prio(PASS == 1 ? min(p, ZW_P1_LUMA_MAX) : p);
            }
#endif
            PH_MARK(0);
            setup_ctx(C, &a, seg_lut, W, mbx, mby, cur);
            build_luma_border(C, 0);
            int lm;
            unsigned long long i16s;
            pick_i16<PASS>(C, lm, i16s);
            wsync();
            PH_MARK(1);
            int cm = 0;
            uint32_t i4nz = 0;
            bool i4reuse = false;
            if (PASS == 2) {
                build_chroma_border(C);
                cm = pick_uv<PASS>(C);
            }
            PH_MARK(3);
            if (C.method > 1) {
                const unsigned long long thr = 211ull * C.S->l_mode;
                if (C.method >= 5 || i16s > thr || lm != 0) {
                    wait_above(min(mbx + 2, mbw));
                    if (ROWS && mby > 0 && mbx + 1 < mbw) {
                        // the above-right MB's bottom row
                        uint32_t v = 0;
                        if (lane < 4) v = ld_sc1(gty + (mbx + 1) * 16 + 4 * lane);
                        if (lane < 4) ((uint32_t*)W->win_y)[4 + lane] = v;
                        wsync();
                    }
                    build_luma_border(C, 1);
                    PH_MARK(21);
                    if (pick_i4<PASS>(C, i16s, keep_i4, i4nz)) {
                        lm = 4;
                        i4reuse = keep_i4;
                    }
                }
            }
            PH_MARK(2);
            mb_store(C, lm, cm, i4reuse, i4nz, trel);
            PH_RESET();
            if (ROWS) {
                // push this MB's state for the row below (sc1), then publish
                if (mby + 1 < mbh) {
                    if (lane < 4) st_sc1(gty + mbx * 16 + 4 * lane, ((const uint32_t*)W->win_y)[lane]);
                    else if (PASS == 2 && lane < 6) st_sc1(gtu + mbx * 8 + 4 * (lane - 4), ((const uint32_t*)W->win_u)[lane - 4]);
                    else if (PASS == 2 && lane < 8) st_sc1(gtv + mbx * 8 + 4 * (lane - 6), ((const uint32_t*)W->win_v)[lane - 6]);
                    else if (PASS == 2 && lane < 11) st_sc1(gtc + mbx * 12 + 4 * (lane - 8), ((const uint32_t*)W->win_c)[lane - 8]);
                    else if (PASS == 2 && lane < 12) st_sc1(gtd + mbx * 4, ((const uint32_t*)W->win_d)[0]);
                    row_publish(rsync + 4 + mby, mbx + 1);
                }
            } else {
                publish(progress, wv, mby * 65536 + mbx + 1);
            }
            PH_MARK(6);
        }
    }
    ph_flush();
}

extern "C" __global__ __launch_bounds__(PassShape<1>::WG) void k_encode_pass1(EncArgs a) { encode_body<1, false>(a); }
extern "C" __global__ __launch_bounds__(PassShape<1>::WG) void k_encode_pass1_fp(EncArgs a) { encode_body<1, false, 2>(a); }
extern "C" __global__ __launch_bounds__(PassShape<2>::WG) void k_encode_pass2(EncArgs a) { encode_body<2, false>(a); }
extern "C" __global__ __launch_bounds__(PassShape<2>::WG) void k_encode_pass2_fp(EncArgs a) { encode_body<2, false, 2>(a); }
extern "C" __global__ __launch_bounds__(64 * RowsShape<1>::NW) void k_encode_rows_pass1(EncArgs a) { encode_body<1, true>(a); }
extern "C" __global__ __launch_bounds__(64) void k_encode_rows_pass2(EncArgs a) { encode_body<2, true>(a); }

// ---------------------------------------------------------------------------
// Kernel-level entry: quantisation (simple or trellis) of independent 4x4
// coefficient blocks, one block per thread (quantize_coeff cost.rs:457,
// trellis_quantize_block cost.rs:788).  Used by the parity tests and as the
// building block the encoder kernels share.
// ---------------------------------------------------------------------------
struct QuantBlocksArgs {
    ZwMatrix m;
    uint16_t sharpen[16];
    uint32_t lambda;
    int32_t ctype, first, trel, n;
};

extern "C" __global__ __launch_bounds__(256) void k_quant_blocks(const int* __restrict__ coeffs,
                                                                const uint8_t* __restrict__ ctx0s,
                                                                const ZwLevelCosts* __restrict__ lcost,
                                                                const uint8_t* __restrict__ probs, QuantBlocksArgs a,
                                                                int* __restrict__ levels, int* __restrict__ dq)
{
    __shared__ LdsTables T;
    for (int i = threadIdx.x; i < (int)(sizeof(T.lc) / 2); i += 256) (&T.lc[0][0][0][0])[i] = (&lcost->lc[0][0][0][0])[i];
    for (int i = threadIdx.x; i < 96; i += 256) {
        (&T.eob[0][0][0])[i] = (&lcost->eob[0][0][0])[i];
        (&T.init[0][0][0])[i] = (&lcost->init[0][0][0])[i];
    }
    for (int i = threadIdx.x; i < 4 * 8 * 3 * 11; i += 256) (&T.probs[0][0][0][0])[i] = probs[i];
    load_static_tables(&T, threadIdx.x, 256, probs);
    __syncthreads();
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= a.n) return;
    int c[16], lv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) c[k] = coeffs[(size_t)b * 16 + k];
    const int ctx0 = ctx0s[b];
    if (a.trel) {
        if (a.first) trellis<1>(c, lv, a.m, a.sharpen, a.lambda, &T, a.ctype, ctx0);
        else trellis<0>(c, lv, a.m, a.sharpen, a.lambda, &T, a.ctype, ctx0);
        if (a.first) lv[0] = 0;
    } else {
#pragma unroll
        for (int n = 0; n < 16; n++) {
            const int j = kZZ(n);
            lv[n] = n < a.first ? 0 : quantz(c[j], a.m.iq[j > 0], a.m.bias[j > 0]);
        }
#pragma unroll
        for (int n = 0; n < 16; n++) {
            const int j = kZZ(n);
            c[j] = n < a.first ? 0 : m24(lv[n], (int)a.m.q[j > 0]);
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        levels[(size_t)b * 16 + k] = lv[k];
        dq[(size_t)b * 16 + k] = c[k];
    }
}

// The lane-parallel trellis (trellis_g, used by the final I4 pass): 16 lanes
// per block, lane = zigzag position.
extern "C" __global__ __launch_bounds__(256) void k_quant_blocks_g(const int* __restrict__ coeffs,
                                                                  const uint8_t* __restrict__ ctx0s,
                                                                  const ZwLevelCosts* __restrict__ lcost,
                                                                  const uint8_t* __restrict__ probs, QuantBlocksArgs a,
                                                                  int* __restrict__ levels, int* __restrict__ dq)
{
    __shared__ LdsTables T;
    for (int i = threadIdx.x; i < (int)(sizeof(T.lc) / 2); i += 256) (&T.lc[0][0][0][0])[i] = (&lcost->lc[0][0][0][0])[i];
    for (int i = threadIdx.x; i < 96; i += 256) {
        (&T.eob[0][0][0])[i] = (&lcost->eob[0][0][0])[i];
        (&T.init[0][0][0])[i] = (&lcost->init[0][0][0])[i];
    }
    for (int i = threadIdx.x; i < 4 * 8 * 3 * 11; i += 256) (&T.probs[0][0][0][0])[i] = probs[i];
    load_static_tables(&T, threadIdx.x, 256, probs);
    __syncthreads();
    const int b = (int)((blockIdx.x * 256 + threadIdx.x) >> 4), n = threadIdx.x & 15;
    const int bb = min(b, a.n - 1);  // whole groups stay active (DPP/ballot need every lane)
    const int cn = coeffs[(size_t)bb * 16 + zz_of(n)];
    const int ctx0 = ctx0s[bb];
    int lvl;
    if (a.first) (void)trellis_g<1>(cn, n, a.m, a.sharpen, a.lambda, &T, a.ctype, ctx0, lvl);
    else (void)trellis_g<0>(cn, n, a.m, a.sharpen, a.lambda, &T, a.ctype, ctx0, lvl);
    if (b < a.n) {
        const int j = zz_of(n);
        levels[(size_t)b * 16 + n] = lvl;
        // positions before `first` keep their input coefficient (as trellis<1> leaves coeffs[0])
        dq[(size_t)b * 16 + j] = n < a.first ? cn : lvl * (int)(j == 0 ? a.m.q[0] : a.m.q[1]);
    }
}

extern "C" hipError_t zwk_quant_blocks(hipStream_t s, const int* coeffs, const uint8_t* ctx0s, const ZwLevelCosts* lcost,
                                       const uint8_t* probs, const void* args, int* levels, int* dq)
{
    const QuantBlocksArgs& a = *(const QuantBlocksArgs*)args;
    if (a.trel == 2)
        hipLaunchKernelGGL(k_quant_blocks_g, dim3((a.n * 16 + 255) / 256), dim3(256), 0, s, coeffs, ctx0s, lcost, probs,
                           a, levels, dq);
    else
        hipLaunchKernelGGL(k_quant_blocks, dim3((a.n + 255) / 256), dim3(256), 0, s, coeffs, ctx0s, lcost, probs, a,
                           levels, dq);
    return hipGetLastError();
}

static size_t encode_lds_bytes(int mbw, int nw, bool rows, int pass, int fp = 1)
{
    size_t off = 0;
    off += ((sizeof(LdsTables) + 15) & ~(size_t)15) * fp;
    off += ((4 * sizeof(ZwSegment) + 15) & ~(size_t)15) * fp;
    off += 256 * fp;
    off += ((sizeof(WaveLds) + 15) & ~(size_t)15) * nw;
    if (fp == 2) off += ((sizeof(MbLds) + 15) & ~(size_t)15) * nw;
    off += 64;
    off += 256;
    const TopLds t(mbw, rows, pass);
    return off + (t.y + t.u + t.v + t.c + t.d) * fp;
}

// Frame pairs (k_encode_pass1_fp / k_encode_pass2_fp) for launches of at
// least two frames per CU whose pair shape fits in LDS; ZW_ENC_FP=0/1 forces
// them off/on (where they fit), ZW_ENC_FP1 the same for pass 1 alone.
static bool encode_fp_for(int pass, int mbw, int nframes)
{
    static const int mode2 = [] { const char* e = getenv("ZW_ENC_FP"); return e && *e ? atoi(e) : -1; }();
    static const int mode1 = [] { const char* e = getenv("ZW_ENC_FP1"); return e && *e ? atoi(e) : mode2; }();
    const int mode = pass == 1 ? mode1 : mode2;
    static const int cus = [] {
        int dev = 0;
        hipDeviceProp_t prop;
        return hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess &&
                       prop.multiProcessorCount > 0
                   ? prop.multiProcessorCount
                   : 256;
    }();
    if (mode == 0 || nframes < 2) return false;
    if (encode_lds_bytes(mbw, pass == 1 ? PassShape<1>::NW : PassShape<2>::NW, false, pass, 2) > 160 * 1024) return false;
    return mode == 1 || nframes >= 2 * cus;
}
extern "C" int zwk_encode_fp(int pass, int mbw, int nframes) { return encode_fp_for(pass, mbw, nframes) ? 1 : 0; }


// ---------------------------------------------------------------------------
// Host-side launch wrappers (called from zw_host.cpp).
// ---------------------------------------------------------------------------
extern "C" hipError_t zwk_rgb2yuv(hipStream_t s, const uint8_t* img, int w, int h, int bpp, int mbw, int mbh,
                                  uint8_t* Y, uint8_t* U, uint8_t* V, size_t img_stride, size_t ysz, size_t csz,
                                  int nframes)
{
    // the row-coalesced kernel needs every 8-pixel run aligned for its loads
    // (16 B for RGBA, 8 B for RGB) and 8-byte aligned luma rows
    const uintptr_t base = (uintptr_t)img;
    const bool planes_ok = ((uintptr_t)Y | (uintptr_t)U | (uintptr_t)V | ysz | csz) % 8 == 0;
    const int ng = mbw * 2 * mbh * 8;
    if (planes_ok && bpp == 4 && base % 16 == 0 && img_stride % 16 == 0 && w % 4 == 0) {
        hipLaunchKernelGGL(k_rgb2yuv_rows<4>, dim3((ng + 255) / 256, nframes), dim3(256), 0, s, img, w, h, mbw, mbh,
                           Y, U, V, img_stride, ysz, csz);
    } else if (planes_ok && bpp == 3 && base % 8 == 0 && img_stride % 8 == 0 && w % 8 == 0) {
        hipLaunchKernelGGL(k_rgb2yuv_rows<3>, dim3((ng + 255) / 256, nframes), dim3(256), 0, s, img, w, h, mbw, mbh,
                           Y, U, V, img_stride, ysz, csz);
    } else {
        const int n = mbw * 8 * mbh * 8;
        hipLaunchKernelGGL(k_rgb2yuv, dim3((n + 255) / 256, nframes), dim3(256), 0, s, img, w, h, bpp, mbw, mbh, Y, U,
                           V, img_stride, ysz, csz);
    }
    return hipGetLastError();
}

extern "C" hipError_t zwk_analysis(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, int mbw,
                                   int mbh, size_t ysz, size_t csz, uint8_t* alpha, uint32_t* histo, int nframes)
{
    const int nmb = mbw * mbh;
#ifndef ZW_AN_FORM
#define ZW_AN_FORM 4  // 4: k_analysis4 (four MBs a wave); 1: k_analysis (one MB a wave)
#endif
    if (ZW_AN_FORM == 4)
        hipLaunchKernelGGL(k_analysis4, dim3((nmb + 16 * ZW_AN4_GPW - 1) / (16 * ZW_AN4_GPW), nframes), dim3(256), 0, s, Y,
                           U, V, mbw, mbh, ysz, csz, alpha, histo);
    else
        hipLaunchKernelGGL(k_analysis, dim3((nmb + 4 * ZW_AN_MPW - 1) / (4 * ZW_AN_MPW), nframes), dim3(256), 0, s, Y, U,
                           V, mbw, mbh, ysz, csz, alpha, histo);
    return hipGetLastError();
}

extern "C" hipError_t zwk_segments(hipStream_t s, uint32_t* histo, const ZwFrameParams* tmpl,
                                   ZwFrameParams* params, int nframes)
{
    hipLaunchKernelGGL(k_segments, dim3((nframes + 63) / 64), dim3(64), 0, s, histo, tmpl, params, nframes);
    return hipGetLastError();
}

// The widest frame (in MBs) whose LDS fits the 160 KiB of a CU in the batch
// shapes (rows = false: every row array of the frame in LDS) or in the
// row-parallel shapes (rows = true: only pass 1's chroma chain keeps rows).
// encode_frame_lossy takes any u16 width (vp8.rs:3143-3148): 4 096 MBs, which
// the row-parallel kernels hold; wider frames than the batch shapes take go to them.
extern "C" int zwk_encode_max_mbw(int rows)
{
    int lo = 1, hi = 65536 / 16;
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        const bool ok = rows ? encode_lds_bytes(mid, RowsShape<1>::NW, true, 1) <= 160 * 1024 &&
                                   encode_lds_bytes(mid, RowsShape<2>::NW, true, 2) <= 160 * 1024
                             : encode_lds_bytes(mid, PassShape<1>::NW, false, 1) <= 160 * 1024 &&
                                   encode_lds_bytes(mid, PassShape<2>::NW, false, 2) <= 160 * 1024;
        if (ok) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Bytes of zero-filled scratch the row-parallel kernels need for nframes frames.
extern "C" size_t zwk_encode_rows_bytes(int mbw, int mbh, int nframes)
{
    return ZW_ROWS_HDR + (size_t)nframes * RowsLayout(mbw, mbh).frame;
}

// rows: null -> one 12-wave workgroup per frame (batches); otherwise the
// row-parallel kernels with that zero-filled scratch (zwk_encode_rows_bytes).
extern "C" hipError_t zwk_encode(hipStream_t s, int pass, const uint8_t* Y, const uint8_t* U, const uint8_t* V,
                                 const uint8_t* alpha, const ZwFrameParams* params, const ZwLevelCosts* lcost,
                                 int8_t* derr, ZwMbOut* out, uint8_t* ry, uint8_t* ru, uint8_t* rv, size_t ysz,
                                 size_t csz, int mbw, int mbh, int nframes, int* dbg, uint8_t* rows, uint32_t* sizes)
{
    EncArgs a;
    a.dbg = dbg;
    a.sizes = pass == 2 ? sizes : nullptr;
    a.Y = Y; a.U = U; a.V = V; a.alpha = alpha; a.params = params; a.lcost = lcost; a.derr = derr; a.out = out;
    a.ry = ry; a.ru = ru; a.rv = rv; a.ysz = ysz; a.csz = csz; a.mbw = mbw; a.mbh = mbh; a.pass = pass;
    a.rows = rows;
    a.nframes = nframes;
    static const bool attr_set = []() {
        (void)hipFuncSetAttribute((const void*)k_encode_pass1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode_pass2, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode_pass2_fp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode_pass1_fp, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode_rows_pass1, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_encode_rows_pass2, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr_set;
    if (rows) {
        // one wave per MB row (+ pass 1's chroma chain in workgroup 0)
        if (pass == 1) {
            constexpr int nw = RowsShape<1>::NW;
            hipLaunchKernelGGL(k_encode_rows_pass1, dim3(1 + (mbh + nw - 1) / nw, nframes), dim3(64 * nw),
                               encode_lds_bytes(mbw, nw, true, 1), s, a);
        } else {
            hipLaunchKernelGGL(k_encode_rows_pass2, dim3(mbh, nframes), dim3(64), encode_lds_bytes(mbw, 1, true, 2), s,
                               a);
        }
        return hipGetLastError();
    }
    if (encode_fp_for(pass, mbw, nframes)) {
        if (pass == 1)
            hipLaunchKernelGGL(k_encode_pass1_fp, dim3((nframes + 1) / 2), dim3(PassShape<1>::WG),
                               encode_lds_bytes(mbw, PassShape<1>::NW, false, 1, 2), s, a);
        else
            hipLaunchKernelGGL(k_encode_pass2_fp, dim3((nframes + 1) / 2), dim3(PassShape<2>::WG),
                               encode_lds_bytes(mbw, PassShape<2>::NW, false, 2, 2), s, a);
        return hipGetLastError();
    }
    const size_t lds = encode_lds_bytes(mbw, pass == 1 ? PassShape<1>::NW : PassShape<2>::NW, false, pass);
    if (pass == 1) hipLaunchKernelGGL(k_encode_pass1, dim3(nframes), dim3(PassShape<1>::WG), lds, s, a);
    else hipLaunchKernelGGL(k_encode_pass2, dim3(nframes), dim3(PassShape<2>::WG), lds, s, a);
    return hipGetLastError();
}
