// zw_dev.h -- device-side helpers shared by the HIP kernels: constant tables,
// exact integer transforms, quantizer, residual cost and trellis.  Every
// function restates the reference function named in its comment; the HIP
// kernels compose them per macroblock.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "zw_common.h"

#define ZW_TABLE(T, N, D, ...) __constant__ T d_##N D = {__VA_ARGS__};
#include "zw_tables.inc"
#undef ZW_TABLE

// (mode, pixel) -> index into the I4 value vector (tools/gen_i4_table.py);
// 255 = DC, 254 = TM.  Value vector: E = [L3 L2 L1 L0 P A0..A7], then
// avg3 of consecutive triples (13..23), avg2 of pairs (24..35),
// avg3(A6,A7,A7) (36), avg3(L2,L3,L3) (37).
__constant__ uint8_t d_I4_IDX[10][16] = {
    {255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255},
    {254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254, 254},
    {17, 18, 19, 20, 17, 18, 19, 20, 17, 18, 19, 20, 17, 18, 19, 20},
    {15, 15, 15, 15, 14, 14, 14, 14, 13, 13, 13, 13, 37, 37, 37, 37},
    {18, 19, 20, 21, 19, 20, 21, 22, 20, 21, 22, 23, 21, 22, 23, 36},
    {16, 17, 18, 19, 15, 16, 17, 18, 14, 15, 16, 17, 13, 14, 15, 16},
    {28, 29, 30, 31, 16, 17, 18, 19, 15, 28, 29, 30, 14, 16, 17, 18},
    {29, 30, 31, 32, 18, 19, 20, 21, 30, 31, 32, 22, 19, 20, 21, 23},
    {27, 16, 17, 18, 26, 15, 27, 16, 25, 14, 26, 15, 24, 13, 25, 14},
    {26, 14, 25, 13, 25, 13, 24, 37, 24, 37, 0, 0, 0, 0, 0, 0},
};

#define DI __device__ __forceinline__

// Small position tables as 64-bit immediates: with a constant index they fold,
// with a dynamic one (a loop the compiler kept rolled) they are a shift -- never
// a load from constant memory.
DI int kZZ(int n) { return (int)((0xfeb7adc963258410ull >> (4 * n)) & 15); }  // ZIGZAG
DI int kBand(int n)  // VP8_ENC_BANDS[n], n in 0..16
{
    return n >= 16 ? 0 : (int)((0x7666666665463210ull >> (4 * n)) & 15);
}
DI int kWTrellis(int j)  // VP8_WEIGHT_TRELLIS {30,27,19,11,27,24,17,10,19,17,12,8,11,10,8,6}
{
    const unsigned long long lo = 0x0a11181b0b131b1eull, hi = 0x06080a0b080c1113ull;
    return (int)(((j < 8 ? lo : hi) >> (8 * (j & 7))) & 255);
}
DI int kWY(int j)  // kWeightY {38,32,20,9,32,28,17,7,20,17,10,4,9,7,4,2}
{
    const unsigned long long lo = 0x07111c2009142026ull, hi = 0x02040709040a1114ull;
    return (int)(((j < 8 ? lo : hi) >> (8 * (j & 7))) & 255);
}

// Small position tables packed 4 bits per entry into 64-bit immediates: a
// lane-varying index becomes one 64-bit shift (no memory access, no branches).
DI int band_of(int n)  // VP8_ENC_BANDS[n], n in 0..16
{
    return n >= 16 ? 0 : (int)((0x7666666665463210ull >> (4 * n)) & 15);
}
DI int zz_of(int n) { return (int)((0xfeb7adc963258410ull >> (4 * n)) & 15); }   // ZIGZAG
DI int izz_of(int k) { return (int)((0xfea9db83c7426510ull >> (4 * k)) & 15); }  // inverse ZIGZAG

DI int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
DI int iabs(int v) { return v < 0 ? -v : v; }

// rgb_to_y / the raw U and V sums of yuv.rs:859-896 on a pixel word 0x..BBGGRR
// (U/V: the 2x2 sum of these + (512 << 16), then (s + 2^17) >> 18)
__device__ __forceinline__ int pk_y(uint32_t p)
{
    return (16839 * (int)(p & 255u) + 33059 * (int)((p >> 8) & 255u) + 6420 * (int)((p >> 16) & 255u) + (1 << 15) +
            (16 << 16)) >> 16;
}
__device__ __forceinline__ int pk_u(uint32_t p)
{
    return -9719 * (int)(p & 255u) - 19081 * (int)((p >> 8) & 255u) + 28800 * (int)((p >> 16) & 255u);
}
__device__ __forceinline__ int pk_v(uint32_t p)
{
    return 28800 * (int)(p & 255u) - 24116 * (int)((p >> 8) & 255u) - 4684 * (int)((p >> 16) & 255u);
}
// The same sums by 16-bit dot products (identical integers): Y from the (R, G)
// pair of the pixel word by one v_dot2_u32_u16 plus 6420 B; the 2x2 U / V sums
// from the four pixels' (R, B) pairs and G added first (packed u16 adds, at
// most 1 020 each), then one v_dot2_i32_i16 and one multiply-add per plane.
__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t d;
    asm("v_dot2_u32_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ int sdot2(uint32_t a, uint32_t b, int c)
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t pk_y2(uint32_t p)
{
    const uint32_t rg = __builtin_amdgcn_perm(0u, p, 0x0c010c00u);  // (R, G)
    return udot2(rg, 0x812341c7u /* (16839, 33059) */, ((p >> 16) & 255u) * 6420u + (1u << 15) + (16u << 16)) >> 16;
}
// Y of four pixels (0x..BBGGRR words) as one packed word.  Each coefficient
// split into high and low bytes (16839 = 65:199, 33059 = 129:35, 6420 = 25:20)
// makes the sum two v_dot4_u32_u8 and a shift-add; it stays below 2^24, so the
// Y byte is byte 2 of it and two v_perm gather the four (equal to pk_y for
// every (R, G, B): checked exhaustively).
__device__ __forceinline__ uint32_t pk_y4(uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3)
{
    auto y = [](uint32_t p) {
        const uint32_t hi = __builtin_amdgcn_udot4(p, 0x00198141u, 0u, false);
        const uint32_t lo = __builtin_amdgcn_udot4(p, 0x001423c7u, (1u << 15) + (16u << 16), false);
        return (hi << 8) + lo;
    };
    const uint32_t lo = __builtin_amdgcn_perm(y(p1), y(p0), 0x0c0c0602u);  // Y0, Y1 in bytes 0, 1
    const uint32_t hi = __builtin_amdgcn_perm(y(p3), y(p2), 0x06020c0cu);  // Y2, Y3 in bytes 2, 3
    return lo | hi;
}
// (U, V) bytes of the 2x2 of pixels a, b (row 0) and c, d (row 1): (s + 2^17) >> 18
// of s = sum of pk_u / pk_v + (512 << 16)
__device__ __forceinline__ void pk_uv4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t& u, uint32_t& v)
{
    const uint32_t sel = 0x0c020c00u;  // (R, B)
    const uint32_t rb = __builtin_amdgcn_perm(0u, a, sel) + __builtin_amdgcn_perm(0u, b, sel) +
                        __builtin_amdgcn_perm(0u, c, sel) + __builtin_amdgcn_perm(0u, d, sel);
    const int g = (int)(((a >> 8) & 255u) + ((b >> 8) & 255u) + ((c >> 8) & 255u) + ((d >> 8) & 255u));
    const int su = sdot2(rb, 0x7080da09u /* (-9719, 28800) */, g * -19081 + (512 << 16));
    const int sv = sdot2(rb, 0xedb47080u /* (28800, -4684) */, g * -24116 + (512 << 16));
    u = (uint32_t)((su + (1 << 17)) >> 18);
    v = (uint32_t)((sv + (1 << 17)) >> 18);
}

// Intra-wave LDS hand-off: lanes of one wave exchange data through LDS.  A
// wave's DS instructions execute in issue order, so a wavefront-scope fence
// (compiler ordering only, no s_waitcnt on outstanding global stores) is all
// the hand-off needs.  Cross-wave hand-offs use release/acquire at workgroup
// scope (publish / wait_row).
DI void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Raw buffer loads / stores with a per-lane offset; ZW_OOB (past num_records)
// makes a lane's load return 0 and its store vanish.  The streaming kernels
// issue every global access of a step this way, unconditionally, so the number
// of memory operations between a prefetch and its use is the same on every
// path: the compiler then waits for the prefetch alone (vmcnt(N)) instead of
// vmcnt(0), which would also wait for the step's own stores.  The *nt forms
// set the nontemporal cache policy (CPol NT, bit 1).
#define ZW_OOB 0x80000000u
typedef uint32_t zu2 __attribute__((ext_vector_type(2)));
typedef uint32_t zu4 __attribute__((ext_vector_type(4)));
DI __amdgpu_buffer_rsrc_t brsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
DI uint32_t bld32(__amdgpu_buffer_rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0); }
DI zu2 bld64nt(__amdgpu_buffer_rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 2); }
DI zu4 bld128(__amdgpu_buffer_rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0); }
DI zu4 bld128nt(__amdgpu_buffer_rsrc_t r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 2); }
DI void bst8(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, (int)off, 0, 0); }
DI void bst32(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)off, 0, 0); }
DI void bst64(zu2 v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 0); }
DI void bst64nt(zu2 v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 2); }
DI void bst128(zu4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0); }
DI void bst128nt(zu4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) { __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 2); }

DI int wave_sum(int v)
{
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
DI long long shfl64(long long v, int src)
{
    int lo = __shfl((int)(v & 0xffffffff), src);
    int hi = __shfl((int)(v >> 32), src);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// 24-bit multiplies (full-rate v_mul_*_24 instead of quarter-rate v_mul_lo_u32).
// Every operand on these paths is below 2^23 in magnitude and every product
// fits in 32 bits, so the low 32 bits equal the plain int product.
DI int m24(int a, int b) { return __mul24(a, b); }

// VP8Matrix::quantize_coeff (cost.rs:457): sign * ((|c| * iq + bias) >> 17).
// |c| * iq < 2^31 for every coefficient an 8-bit source can produce.
DI int quantz(int c, uint32_t iq, uint32_t bias)
{
    uint32_t a = (uint32_t)iabs(c);
    int l = (int)((__umul24(a, iq) + bias) >> 17);
    return c < 0 ? -l : l;
}

// dct4x4_scalar (transform.rs:176).  For residuals in [-255,255] it equals the
// SSE2 build the reference ships (verified exhaustively in tests).
DI void fdct16(int* b)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a = (b[i * 4] + b[i * 4 + 3]) * 8, bb = (b[i * 4 + 1] + b[i * 4 + 2]) * 8;
        int c = (b[i * 4 + 1] - b[i * 4 + 2]) * 8, d = (b[i * 4] - b[i * 4 + 3]) * 8;
        b[i * 4] = a + bb;
        b[i * 4 + 2] = a - bb;
        b[i * 4 + 1] = (c * 2217 + d * 5352 + 14500) >> 12;
        b[i * 4 + 3] = (d * 2217 - c * 5352 + 7500) >> 12;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a = b[i] + b[i + 12], bb = b[i + 4] + b[i + 8];
        int c = b[i + 4] - b[i + 8], d = b[i] - b[i + 12];
        b[i] = (a + bb + 7) >> 4;
        b[i + 8] = (a - bb + 7) >> 4;
        b[i + 4] = ((c * 2217 + d * 5352 + 12000) >> 16) + (d != 0 ? 1 : 0);
        b[i + 12] = (d * 2217 - c * 5352 + 51000) >> 16;
    }
}

// idct4x4 in i32.  Equal to the reference's SSE2 i16 iDCT for every
// dequantized block the encoder produces (no i16 overflow is reachable).
DI void idct16(int* b)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a1 = b[i] + b[8 + i], b1 = b[i] - b[8 + i];
        int c1 = (m24(b[4 + i], 35468) >> 16) - (b[12 + i] + (m24(b[12 + i], 20091) >> 16));
        int d1 = (b[4 + i] + (m24(b[4 + i], 20091) >> 16)) + (m24(b[12 + i], 35468) >> 16);
        b[i] = a1 + d1;
        b[4 + i] = b1 + c1;
        b[12 + i] = a1 - d1;
        b[8 + i] = b1 - c1;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a1 = b[4 * i] + b[4 * i + 2], b1 = b[4 * i] - b[4 * i + 2];
        int c1 = (m24(b[4 * i + 1], 35468) >> 16) - (b[4 * i + 3] + (m24(b[4 * i + 3], 20091) >> 16));
        int d1 = (b[4 * i + 1] + (m24(b[4 * i + 1], 20091) >> 16)) + (m24(b[4 * i + 3], 35468) >> 16);
        b[4 * i] = (a1 + d1 + 4) >> 3;
        b[4 * i + 3] = (a1 - d1 + 4) >> 3;
        b[4 * i + 1] = (b1 + c1 + 4) >> 3;
        b[4 * i + 2] = (b1 - c1 + 4) >> 3;
    }
}

// idct4x4_sse2 with exact i16 semantics (transform_simd_intrinsics.rs:478):
// saturating pack, wrapping i16 adds, _mm_mulhi_epi16, i16 >>3.  Used by the
// decoder, whose inputs come from arbitrary bitstreams.
DI int w16(int v) { return (int)(short)(unsigned short)(unsigned)v; }
DI int sat16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
DI int mulhi16(int x, int k) { return (x * k) >> 16; }
DI void idct16_exact(int* b)
{
    int t[16];
#pragma unroll
    for (int i = 0; i < 16; i++) b[i] = sat16(b[i]);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int x0 = b[i], x1 = b[4 + i], x2 = b[8 + i], x3 = b[12 + i];
        int a = w16(x0 + x2), bb = w16(x0 - x2);
        int c = w16(w16(x1 - x3) + w16(mulhi16(x1, -30068) - mulhi16(x3, 20091)));
        int d = w16(w16(x1 + x3) + w16(mulhi16(x1, 20091) + mulhi16(x3, -30068)));
        t[i] = w16(a + d);
        t[4 + i] = w16(bb + c);
        t[8 + i] = w16(bb - c);
        t[12 + i] = w16(a - d);
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        int y0 = t[r * 4], y1 = t[r * 4 + 1], y2 = t[r * 4 + 2], y3 = t[r * 4 + 3];
        int dc = w16(y0 + 4);
        int a = w16(dc + y2), bb = w16(dc - y2);
        int c = w16(w16(y1 - y3) + w16(mulhi16(y1, -30068) - mulhi16(y3, 20091)));
        int d = w16(w16(y1 + y3) + w16(mulhi16(y1, 20091) + mulhi16(y3, -30068)));
        b[r * 4] = w16(a + d) >> 3;
        b[r * 4 + 1] = w16(bb + c) >> 3;
        b[r * 4 + 2] = w16(bb - c) >> 3;
        b[r * 4 + 3] = w16(a - d) >> 3;
    }
}

// wht4x4 (transform.rs:116)
DI void wht16(int* b)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a = b[i * 4] + b[i * 4 + 3], bb = b[i * 4 + 1] + b[i * 4 + 2];
        int c = b[i * 4 + 1] - b[i * 4 + 2], d = b[i * 4] - b[i * 4 + 3];
        b[i * 4] = a + bb;
        b[i * 4 + 1] = c + d;
        b[i * 4 + 2] = a - bb;
        b[i * 4 + 3] = d - c;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a1 = b[i] + b[i + 12], b1 = b[i + 4] + b[i + 8];
        int c1 = b[i + 4] - b[i + 8], d1 = b[i] - b[i + 12];
        int a2 = a1 + b1, b2 = c1 + d1, c2 = a1 - b1, d2 = d1 - c1;
        b[i] = (a2 + (a2 > 0 ? 1 : 0)) / 2;
        b[i + 4] = (b2 + (b2 > 0 ? 1 : 0)) / 2;
        b[i + 8] = (c2 + (c2 > 0 ? 1 : 0)) / 2;
        b[i + 12] = (d2 + (d2 > 0 ? 1 : 0)) / 2;
    }
}

// iwht4x4 (transform.rs:82)
DI void iwht16(int* b)
{
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a1 = b[i] + b[12 + i], b1 = b[4 + i] + b[8 + i];
        int c1 = b[4 + i] - b[8 + i], d1 = b[i] - b[12 + i];
        b[i] = a1 + b1;
        b[4 + i] = c1 + d1;
        b[8 + i] = a1 - b1;
        b[12 + i] = d1 - c1;
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
        int a1 = b[4 * r] + b[4 * r + 3], b1 = b[4 * r + 1] + b[4 * r + 2];
        int c1 = b[4 * r + 1] - b[4 * r + 2], d1 = b[4 * r] - b[4 * r + 3];
        b[4 * r] = (a1 + b1 + 3) >> 3;
        b[4 * r + 1] = (c1 + d1 + 3) >> 3;
        b[4 * r + 2] = (a1 - b1 + 3) >> 3;
        b[4 * r + 3] = (d1 - c1 + 3) >> 3;
    }
}

// t_transform (cost.rs:59): weighted Hadamard magnitude of a 4x4 u8 block.
DI int ttransform(const int* in)
{
    int tmp[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int* r = in + i * 4;
        int a0 = r[0] + r[2], a1 = r[1] + r[3], a2 = r[1] - r[3], a3 = r[0] - r[2];
        tmp[i * 4] = a0 + a1;
        tmp[i * 4 + 1] = a3 + a2;
        tmp[i * 4 + 2] = a3 - a2;
        tmp[i * 4 + 3] = a0 - a1;
    }
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int a0 = tmp[i] + tmp[8 + i], a1 = tmp[4 + i] + tmp[12 + i];
        int a2 = tmp[4 + i] - tmp[12 + i], a3 = tmp[i] - tmp[8 + i];
        sum += kWY(i) * iabs(a0 + a1) + kWY(4 + i) * iabs(a3 + a2) +
               kWY(8 + i) * iabs(a3 - a2) + kWY(12 + i) * iabs(a0 - a1);
    }
    return sum;
}

// Tables the encoder kernels keep in LDS (per-lane indexed lookups must not go
// to constant memory: a divergent index turns into a vector load from L2).
struct LdsTables {
    uint16_t lc[4][8][3][68];
    uint16_t eob[4][8][3];
    uint16_t init[4][8][3];
    uint8_t probs[4][8][3][11];
    uint16_t lfc[2048];       // VP8_LEVEL_FIXED_COSTS
    uint16_t ent[256];        // VP8_ENTROPY_COST
    uint16_t fci4[10][10][10];  // VP8_FIXED_COSTS_I4
    uint8_t i4idx[10][16];    // d_I4_IDX
    uint8_t i4qa[10][16];     // 4 x the V index of pixel p under mode m (254 -> 3 - row, 255 -> 38)
    uint8_t zz[16];           // ZIGZAG
    uint8_t bands[17];        // VP8_ENC_BANDS
    uint8_t izz[16];          // inverse zigzag: natural index -> position
    uint8_t pad[15];
    uint16_t beob[4][8][3];   // bitcost(0, probs[..][0]) of the current probabilities
    uint16_t binit[4][8][3];  // bitcost(1, probs[..][0])
};

// Static (frame-independent) part of LdsTables; all threads of the block call it.
DI void load_static_tables(LdsTables* T, int tid, int nt, const uint8_t* probs /* [4][8][3][11] */)
{
    for (int i = tid; i < 96; i += nt) {
        const int p0 = probs[i * 11];
        (&T->beob[0][0][0])[i] = d_VP8_ENTROPY_COST[p0];
        (&T->binit[0][0][0])[i] = d_VP8_ENTROPY_COST[255 - p0];
    }
    for (int i = tid; i < 2048; i += nt) T->lfc[i] = d_VP8_LEVEL_FIXED_COSTS[i];
    for (int i = tid; i < 256; i += nt) T->ent[i] = d_VP8_ENTROPY_COST[i];
    for (int i = tid; i < 1000; i += nt) (&T->fci4[0][0][0])[i] = (&d_VP8_FIXED_COSTS_I4[0][0][0])[i];
    for (int i = tid; i < 160; i += nt) {
        const int idx = (&d_I4_IDX[0][0])[i], p = i & 15;
        (&T->i4idx[0][0])[i] = (uint8_t)idx;
        (&T->i4qa[0][0])[i] = (uint8_t)(4 * (idx == 254 ? 3 - (p >> 2) : (idx == 255 ? 38 : idx)));
    }
    for (int i = tid; i < 16; i += nt) T->zz[i] = d_ZIGZAG[i];
    for (int i = tid; i < 17; i += nt) T->bands[i] = d_VP8_ENC_BANDS[i];
    for (int i = tid; i < 16; i += nt) T->izz[d_ZIGZAG[i]] = (uint8_t)i;
}

DI uint32_t bitcost(const LdsTables* T, int bit, int p) { return bit ? T->ent[255 - p] : T->ent[p]; }

// get_residual_cost (cost.rs:1670 / SSE2 :1735).  'c' is indexed by position n
// exactly as the reference indexes Residual::coeffs (natural-order arrays are
// passed by the RD code: quirk A1).  'last' spans all 16 entries.
template <int FIRST>
DI uint32_t rcost(const int* c, int ctx0, int ctype, const LdsTables* T)
{
    int last = -1;
#pragma unroll
    for (int n = 0; n < 16; n++)
        if (c[n] != 0) last = n;
    const int p0 = T->probs[ctype][kBand(FIRST)][ctx0][0];
    if (last < 0) return bitcost(T, 0, p0);
    uint32_t cost = ctx0 == 0 ? bitcost(T, 1, p0) : 0;
    int ctx = ctx0;
#pragma unroll
    for (int n = FIRST; n < 16; n++) {
        if (n <= last) {
            int v = iabs(c[n]);
            cost += T->lfc[v < 2047 ? v : 2047] + T->lc[ctype][kBand(n)][ctx][v < 67 ? v : 67];
            ctx = v < 2 ? v : 2;
        }
    }
    if (last < 15) cost += bitcost(T, 0, T->probs[ctype][band_of(last + 1)][ctx][0]);
    return cost;
}

// ---------------------------------------------------------------------------
// 16-lane group forms: lane k = lane & 15 holds element k of one 4x4 block
// (row k >> 2, column k & 3); four blocks per wave.  Same arithmetic as the
// serial forms above.  Row exchanges use DPP quad_perm, column exchanges DPP
// row_ror (lane i reads lane (i - n) mod 16 of its row), sums the DPP
// butterfly xor1 / xor2 / half_mirror / mirror: no LDS round trips.
// ---------------------------------------------------------------------------
#define DPP(v, ctrl) __builtin_amdgcn_mov_dpp((v), (ctrl), 0xf, 0xf, false)
DI int qb0(int v) { return DPP(v, 0x00); }
DI int qb1(int v) { return DPP(v, 0x55); }
DI int qb2(int v) { return DPP(v, 0xAA); }
DI int qb3(int v) { return DPP(v, 0xFF); }
DI int ror4(int v) { return DPP(v, 0x124); }
DI int ror8(int v) { return DPP(v, 0x128); }
DI int ror12(int v) { return DPP(v, 0x12C); }
DI int shr1(int v) { return __builtin_amdgcn_update_dpp(0, (v), 0x111, 0xf, 0xf, false); }
DI int red16(int v)  // sum within aligned 16-lane groups, result in every lane
{
    v += DPP(v, 0xB1);   // quad xor 1
    v += DPP(v, 0x4E);   // quad xor 2
    v += DPP(v, 0x141);  // row half mirror (lane i <-> 7-i)
    v += DPP(v, 0x140);  // row mirror (lane i <-> 15-i)
    return v;
}
DI int gget(int v, int k) { return __shfl(v, k, 16); }

// Arithmetic select: both operands already computed; never becomes a branch.
DI int csel(bool c, int a, int b) { return b + ((a - b) & -(int)c); }

// Branch-free 4-way select (lane-varying i in 0..3): all operands are already
// computed, so the compiler cannot turn the choice into divergent branches.
DI int sel4(int i, int a, int b, int c, int d)
{
    const int m0 = -(int)(i == 0), m1 = -(int)(i == 1), m2 = -(int)(i == 2), m3 = -(int)(i == 3);
    return (a & m0) | (b & m1) | (c & m2) | (d & m3);
}

// column values t_0..t_3 (rows 0..3 of this lane's column) from the lane's row i
DI void gcol(int t, int i, int& t0, int& t1, int& t2, int& t3)
{
    const int m1 = ror4(t), p2 = ror8(t), p1 = ror12(t);  // rows i-1, i+2, i+1
    t0 = sel4(i, t, m1, p2, p1);
    t1 = sel4(i, p1, t, m1, p2);
    t2 = sel4(i, p2, p1, t, m1);
    t3 = sel4(i, m1, p2, p1, t);
}

DI int qrev(int v) { return DPP(v, 0x1B); }   // quad lane j <- 3-j
DI int qnext(int v) { return DPP(v, 0x39); }  // quad lane j <- (j+1)&3
DI int qprev(int v) { return DPP(v, 0x93); }  // quad lane j <- (j-1)&3
DI int qxor2(int v) { return DPP(v, 0x4E); }  // quad lane j <- j^2
DI int rrev(int v) { return DPP(DPP(v, 0x140), 0x1B); }  // row r <- 3-r, same column

// dct4x4 (transform.rs:176) in butterfly form: every lane forms the partner
// sum / difference (s, d) of its pair, then takes one value from the
// neighbouring row / column -- ~35 VALU ops instead of a full gather.
DI int fdct_g(int v, int k)
{
    const int i = k >> 2, j = k & 3;
    // rows: pair columns j <-> 3-j
    {
        const int r = qrev(v);
        const int s = v + r, d = v - r;              // col0: a/8, dd/8  col1: bb/8, c/8  col2: bb/8,-c/8  col3: a/8,-dd/8
        const int X = qnext(s), Y = qprev(d);
        const int ev = csel(j == 0, s + X, X - s) * 8;  // col0: a+bb  col2: a-bb
        const int od = (m24(Y, 8 * 5352) + m24(d, csel(j == 1, 8 * 2217, -8 * 2217)) + csel(j == 1, 14500, 7500)) >> 12;
        v = csel((j & 1) == 0, ev, od);
    }
    // columns: pair rows i <-> 3-i
    {
        const int r = rrev(v);
        const int s = v + r, d = v - r;              // row0: A, D  row1: B, C  row2: B,-C  row3: A,-D
        const int X = ror12(s), Y = ror4(d);          // row i+1 / row i-1
        const int ev = (csel(i == 0, s + X, X - s) + 7) >> 4;
        const int od = ((m24(Y, 5352) + m24(d, csel(i == 1, 2217, -2217)) + csel(i == 1, 12000, 51000)) >> 16) +
                       (int)(i == 1 && Y != 0);
        return csel((i & 1) == 0, ev, od);
    }
}

// idct4x4 in butterfly form (same arithmetic as idct16).
DI int idct_g(int x, int k)
{
    const int i = k >> 2, j = k & 3;
    // vertical: rows i and i^2 pair up; even rows hold (a1, b1), odd rows (d1, c1)
    {
        const int o = ror8(x);                 // row i+2
        const bool even = (i & 1) == 0;
        const int x0 = csel(i == 0, x, o), x2 = csel(i == 0, o, x);      // even rows
        const int x1 = csel(i == 1, x, o), x3 = csel(i == 1, o, x);      // odd rows
        const int a1 = x0 + x2, b1 = x0 - x2;
        const int c1 = (m24(x1, 35468) >> 16) - (x3 + (m24(x3, 20091) >> 16));
        const int d1 = (x1 + (m24(x1, 20091) >> 16)) + (m24(x3, 35468) >> 16);
        const int p = csel(even, a1, d1), q = csel(even, b1, c1);
        // row0 <- d1 (row1, i+1); row1 <- b1 (row0, i-1); row2 <- c1 (row3, i+1); row3 <- a1 (row2, i-1)
        const int send = csel(i == 0 || i == 3, q, p);
        const int nb = csel(even, ror12(send), ror4(send));
        const int base = csel(i == 0 || i == 3, p, q);
        x = csel(i == 3, -base, base) + csel(i == 2, -nb, nb);
    }
    // horizontal: columns j and j^2 pair up
    {
        const int o = qxor2(x);
        const bool even = (j & 1) == 0;
        const int y0 = csel(j == 0, x, o), y2 = csel(j == 0, o, x);
        const int y1 = csel(j == 1, x, o), y3 = csel(j == 1, o, x);
        const int a1 = y0 + y2, b1 = y0 - y2;
        const int c1 = (m24(y1, 35468) >> 16) - (y3 + (m24(y3, 20091) >> 16));
        const int d1 = (y1 + (m24(y1, 20091) >> 16)) + (m24(y3, 35468) >> 16);
        const int p = csel(even, a1, d1), q = csel(even, b1, c1);
        const int send = csel(j == 0 || j == 3, q, p);
        const int nb = csel(even, qnext(send), qprev(send));
        const int base = csel(j == 0 || j == 3, p, q);
        return (csel(j == 3, -base, base) + csel(j == 2, -nb, nb) + 4) >> 3;
    }
}

// 16-bit nonzero mask of the lane's group.
DI unsigned gmask(bool pred)
{
    const unsigned long long b = __ballot(pred);
    return (unsigned)(b >> (__lane_id() & 48)) & 0xffffu;
}

// rcost<FIRST> with lane k holding c[k] (position n = k, quirk A1).  Result is
// uniform across the group.  T->beob / T->binit are bitcost(0/1, p[0]) of the
// current probabilities.
// LC = false: the LevelCosts tables are all zero (pass 1, quirk A2), so their
// lookups are skipped (the sum is the same).
template <int FIRST, bool LC = true>
DI uint32_t rcost_g(int v, int k, int ctx0, int ctype, const LdsTables* T)
{
    const unsigned m = gmask(v != 0);
    const int last = m ? 31 - __clz((int)m) : -1;
    const int av = iabs(v);
    const int pav = shr1(av);
    const int ctx = k == FIRST ? ctx0 : min(pav, 2);
    // unconditional lookups with clamped indices, masked arithmetic (no branches)
    const int tl = T->lfc[min(av, 2047)] + (LC ? (int)T->lc[ctype][band_of(k)][ctx][min(av, 67)] : 0);
    const int term = tl & -(int)(k >= FIRST && k <= last);
    const int lastc = max(last, 0);
    const int lastv = gget(av, lastc);
    const int bf = band_of(FIRST);
    const int e_none = T->beob[ctype][bf][ctx0];
    const int e_init = T->binit[ctype][bf][ctx0] & -(int)(ctx0 == 0);
    const int e_tail = T->beob[ctype][band_of(min(lastc + 1, 15))][lastv == 1 ? 1 : 2] & -(int)(last < 15);
    const int extra = last < 0 ? e_none : e_init + e_tail;
    return (uint32_t)(red16(term) + extra);
}

// trellis_quantize_block (cost.rs:788-1006).  coeffs (natural order) become the
// dequantized values; out (zigzag) the levels.  Returns has_nz.
// SMALL: every product is formed with full-rate 24-bit multiplies, exact for
// the encoder's operands (|coeff| + sharpening < 2^12, lambda < 2^16, level
// cost < 2^16); the general form (any int32 input) uses 32/64-bit multiplies.
template <int FIRST, bool SMALL = false>
DI int trellis(int* coeffs, int* out, const ZwMatrix& m, const uint16_t* sharpen, uint32_t lambda,
               const LdsTables* T, int ctype, int ctx0)
{
    auto mul = [](int a, int b) -> int { return SMALL ? m24(a, b) : a * b; };
    auto umul = [](uint32_t a, uint32_t b) -> uint32_t { return SMALL ? __umul24(a, b) : a * b; };
    auto rate = [&](int r) -> long long {
        return SMALL ? (long long)__umul24((uint32_t)r, lambda) : (long long)r * lambda;
    };
    const long long MAXC = 0x3fffffffffffffffLL;
    const int qac = (int)m.q[1];
    const int thresh = (qac * qac) / 4;
    int last = FIRST - 1;
#pragma unroll
    for (int n = FIRST; n < 16; n++) {
        int j = kZZ(n);
        if (mul(coeffs[j], coeffs[j]) > thresh) last = n;
    }
    if (last < 15) last++;
    const int bfirst = kBand(FIRST);
    long long best = rate(T->eob[ctype][bfirst][ctx0]);
    long long init = ctx0 == 0 ? rate(T->init[ctype][bfirst][ctx0]) : 0;
    long long s0 = init, s1 = init;
    int c0 = ctx0, c1 = ctx0;  // ctx selecting the predecessor's cost table
    int bn = -1, bd = 0, bp = 0;
    unsigned prevbits = 0;
    int lv0[16], sg[16];
    const uint32_t nbias = ((0u << 17) + 128) >> 8, tbias = ((0x80u << 17) + 128) >> 8;
#pragma unroll
    for (int n = FIRST; n < 16; n++) {
        lv0[n] = 0;
        sg[n] = 0;
        if (n <= last) {
            const int j = kZZ(n);
            const int q = j == 0 ? (int)m.q[0] : qac;
            const uint32_t iq = j == 0 ? m.iq[0] : m.iq[1];
            const int sign = coeffs[j] < 0;
            const int cws = iabs(coeffs[j]) + sharpen[j];
            const uint32_t prod = umul((uint32_t)cws, iq);
            int l0 = (int)((prod + nbias) >> 17);
            l0 = l0 < 2047 ? l0 : 2047;
            int thr = (int)((prod + tbias) >> 17);
            thr = thr < 2047 ? thr : 2047;
            const int band = kBand(n);
            long long ns0 = MAXC, ns1 = MAXC;
            int nc0 = 0, nc1 = 0;
#pragma unroll
            for (int d = 0; d < 2; d++) {
                const int level = l0 + d;
                const int ctx = level < 2 ? level : 2;
                if (d == 0) nc0 = ctx;
                else nc1 = ctx;
                if (level <= thr) {
                    const int ne = cws - mul(level, q);
                    const long long dd = SMALL ? (long long)m24(kWTrellis(j), m24(ne, ne) - m24(cws, cws))
                                               : (long long)kWTrellis(j) * ((long long)(ne * ne) - (long long)(cws * cws));
                    const long long base = 256 * dd;
                    const int lv = level < 67 ? level : 67;
                    const int fixed = T->lfc[level] + (level > 0 ? 256 : 0);
                    long long sc0 = s0 + rate(fixed + T->lc[ctype][band][c0][lv]);
                    long long sc1 = s1 + rate(fixed + T->lc[ctype][band][c1][lv]);
                    int pb = sc1 < sc0;
                    long long cur = (pb ? sc1 : sc0) + base;
                    prevbits |= (unsigned)pb << (2 * n + d);
                    if (d == 0) ns0 = cur;
                    else ns1 = cur;
                    if (level != 0 && cur < best) {
                        long long eob = 0;
                        if (n < 15) eob = rate(T->eob[ctype][kBand(n + 1)][ctx]);
                        long long term = cur + eob;
                        if (term < best) {
                            best = term;
                            bn = n;
                            bd = d;
                            bp = pb;
                        }
                    }
                }
            }
            s0 = ns0;
            s1 = ns1;
            c0 = nc0;
            c1 = nc1;
            lv0[n] = l0;
            sg[n] = sign;
        }
    }
#pragma unroll
    for (int n = FIRST; n < 16; n++) {
        out[n] = 0;
        coeffs[kZZ(n)] = 0;
    }
    if (bn < 0) return 0;
    int nz = 0, cd = bd;
#pragma unroll
    for (int n = 15; n >= FIRST; n--) {
        if (n <= bn) {
            const int j = kZZ(n);
            const int level = lv0[n] + cd;
            const int v = sg[n] ? -level : level;
            out[n] = v;
            coeffs[j] = mul(v, (int)(j == 0 ? m.q[0] : m.q[1]));
            nz |= v != 0;
            cd = (n == bn) ? bp : (int)((prevbits >> (2 * n + cd)) & 1);
        }
    }
    return nz;
}

// ---------------------------------------------------------------------------
// Full-block lane forms: one lane holds a whole 4x4 block (16 values).
// ---------------------------------------------------------------------------
DI int red8(int v)  // sum within aligned 8-lane groups (DPP), result in every lane
{
    v += DPP(v, 0xB1);   // quad xor 1
    v += DPP(v, 0x4E);   // quad xor 2
    v += DPP(v, 0x141);  // row half mirror (lane i <-> 7-i)
    return v;
}

typedef short zs2 __attribute__((ext_vector_type(2)));
DI zs2 as_zs2(uint32_t v) { return __builtin_bit_cast(zs2, v); }
DI uint32_t as_zu(zs2 v) { return __builtin_bit_cast(uint32_t, v); }
// (lo16(a), lo16(b)) packed
DI uint32_t pack_lo(int a, int b) { return __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x05040100u); }
DI uint32_t clamp_pk(uint32_t v)  // per i16 half: clamp to [0, 255]
{
    const zs2 z = {0, 0}, m = {255, 255};
    return as_zu(__builtin_elementwise_min(__builtin_elementwise_max(as_zs2(v), z), m));
}
DI uint32_t add_pk(uint32_t a, uint32_t b) { return as_zu(as_zs2(a) + as_zs2(b)); }
DI uint32_t sub_pk(uint32_t a, uint32_t b) { return as_zu(as_zs2(a) - as_zs2(b)); }
// VOP3P v_dot2_i32_i16, accumulator from an SGPR (the builtin selects the VOP2
// dot2c form, which costs a v_mov of the accumulator every time)
DI int dot2(zs2 a, zs2 b, int c)
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

// dct4x4 (transform.rs:176) of one block of residuals r[16] (|r| <= 255) in
// packed-i16 form: rows as pairs (r0,r1),(r3,r2), butterflies v_pk_add/sub,
// rotations v_dot2 with the rounding folded in (see zw_xform_kernels.hip).
DI void fdct16_pk(const int* r, int* c)
{
    const zs2 k8p = {8, 8}, k8m = {8, -8}, k1a = {10704, 4434}, k1b = {4434, -10704};
    int o[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 R01 = as_zs2(pack_lo(r[4 * i], r[4 * i + 1])), R32 = as_zs2(pack_lo(r[4 * i + 3], r[4 * i + 2]));
        const zs2 A = R01 + R32, D = R01 - R32;
        o[4 * i] = dot2(A, k8p, 0);
        o[4 * i + 2] = dot2(A, k8m, 0);
        o[4 * i + 1] = dot2(D, k1a, 3625) >> 10;
        o[4 * i + 3] = dot2(D, k1b, 1875) >> 10;
    }
    const zs2 k1p = {1, 1}, k1m = {1, -1}, k2a = {5352, 2217}, k2b = {2217, -5352};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 X01 = as_zs2(pack_lo(o[i], o[4 + i])), X32 = as_zs2(pack_lo(o[12 + i], o[8 + i]));
        const zs2 A = X01 + X32, D = X01 - X32;
        c[i] = dot2(A, k1p, 7) >> 4;
        c[8 + i] = dot2(A, k1m, 7) >> 4;
        c[4 + i] = (dot2(D, k2a, 12000) >> 16) + ((as_zu(D) & 0xffffu) != 0u ? 1 : 0);
        c[12 + i] = dot2(D, k2b, 51000) >> 16;
    }
}

// rcost<FIRST> (get_residual_cost, cost.rs:1670) without branches: every
// table lookup is issued, terms past the last nonzero are masked.  v[n] is
// indexed by position n exactly as rcost (quirk A1); av[n] = |v[n]|.
template <int FIRST, bool LC = true>
DI uint32_t rcost_bf(const int* av, int ctx0, int ctype, const LdsTables* T)
{
    uint32_t nzm = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) nzm |= (uint32_t)min(av[n], 1) << n;
    const int last = 31 - __clz((int)nzm);  // -1 when nzm == 0 (clz(0) == 32)
    const int p0 = T->probs[ctype][kBand(FIRST)][ctx0][0];
    uint32_t cost = 0;
#pragma unroll
    for (int n = FIRST; n < 16; n++) {
        const int ctx = n == FIRST ? ctx0 : min(av[n - 1], 2);
        const int t = T->lfc[min(av[n], 2047)] + (LC ? (int)T->lc[ctype][kBand(n)][ctx][min(av[n], 67)] : 0);
        cost += (uint32_t)(t & -(int)(n <= last));
    }
    int lastv = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) lastv = n == last ? av[n] : lastv;
    const int ctx_t = last >= FIRST ? min(lastv, 2) : ctx0;  // the loop's final ctx
    const uint32_t tail =
        bitcost(T, 0, T->probs[ctype][band_of(min(last + 1, 15))][ctx_t][0]) & -(uint32_t)(last < 15);
    const uint32_t head = ctx0 == 0 ? bitcost(T, 1, p0) : 0u;
    return last < 0 ? bitcost(T, 0, p0) : head + cost + tail;
}

DI int dot2sv(zs2 a, zs2 b_uniform, int acc)  // v_dot2_i32_i16 with the multiplier pair in an SGPR
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_uniform), "v"(acc));
    return d;
}

// sum_k kWY(k) * (|T(a)_k| - |T(b)_k|) for the TDisto 4x4 Hadamard T
// (ttransform) of two blocks at once: a in the low and b in the high i16 half
// of every register, so each butterfly is one packed op and each weighted
// |coefficient| difference one v_dot2 against (w, -w).  |T(.)| <= 4080.
DI int ttransform_diff_pk(const int* a, const int* b)
{
    zs2 t[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 r0 = as_zs2(pack_lo(a[4 * i], b[4 * i])), r1 = as_zs2(pack_lo(a[4 * i + 1], b[4 * i + 1]));
        const zs2 r2 = as_zs2(pack_lo(a[4 * i + 2], b[4 * i + 2])), r3 = as_zs2(pack_lo(a[4 * i + 3], b[4 * i + 3]));
        const zs2 a0 = r0 + r2, a1 = r1 + r3, a2 = r1 - r3, a3 = r0 - r2;
        t[4 * i] = a0 + a1;
        t[4 * i + 1] = a3 + a2;
        t[4 * i + 2] = a3 - a2;
        t[4 * i + 3] = a0 - a1;
    }
    int acc = 0;
    const zs2 z = {0, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const zs2 a0 = t[i] + t[8 + i], a1 = t[4 + i] + t[12 + i];
        const zs2 a2 = t[4 + i] - t[12 + i], a3 = t[i] - t[8 + i];
        const zs2 o[4] = {a0 + a1, a3 + a2, a3 - a2, a0 - a1};
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const zs2 ab = __builtin_elementwise_max(o[r], z - o[r]);
            const short w = (short)kWY(4 * r + i);
            const zs2 wp = {w, (short)-w};
            acc = dot2sv(ab, wp, acc);
        }
    }
    return acc;
}

// kWTrellis[j] for a lane-varying j (two 64-bit immediates, 8 bits per entry)
DI int wtrellis_of(int j)
{
    const unsigned long long lo = 0x0a11181b0b131b1eull, hi = 0x06080a0b080c1113ull;
    return (int)(((j < 8 ? lo : hi) >> (8 * (j & 7))) & 255ull);
}

DI long long llmin(long long a, long long b) { return a < b ? a : b; }
// Materialise a cross-lane result at this point of the program: a DPP whose
// value feeds only a lane-dependent select may otherwise be sunk into a
// branch, where it would read inactive source lanes.
DI int pin(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}
DI long long pin(long long v)
{
    asm volatile("" : "+v"(v));
    return v;
}
template <int CTRL>
DI long long dpp_ll(long long v, long long old)  // 64-bit DPP row op; lanes without a source get `old`
{
    const int lo = __builtin_amdgcn_update_dpp((int)(old & 0xffffffff), (int)(v & 0xffffffff), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(old >> 32), (int)(v >> 32), CTRL, 0xf, 0xf, false);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}
// one step of the inclusive min-plus scan of 2x2 matrices (row_shr CTRL)
template <int CTRL>
DI void mp_scan_step(long long& P00, long long& P01, long long& P10, long long& P11, long long INF)
{
    const long long Q00 = dpp_ll<CTRL>(P00, 0), Q01 = dpp_ll<CTRL>(P01, INF);
    const long long Q10 = dpp_ll<CTRL>(P10, INF), Q11 = dpp_ll<CTRL>(P11, 0);
    const long long R00 = llmin(P00 + Q00, P01 + Q10), R01 = llmin(P00 + Q01, P01 + Q11);
    const long long R10 = llmin(P10 + Q00, P11 + Q10), R11 = llmin(P10 + Q01, P11 + Q11);
    P00 = R00;
    P01 = R01;
    P10 = R10;
    P11 = R11;
}
// group min of (t, i) with the smallest i on ties, one xor-butterfly step
template <int CTRL>
DI void argmin_step(long long& t, int& i)
{
    const long long ot = dpp_ll<CTRL>(t, 0);
    const int oi = DPP(i, CTRL);
    const bool take = ot < t || (ot == t && oi < i);
    t = take ? ot : t;
    i = take ? oi : i;
}

// trellis_quantize_block (cost.rs:788-1006) in 16-lane group form: lane n =
// zigzag position n, cn = the coefficient at that position.  The per-position
// node costs do not depend on the path (a node's context is fixed by its own
// level), so the Viterbi recurrence over positions is a min-plus product of
// 2x2 transition matrices: an inclusive scan of them (4 DPP row_shr steps)
// gives every position's node scores at once.  Ties and the early-stop rule
// are the serial version's: argmin strict (sc1 < sc0), best term the first
// strict minimum in (n, d) order.  Returns the group's any-nonzero flag and
// the signed level at position n in lvl.
template <int FIRST>
DI int trellis_g(int cn, int n, const ZwMatrix& m, const uint16_t* sharpen, uint32_t lambda, const LdsTables* T,
                 int ctype, int ctx0, int& lvl)
{
    const long long INF = 1LL << 57;
    const int j = zz_of(n);
    const int qac = (int)m.q[1];
    const int thresh = (qac * qac) / 4;
    const long long lam = lambda;
    // last position processed: highest n >= FIRST with c^2 > thresh (or FIRST - 1), plus one
    const unsigned big = gmask(n >= FIRST && cn * cn > thresh);
    int last = big ? 31 - __clz((int)big) : FIRST - 1;
    if (last < 15) last++;
    const bool inpos = n >= FIRST && n <= last;
    const int q = j == 0 ? (int)m.q[0] : qac;
    const uint32_t iq = j == 0 ? m.iq[0] : m.iq[1];
    const int sign = cn < 0;
    const int cws = iabs(cn) + sharpen[j];
    const int l0 = min((int)(((uint32_t)cws * iq) >> 17), 2047);
    const int thr = min((int)(((uint32_t)cws * iq + 65536u) >> 17), 2047);
    const int band = kBand(n);
    const int w = wtrellis_of(j);
    // predecessor contexts (position n - 1's node levels), ctx0 at FIRST
    const int l0p = pin(shr1(l0));
    const int cp0 = n == FIRST ? ctx0 : min(l0p, 2), cp1 = n == FIRST ? ctx0 : min(l0p + 1, 2);
    long long M[2][2], base[2], eobc[2];
    int valid[2];
#pragma unroll
    for (int d = 0; d < 2; d++) {
        const int level = l0 + d;
        valid[d] = inpos && level <= thr;
        const int ne = cws - level * q;
        base[d] = 256LL * ((long long)w * ((long long)(ne * ne) - (long long)(cws * cws)));
        const int lv = min(level, 67);
        const int fixed = T->lfc[min(level, 2047)] + (level > 0 ? 256 : 0);
        const long long c0 = (long long)(fixed + T->lc[ctype][band][cp0][lv]) * lam;
        const long long c1 = (long long)(fixed + T->lc[ctype][band][cp1][lv]) * lam;
        M[d][0] = valid[d] ? c0 + base[d] : INF;
        M[d][1] = valid[d] ? c1 + base[d] : INF;
        eobc[d] = n < 15 ? (long long)T->eob[ctype][kBand(n + 1)][min(level, 2)] * lam : 0;
    }
    if (!inpos) {  // positions outside FIRST..last leave the scores unchanged
        M[0][0] = 0;
        M[0][1] = INF;
        M[1][0] = INF;
        M[1][1] = 0;
    }
    // inclusive min-plus scan: P_n = M_n (x) M_{n-1} (x) ... (x) M_0
    long long P00 = M[0][0], P01 = M[0][1], P10 = M[1][0], P11 = M[1][1];
    mp_scan_step<0x111>(P00, P01, P10, P11, INF);  // row_shr:1
    mp_scan_step<0x112>(P00, P01, P10, P11, INF);  // row_shr:2
    mp_scan_step<0x114>(P00, P01, P10, P11, INF);  // row_shr:4
    mp_scan_step<0x118>(P00, P01, P10, P11, INF);  // row_shr:8
    const long long init = ctx0 == 0 ? (long long)T->init[ctype][kBand(FIRST)][ctx0] * lam : 0;
    const long long s0 = init + llmin(P00, P01), s1 = init + llmin(P10, P11);  // node scores after position n
    // predecessor scores -> the serial version's argmin bits
    const long long q0 = pin(dpp_ll<0x111>(s0, init)), q1 = pin(dpp_ll<0x111>(s1, init));
    const long long p0 = n == FIRST ? init : q0, p1 = n == FIRST ? init : q1;
    int pb[2];
#pragma unroll
    for (int d = 0; d < 2; d++) pb[d] = (p1 + (M[d][1] - base[d])) < (p0 + (M[d][0] - base[d]));
    // best terminating node: first strict minimum of s_d + eob_d over (n, d), against the empty block
    const long long best0 = (long long)T->eob[ctype][kBand(FIRST)][ctx0] * lam;
    const long long t0 = (valid[0] && l0 != 0) ? s0 + eobc[0] : INF;
    const long long t1 = valid[1] ? s1 + eobc[1] : INF;
    long long bt = t1 < t0 ? t1 : t0;
    int bi = 2 * n + (t1 < t0 ? 1 : 0);
    argmin_step<0xB1>(bt, bi);   // quad xor 1
    argmin_step<0x4E>(bt, bi);   // quad xor 2
    argmin_step<0x141>(bt, bi);  // row half mirror
    argmin_step<0x140>(bt, bi);  // row mirror
    lvl = 0;
    if (!(bt < best0)) return 0;  // the empty block wins (bn = -1)
    const int bn = bi >> 1, bd = bi & 1;
    // backtrack: cd_{n-1} = pb_n[cd_n], from (bn, bd)
    const unsigned long long ball = __ballot(pb[0] != 0), ball1 = __ballot(pb[1] != 0);
    const int gsh = __lane_id() & 48;
    const unsigned pbm0 = (unsigned)(ball >> gsh) & 0xffffu, pbm1 = (unsigned)(ball1 >> gsh) & 0xffffu;
    unsigned cdm = 0;
    int cd = bd;
    for (int k = bn; k >= FIRST; k--) {
        cdm |= (unsigned)cd << k;
        cd = (int)(((cd ? pbm1 : pbm0) >> k) & 1u);
    }
    const int level = (n >= FIRST && n <= bn) ? l0 + (int)((cdm >> n) & 1u) : 0;
    lvl = sign ? -level : level;
    return gmask(level != 0) != 0;
}

// 4-point Walsh-Hadamard butterflies in 16-lane group form (lane k = element k
// of a 4x4 block, row k >> 2, column k & 3).  Row pass: out0 = a + b, out1 =
// c + d, out2 = a - b, out3 = d - c with a = x0 + x3, b = x1 + x2, c = x1 - x2,
// d = x0 - x3 (the pass shared by wht16's rows and iwht16's rows); column
// pass: the same on the rows of a column.
DI int hrow_g(int x, int j)
{
    const int r = qrev(x);
    const int s = x + r, df = x - r;  // col0: a, d  col1: b, c  col2: b, -c  col3: a, -d
    const int X = pin(qnext(s)), Y = pin(qprev(df));
    return sel4(j, s + X, df + Y, X - s, Y - df);
}
DI int hcol_g(int x, int i)
{
    const int r = pin(rrev(x));
    const int s = x + r, df = x - r;
    const int X = pin(ror12(s)), Y = pin(ror4(df));  // row i + 1 / row i - 1
    return sel4(i, s + X, df + Y, X - s, Y - df);
}
// wht16 (transform.rs:58): rows, then columns with (v + (v > 0)) / 2
DI int wht_g(int x, int k)
{
    const int v = hcol_g(hrow_g(x, k & 3), k >> 2);
    return (v + (v > 0 ? 1 : 0)) / 2;
}
// iwht16 (transform.rs:82): columns, then rows with (v + 3) >> 3
DI int iwht_g(int x, int k) { return (hrow_g(hcol_g(x, k >> 2), k & 3) + 3) >> 3; }

// idct16_exact (SSE2 i16 semantics, transform_simd_intrinsics.rs:478) in
// 16-lane group form: the butterfly of idct_g with every intermediate wrapped
// to i16, the multiplies as _mm_mulhi_epi16 and the input saturated.
DI int idct_g_exact(int x, int k)
{
    const int i = k >> 2, j = k & 3;
    x = sat16(x);
    {
        const int o = pin(ror8(x));  // row i+2
        const bool even = (i & 1) == 0;
        const int x0 = csel(i == 0, x, o), x2 = csel(i == 0, o, x);
        const int x1 = csel(i == 1, x, o), x3 = csel(i == 1, o, x);
        const int a = w16(x0 + x2), bb = w16(x0 - x2);
        const int c = w16(w16(x1 - x3) + w16(mulhi16(x1, -30068) - mulhi16(x3, 20091)));
        const int d = w16(w16(x1 + x3) + w16(mulhi16(x1, 20091) + mulhi16(x3, -30068)));
        const int p = csel(even, a, d), q = csel(even, bb, c);
        const int send = csel(i == 0 || i == 3, q, p);
        const int nb = csel(even, pin(ror12(send)), pin(ror4(send)));
        const int base = csel(i == 0 || i == 3, p, q);
        x = w16(csel(i == 3, -base, base) + csel(i == 2, -nb, nb));
    }
    {
        x = csel(j == 0, w16(x + 4), x);  // dc = y0 + 4
        const int o = pin(qxor2(x));
        const bool even = (j & 1) == 0;
        const int y0 = csel(j == 0, x, o), y2 = csel(j == 0, o, x);
        const int y1 = csel(j == 1, x, o), y3 = csel(j == 1, o, x);
        const int a = w16(y0 + y2), bb = w16(y0 - y2);
        const int c = w16(w16(y1 - y3) + w16(mulhi16(y1, -30068) - mulhi16(y3, 20091)));
        const int d = w16(w16(y1 + y3) + w16(mulhi16(y1, 20091) + mulhi16(y3, -30068)));
        const int p = csel(even, a, d), q = csel(even, bb, c);
        const int send = csel(j == 0 || j == 3, q, p);
        const int nb = csel(even, pin(qnext(send)), pin(qprev(send)));
        const int base = csel(j == 0 || j == 3, p, q);
        return w16(csel(j == 3, -base, base) + csel(j == 2, -nb, nb)) >> 3;
    }
}

// ---- quad-form 4x4 transform (lane q of a quad: row q of the pixels, column q of
// the coefficients); the encoder's I4 candidates and k_xform_mb_i4
DI int dot2v(uint32_t a, uint32_t b, int acc)  // v_dot2_i32_i16, both operands in VGPRs
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(acc));
    return d;
}
// The quad's row-transform inputs broadcast to every lane: lane q forms
// column q of the row stage (dct4x4 transform.rs:176) for rows 0..3, then the
// column stage: c[r] = coefficient (r, q), natural index 4 r + q.
DI void uvq_fdct(uint32_t A, uint32_t D, int q, int c[4])
{
    const bool odd = q & 1;
    const zs2 k0 = {8, 8}, k2 = {8, -8}, k1 = {10704, 4434}, k3 = {4434, -10704};
    // (arithmetic selects: lane-dependent ?: chains became divergent branches)
    const uint32_t k = (uint32_t)sel4(q, (int)as_zu(k0), (int)as_zu(k1), (int)as_zu(k2), (int)as_zu(k3));
    const int rnd = sel4(q, 0, 3625, 0, 1875);
    const int sh = csel(odd, 10, 0);
    // (csel, not ?: -- a select of two DPP results may be folded into one DPP
    // of a select, which would take the source lane's choice)
    int t[4];
    t[0] = dot2v((uint32_t)csel(odd, qb0((int)D), qb0((int)A)), k, rnd) >> sh;
    t[1] = dot2v((uint32_t)csel(odd, qb1((int)D), qb1((int)A)), k, rnd) >> sh;
    t[2] = dot2v((uint32_t)csel(odd, qb2((int)D), qb2((int)A)), k, rnd) >> sh;
    t[3] = dot2v((uint32_t)csel(odd, qb3((int)D), qb3((int)A)), k, rnd) >> sh;
    const uint32_t X01 = pack_lo(t[0], t[1]), X32 = pack_lo(t[3], t[2]);
    const zs2 XA = as_zs2(X01) + as_zs2(X32), XD = as_zs2(X01) - as_zs2(X32);
    const zs2 k1p = {1, 1}, k1m = {1, -1}, k2a = {5352, 2217}, k2b = {2217, -5352};
    c[0] = dot2(XA, k1p, 7) >> 4;
    c[2] = dot2(XA, k1m, 7) >> 4;
    c[1] = (dot2(XD, k2a, 12000) >> 16) + ((as_zu(XD) & 0xffffu) != 0u ? 1 : 0);
    c[3] = dot2(XD, k2b, 51000) >> 16;
}

// idct4x4 (transform.rs:19) of the quad's dequantised columns (lane q holds
// column q, rows 0..3), then the reconstruction clamp(pred + residual) of row q
// as i16 pairs (x0, x1), (x3, x2).
DI void uvq_idct_recon(const int dq[4], uint32_t p01, uint32_t p32, int q, uint32_t& r01, uint32_t& r32)
{
    uint32_t lo, hi;
    {
        const int x0 = dq[0], x1 = dq[1], x2 = dq[2], x3 = dq[3];
        const int a1 = x0 + x2, b1 = x0 - x2;
        const int c1 = (m24(x1, 35468) >> 16) - (x3 + (m24(x3, 20091) >> 16));
        const int d1 = (x1 + (m24(x1, 20091) >> 16)) + (m24(x3, 35468) >> 16);
        lo = pack_lo(a1 + d1, b1 + c1);
        hi = pack_lo(b1 - c1, a1 - d1);
    }
    // row q of every column: the lane of column j holds it in lo (rows 0, 1) or hi (rows 2, 3)
    const bool upper = q >= 2;
    const uint32_t off = 16u * (uint32_t)(q & 1);
    const int y0 = __builtin_amdgcn_sbfe(csel(upper, qb0((int)hi), qb0((int)lo)), off, 16);
    const int y1 = __builtin_amdgcn_sbfe(csel(upper, qb1((int)hi), qb1((int)lo)), off, 16);
    const int y2 = __builtin_amdgcn_sbfe(csel(upper, qb2((int)hi), qb2((int)lo)), off, 16);
    const int y3 = __builtin_amdgcn_sbfe(csel(upper, qb3((int)hi), qb3((int)lo)), off, 16);
    const int a1 = y0 + y2, b1 = y0 - y2;
    const int c1 = (m24(y1, 35468) >> 16) - (y3 + (m24(y3, 20091) >> 16));
    const int d1 = (y1 + (m24(y1, 20091) >> 16)) + (m24(y3, 35468) >> 16);
    const int o0 = (a1 + d1 + 4) >> 3, o1 = (b1 + c1 + 4) >> 3, o2 = (b1 - c1 + 4) >> 3, o3 = (a1 - d1 + 4) >> 3;
    r01 = clamp_pk(add_pk(pack_lo(o0, o1), p01));
    r32 = clamp_pk(add_pk(pack_lo(o3, o2), p32));
}

