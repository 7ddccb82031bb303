// zw_pack_kernels.hip -- device-side compaction of the per-MB encoder records
// before they cross PCIe to the host entropy stage.
//
// ZwMbOut is 820 B/MB (modes + 25x16 int16 levels, mostly zero).  The host
// only needs each block's levels up to its last nonzero (zigzag eob), so the
// records are packed into a byte stream per frame:
//
//   MB := u8 hdr (luma 0..4 | skip << 3 | segment << 4 | chroma << 6)
//         [8 B sub-modes, 4 bits each, if luma == 4]
//         u8 eob[25]            (blocks 0..15 Y, 16 Y2, 17..20 U, 21..24 V)
//         i16 levels[sum eob]   (block order, zigzag positions 0..eob-1)
//
// k_pack_size: one wave per MB -> eobs + MB size; k_pack_scan: one workgroup
// per frame -> MB offsets and an atomically reserved slice of the output
// buffer (frames land contiguously, in any order; offsets are reported);
// k_pack_write: one wave per MB.
#include "zw_dev.h"

#ifndef PK_WAVES
#define PK_WAVES 4  // MBs (one wave each) per workgroup
#endif

__device__ __forceinline__ int pk_mb_size(int luma, int eobsum) { return 1 + (luma == 4 ? 8 : 0) + 25 + 2 * eobsum; }

// The 800 B of levels of an MB as 200 aligned words (ZwMbOut is 4-byte
// aligned): round r, lane l holds word j = l + 64 r = zigzag positions
// 2 (j & 7), +1 of block j >> 3; the 8 lanes of a block reduce with DPP.
__device__ __forceinline__ int pk_word_eob(uint32_t v, int j)
{
    const int n0 = 2 * (j & 7);
    return (v >> 16) ? n0 + 2 : ((v & 0xffffu) ? n0 + 1 : 0);
}
__device__ __forceinline__ int max8(int e)  // max within aligned 8-lane groups, result in every lane
{
    e = max(e, __builtin_amdgcn_mov_dpp(e, 0xB1, 0xf, 0xf, false));  // quad xor 1
    e = max(e, __builtin_amdgcn_mov_dpp(e, 0x4E, 0xf, 0xf, false));  // quad xor 2
    e = max(e, __builtin_amdgcn_mov_dpp(e, 0x141, 0xf, 0xf, false)); // row half mirror: lane i <-> 7-i
    return e;
}

extern "C" __global__ __launch_bounds__(64 * PK_WAVES) void k_pack_size(const ZwMbOut* __restrict__ mbs, int nmb,
                                                                      int nframes, uint8_t* __restrict__ eobs,
                                                                      uint32_t* __restrict__ sizes)
{
    const size_t mb = (size_t)blockIdx.x * PK_WAVES + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (mb >= (size_t)nmb * nframes) return;
    const ZwMbOut& M = mbs[mb];
    const uint32_t* W = (const uint32_t*)&M.levels[0][0];
    uint32_t w[4];
#pragma unroll
    for (int r = 0; r < 4; r++) w[r] = lane + 64 * r < 200 ? W[lane + 64 * r] : 0u;
    const int skip = M.skip;
    int s = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = lane + 64 * r;
        const int eob = skip ? 0 : max8(pk_word_eob(w[r], j));
        if ((j & 7) == 0 && j < 200) {
            eobs[mb * 25 + (j >> 3)] = (uint8_t)eob;
            s += eob;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) sizes[mb] = (uint32_t)pk_mb_size(M.luma_mode, s);
}

// One workgroup (1024 threads) per frame: exclusive scan of MB sizes in place,
// frame slice reservation.  frame_info[f] = {offset, bytes}.
extern "C" __global__ __launch_bounds__(1024) void k_pack_scan(uint32_t* __restrict__ sizes, int nmb,
                                                              unsigned long long* __restrict__ counter,
                                                              unsigned long long* __restrict__ frame_info)
{
    __shared__ uint32_t part[1024];
    __shared__ unsigned long long base;
    const int f = blockIdx.x, t = threadIdx.x;
    uint32_t* S = sizes + (size_t)f * nmb;
    const int per = (nmb + 1023) / 1024;
    const int b0 = t * per, b1 = min(b0 + per, nmb);
    uint32_t acc = 0;
    for (int i = b0; i < b1; i++) acc += S[i];
    part[t] = acc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - acc;  // exclusive prefix of this thread's chunk
    for (int i = b0; i < b1; i++) {
        const uint32_t v = S[i];
        S[i] = run;
        run += v;
    }
    if (t == 1023) {
        const unsigned long long tot = part[1023];
        base = atomicAdd(counter, tot);
        frame_info[2 * f] = base;
        frame_info[2 * f + 1] = tot;
        // the last frame to reserve its slice publishes the chunk total and
        // clears the counters for the next launch (no memset blit per chunk)
        __threadfence();
        if (atomicAdd(counter + 1, 1ull) == (unsigned long long)gridDim.x - 1) {
            __threadfence();
            const unsigned long long all = atomicAdd(counter, 0ull);
            counter[2] = all;
            atomicExch(counter, 0ull);
            atomicExch(counter + 1, 0ull);
        }
    }
}

// MB sizes are even (header 26 or 34 bytes + 2 per level) and so are the
// frame slices, so every level lands on a 2-byte aligned address.  The eobs
// are recomputed from the level words (as k_pack_size does) rather than read
// back, so every load of a wave is issued in one round: the MB's words, its
// header and its offset.
extern "C" __global__ __launch_bounds__(64 * PK_WAVES) void k_pack_write(
    const ZwMbOut* __restrict__ mbs, int nmb, int nframes, const uint8_t* __restrict__ eobs,
    const uint32_t* __restrict__ offs, const unsigned long long* __restrict__ frame_info, uint8_t* __restrict__ out)
{
    const size_t mb = (size_t)blockIdx.x * PK_WAVES + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (mb >= (size_t)nmb * nframes) return;
    const int f = (int)(mb / nmb);
    const ZwMbOut& M = mbs[mb];
    const uint32_t* W = (const uint32_t*)&M.levels[0][0];
    uint32_t w[4];
#pragma unroll
    for (int r = 0; r < 4; r++) w[r] = lane + 64 * r < 200 ? W[lane + 64 * r] : 0u;
    const uint32_t hw = *(const uint32_t*)&M;  // luma, chroma, skip, segment
    const uint32_t bp = lane < 8 ? *(const uint16_t*)&M.bpred[2 * lane] : 0u;
    uint8_t* o = out + frame_info[2 * f] + offs[mb];
    const int luma = (int)(hw & 255u), chroma = (int)((hw >> 8) & 255u), skip = (int)((hw >> 16) & 255u),
              seg = (int)(hw >> 24);
    const int hdr = 1 + (luma == 4 ? 8 : 0);
    // eob of block j >> 3 in every lane of its 8-lane group, per round
    int eb4[4];
#pragma unroll
    for (int r = 0; r < 4; r++) eb4[r] = skip ? 0 : max8(pk_word_eob(w[r], lane + 64 * r));
    // block b's eob into lane b (lanes 0..24): group b lives in round b >> 3, lanes 8 (b & 7)..
    int eob = 0;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int v = __shfl(eb4[r], 8 * (lane & 7));
        eob = (lane >> 3) == r ? v : eob;
    }
    eob = lane < 25 ? eob : 0;
    if (lane == 0) o[0] = (uint8_t)(luma | (skip << 3) | (seg << 4) | (chroma << 6));
    if (luma == 4 && lane < 8) o[1 + lane] = (uint8_t)((bp & 15u) | (((bp >> 8) & 15u) << 4));
    if (lane < 25) o[hdr + lane] = (uint8_t)eob;
    // exclusive prefix of eobs over lanes 0..24
    int pre = eob;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) {
        const int v = __shfl_up(pre, d);
        if (lane >= d) pre += v;
    }
    pre -= eob;
    int16_t* lv = (int16_t*)(o + hdr + 25);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int j = lane + 64 * r;
        const int b = min(j >> 3, 24), n0 = 2 * (j & 7);
        const int eb = eb4[r], st = __shfl(pre, b);
        if (j < 200 && n0 < eb) {
            const uint32_t v = w[r];
            lv[st + n0] = (int16_t)(v & 0xffffu);
            if (n0 + 1 < eb) lv[st + n0 + 1] = (int16_t)(v >> 16);
        }
    }
}

// sizes_ready: the producing pass already wrote the MB sizes (pass 2 does; see
// EncArgs::sizes), so k_pack_size is skipped.
extern "C" hipError_t zwk_pack(hipStream_t s, const ZwMbOut* mbs, int nmb, int nframes, uint8_t* eobs, uint32_t* sizes,
                               unsigned long long* counter, unsigned long long* frame_info, uint8_t* out,
                               int sizes_ready)
{
    const size_t total = (size_t)nmb * nframes;
    const unsigned grid = (unsigned)((total + PK_WAVES - 1) / PK_WAVES);
    // counter: this chunk's ZW_PACK_CTR_WORDS words (zeroed at creation, reset by k_pack_scan)
    if (!sizes_ready)
        hipLaunchKernelGGL(k_pack_size, dim3(grid), dim3(64 * PK_WAVES), 0, s, mbs, nmb, nframes, eobs, sizes);
    hipLaunchKernelGGL(k_pack_scan, dim3(nframes), dim3(1024), 0, s, sizes, nmb, counter, frame_info);
    hipLaunchKernelGGL(k_pack_write, dim3(grid), dim3(64 * PK_WAVES), 0, s, mbs, nmb, nframes, eobs, sizes, frame_info,
                       out);
    return hipGetLastError();
}
