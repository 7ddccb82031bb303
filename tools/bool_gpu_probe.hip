// Latency of the VP8 bool decoder's serial chain on one GPU wave (scalar
// registers): NDEC decisions with a data-dependent probability (the decoded
// bit picks the next probability, as the token tree does), per variant.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bool_gpu_probe.hip -o tools/_bool_gpu_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

__global__ void k_probe(const uint32_t* __restrict__ words, int nwords, int ndec, int variant, uint64_t* out)
{
    uint64_t value = 0;
    uint32_t range = 254, pos = 0;
    int bits = -8;
    uint32_t prob = 128, acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ndec; i++) {
        if (bits < 0) {
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(words[pos % nwords]);
            const uint32_t w1 = __builtin_amdgcn_readfirstlane(words[(pos + 1) % nwords]);
            value = (value << 56) | ((((uint64_t)w0 << 32) | w1) >> 8);
            bits += 56;
            pos += 2;
        }
        const uint32_t split = (range * prob) >> 8;
        const uint32_t v = (uint32_t)(value >> bits);
        const bool bit = v > split;
        const uint32_t nr = bit ? range - split : split + 1;
        value = bit ? value - ((uint64_t)(split + 1) << bits) : value;
        const int shift = __builtin_clz(nr) - 24;
        bits -= shift;
        range = (nr << shift) - 1;
        acc += bit;
        if (variant == 0) prob = bit ? 200 : 60;                      // next prob from the bit (scalar select)
        else prob = (acc * 37u + 90u) & 255u | 1u;                    // arithmetic on the chain
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = t1 - t0;
        out[2 * blockIdx.x + 1] = acc;
    }
}

int main()
{
    const int nwords = 1 << 16, ndec = 1 << 20;
    std::vector<uint32_t> h(nwords);
    uint32_t x = 12345;
    for (auto& w : h) { x = x * 1664525u + 1013904223u; w = x; }
    uint32_t* d;
    uint64_t* o;
    hipMalloc(&d, nwords * 4);
    hipMalloc(&o, 16 * 256 * 2);
    hipMemcpy(d, h.data(), nwords * 4, hipMemcpyHostToDevice);
    for (int variant = 0; variant < 2; variant++)
        for (int waves : {1, 256, 1024}) {
            hipLaunchKernelGGL(k_probe, dim3(waves), dim3(64), 0, 0, d, nwords, ndec, variant, o);
            hipDeviceSynchronize();
            uint64_t r[2];
            hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
            printf("variant %d, %4d waves: %.1f cycles per decision (wave 0)\n", variant, waves, (double)r[0] / ndec);
        }
    return 0;
}
