// zw_host.cpp -- host runtime of the MI355X VP8 pipeline: context, batch
// pipeline (HBM buffers + kernel orchestration), host entropy stage, C ABI.
//
// Encode flow for a batch of frames (encode_frame_lossy, vp8.rs:1281-1488):
//   k_rgb2yuv -> k_analysis -> k_segments -> k_encode(pass 1)
//   -> D2H pass-1 MB records -> host: statistics replay, probability update,
//      level costs (one thread per frame)
//   -> H2D params/costs -> k_encode(pass 2) -> D2H pass-2 MB records
//   -> host: header + token emission (one thread per frame).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>
#include <condition_variable>
#include <mutex>
#include <new>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <limits>
#include <memory>
#include <thread>
#include <vector>

#include "../../include/zwebp.h"
#include "zw_common.h"
#include "zw_host_entropy.h"
#include "zw_host_internal.h"

extern "C" {
hipError_t zwk_rgb2yuv(hipStream_t s, const uint8_t* img, int w, int h, int bpp, int mbw, int mbh, uint8_t* Y,
                       uint8_t* U, uint8_t* V, size_t img_stride, size_t ysz, size_t csz, int nframes);
hipError_t zwk_analysis(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, int mbw, int mbh,
                        size_t ysz, size_t csz, uint8_t* alpha, uint32_t* histo, int nframes);
hipError_t zwk_segments(hipStream_t s, uint32_t* histo, const ZwFrameParams* tmpl, ZwFrameParams* params,
                        int nframes);
hipError_t zwk_stats(hipStream_t s, const ZwMbOut* mbs, int mbw, int mbh, void* scratch, void* out, int nframes);
size_t zw_stats_scratch_bytes(int nmb, int nframes);
hipError_t zwk_pack(hipStream_t s, const ZwMbOut* mbs, int nmb, int nframes, uint8_t* eobs, uint32_t* sizes,
                     unsigned long long* counter, unsigned long long* frame_info, uint8_t* out, int sizes_ready);
hipError_t zwk_fdct_quant(hipStream_t s, const void* src, const void* pred, size_t n, const ZwMatrix* m, int first,
                          void* levels, void* recon, int cus);
hipError_t zwk_xform_mb(hipStream_t s, const uint8_t* Y, const uint8_t* U, const uint8_t* V, int src_bpp, int w,
                        int h, size_t img_stride, const uint8_t* recs, const void* segs, int mbw, int mbh, int nframes,
                        int16_t* levels, uint8_t* RY, uint8_t* RU, uint8_t* RV, uint32_t* queue, int qp,
                        uint32_t* qerr, int variant);
size_t zwk_xform_mb_seg_bytes(void);
size_t zwk_xform_mb_queue_bytes(int mbw, int mbh, int nframes);
void zwk_xform_mb_pack_segs(const ZwMatrix* m, int n, void* out);
hipError_t zwk_quant_blocks(hipStream_t s, const int* coeffs, const uint8_t* ctx0s, const ZwLevelCosts* lcost,
                            const uint8_t* probs, const void* args, int* levels, int* dq);
hipError_t zwk_encode(hipStream_t s, int pass, const uint8_t* Y, const uint8_t* U, const uint8_t* V,
                      const uint8_t* alpha, const ZwFrameParams* params, const ZwLevelCosts* lcost, int8_t* derr,
                      ZwMbOut* out, uint8_t* ry, uint8_t* ru, uint8_t* rv, size_t ysz, size_t csz, int mbw, int mbh,
                      int nframes, int* dbg, uint8_t* rows, uint32_t* sizes = nullptr);
size_t zwk_encode_rows_bytes(int mbw, int mbh, int nframes);
int zwk_encode_max_mbw(int rows);
int zwk_encode_fp(int pass, int mbw, int nframes);
}

extern "C" const char* zw_strerror(int code)
{
    switch (code) {
    case ZW_OK: return "ok";
    case ZW_EINVALID_DIMENSIONS: return "invalid dimensions";
    case ZW_EINVALID_BUFFER_SIZE: return "invalid buffer size";
    case ZW_EINVAL: return "invalid argument";
    case ZW_EDEVICE: return "device error";
    case ZW_EUNSUPPORTED: return "unsupported";
    case ZW_ENOMEM: return "out of memory";
    case ZW_EVP8_MAGIC: return "invalid VP8 magic";
    case ZW_ECOLORSPACE: return "invalid VP8 color space";
    case ZW_ELUMA_MODE: return "invalid luma prediction mode";
    case ZW_EINTRA_MODE: return "invalid intra prediction mode";
    case ZW_ECHROMA_MODE: return "invalid chroma prediction mode";
    case ZW_EBITSTREAM: return "bitstream error";
    case ZW_EUNSUPPORTED_FEATURE: return "unsupported feature";
    case ZW_ENOT_ENOUGH_INIT_DATA: return "not enough VP8 init data";
    case ZW_ECHUNK_HEADER: return "invalid chunk header";
    case ZW_EWEBP_SIGNATURE: return "invalid WEBP signature";
    case ZW_ECHUNK_MISSING: return "an expected chunk was missing";
    case ZW_EINCONSISTENT_SIZES: return "inconsistent image sizes";
    case ZW_EIMAGE_TOO_LARGE: return "image too large";
    default: return "unknown error";
    }
}

// Contexts alive in the process: the decoded-frame pool (zw_dec_host.cpp) keeps
// freed frame buffers only while some context is, and the last zw_ctx_destroy
// trims it.
static std::atomic<int> g_ctx_alive{0};
bool zw_ctx_any_alive() { return g_ctx_alive.load(std::memory_order_acquire) > 0; }

extern "C" int zw_ctx_create(int device, zw_ctx** out)
{
    if (!out) return ZW_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return ZW_EDEVICE;
    HIPOK(hipSetDevice(device));
    zw_ctx* c = new zw_ctx();
    c->device = device;
    g_ctx_alive.fetch_add(1, std::memory_order_acq_rel);
    *out = c;
    return ZW_OK;
}

// ---- HSA agents of the context's device (PCI location match) and SDMA copies
struct AgentFind {
    uint32_t bdf, domain;
    hsa_agent_t gpu{}, cpu{};
    bool gpu_ok = false, cpu_ok = false;
};
static hsa_status_t find_agents_cb(hsa_agent_t a, void* data)
{
    AgentFind* F = (AgentFind*)data;
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !F->cpu_ok) {
        F->cpu = a;
        F->cpu_ok = true;
    } else if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t bdf = 0, dom = 0;
        (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        (void)hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        if (bdf == F->bdf && dom == F->domain) {
            F->gpu = a;
            F->gpu_ok = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

static int sdma_probe_locked(zw_ctx* c)
{
    if (getenv("ZW_NO_SDMA")) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) return 0;
    if (hsa_init() != HSA_STATUS_SUCCESS) return 0;  // reference-counted; HIP holds one
    AgentFind F;
    F.bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    F.domain = (uint32_t)prop.pciDomainID;
    (void)hsa_iterate_agents(find_agents_cb, &F);
    if (!F.gpu_ok || !F.cpu_ok) return 0;
    c->gpu_agent = F.gpu;
    c->cpu_agent = F.cpu;
    return 1;
}

// Resolved once per context: the first caller probes under sdma_mu, later and
// concurrent callers (pipe lanes) wait for it and then read the published agents.
static bool sdma_probe(zw_ctx* c)
{
    int st = c->sdma.load(std::memory_order_acquire);
    if (st < 0) {
        std::lock_guard<std::mutex> lk(c->sdma_mu);
        st = c->sdma.load(std::memory_order_relaxed);
        if (st < 0) {
            st = sdma_probe_locked(c);
            c->sdma.store(st, std::memory_order_release);  // publishes gpu_agent / cpu_agent
        }
    }
    return st == 1;
}

std::atomic<bool> g_dma_poisoned{false};

int ctx_d2h(zw_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (bytes == 0) return ZW_OK;
    if (c->poisoned.load(std::memory_order_acquire)) return ZW_EDEVICE;
    if (sdma_probe(c)) {
        hsa_signal_t sig;
        if (hsa_signal_create(1, 0, nullptr, &sig) == HSA_STATUS_SUCCESS) {
            const hsa_status_t st =
                hsa_amd_memory_async_copy(dst, c->cpu_agent, src, c->gpu_agent, bytes, 0, nullptr, sig);
            hsa_signal_value_t v = 1;
            // bounded wait: a copy that never completes fails the call instead of hanging it
            const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
            while (st == HSA_STATUS_SUCCESS) {
                v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 100000000ull, HSA_WAIT_STATE_BLOCKED);
                if (v == 0 || std::chrono::steady_clock::now() > deadline) break;
            }
            if (st == HSA_STATUS_SUCCESS && v != 0) {
                // timed out with the copy still queued or running: the engine may yet
                // write `dst` and decrement `sig`, so the signal is leaked, not destroyed,
                // and the context refuses every later copy
                c->poisoned.store(true, std::memory_order_release);
                g_dma_poisoned.store(true, std::memory_order_release);
                return ZW_EDEVICE;
            }
            (void)hsa_signal_destroy(sig);
            if (st == HSA_STATUS_SUCCESS) return ZW_OK;
        }
        c->sdma.store(0, std::memory_order_release);  // HSA path unusable: fall back for good
    }
    HIPOK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return ZW_OK;
}

// Host->device copy on a DMA engine, started (not waited for): `src` must be
// pinned.  The caller waits on `sig` (value 1 -> 0) with sdma_wait.
static int sdma_h2d_start(zw_ctx* c, void* dst, const void* src, size_t bytes, hsa_signal_t sig)
{
    if (c->poisoned.load(std::memory_order_acquire)) return ZW_EDEVICE;
    hsa_signal_store_relaxed(sig, 1);
    return hsa_amd_memory_async_copy(dst, c->gpu_agent, src, c->cpu_agent, bytes, 0, nullptr, sig) ==
                   HSA_STATUS_SUCCESS
               ? ZW_OK
               : ZW_EDEVICE;
}
// Bounded wait for a DMA started by sdma_h2d_start; a copy that does not
// complete poisons the context (its source staging stays allocated).
static int sdma_wait(zw_ctx* c, hsa_signal_t sig)
{
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    for (;;) {
        const hsa_signal_value_t v =
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 100000000ull, HSA_WAIT_STATE_BLOCKED);
        if (v == 0) return ZW_OK;
        if (std::chrono::steady_clock::now() > deadline) {
            c->poisoned.store(true, std::memory_order_release);
            g_dma_poisoned.store(true, std::memory_order_release);
            return ZW_EDEVICE;
        }
    }
}

// RGBA -> RGB for the host-resident upload (zw_pipe_encode_host): the VP8
// payload reads only R, G, B (convert_image_yuv, yuv.rs:656-804; the alpha
// plane goes to ALPH, which that entry point does not write), so an RGBA frame
// crosses PCIe as 3/4 of its bytes and rgb2yuv reads it as RGB.  16 pixels a
// step: four in-lane byte shuffles, spliced into three 16-byte streaming
// stores (`d` 16-byte aligned: the pinned staging slot).
__attribute__((target("ssse3"))) static void pack_rgb_ssse3(uint8_t* d, const uint8_t* s, size_t npx)
{
    const __m128i sh = _mm_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -128, -128, -128, -128);
    size_t i = 0;
    for (; i + 16 <= npx; i += 16, s += 64, d += 48) {
        const __m128i a = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)s), sh);
        const __m128i b = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(s + 16)), sh);
        const __m128i c = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(s + 32)), sh);
        const __m128i e = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(s + 48)), sh);
        _mm_stream_si128((__m128i*)d, _mm_or_si128(a, _mm_slli_si128(b, 12)));
        _mm_stream_si128((__m128i*)(d + 16), _mm_or_si128(_mm_srli_si128(b, 4), _mm_slli_si128(c, 8)));
        _mm_stream_si128((__m128i*)(d + 32), _mm_or_si128(_mm_srli_si128(c, 8), _mm_slli_si128(e, 4)));
    }
    _mm_sfence();
    for (; i < npx; i++, s += 4, d += 3) {
        d[0] = s[0];
        d[1] = s[1];
        d[2] = s[2];
    }
}
// 32 pixels a step: in-lane shuffles, each 32-byte register compacted to its 24
// bytes, three 32-byte streaming stores (`d` 32-byte aligned)
__attribute__((target("avx2"))) static void pack_rgb_avx2(uint8_t* d, const uint8_t* s, size_t npx)
{
    const __m256i sh = _mm256_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -128, -128, -128, -128, 0, 1, 2, 4, 5,
                                        6, 8, 9, 10, 12, 13, 14, -128, -128, -128, -128);
    const __m256i cp = _mm256_setr_epi32(0, 1, 2, 4, 5, 6, 3, 7);  // dwords 0-5 valid
    const __m256i ib0 = _mm256_setr_epi32(0, 0, 0, 0, 0, 0, 0, 1), ib1 = _mm256_setr_epi32(2, 3, 4, 5, 0, 0, 0, 0);
    const __m256i ic1 = _mm256_setr_epi32(0, 0, 0, 0, 0, 1, 2, 3), ic2 = _mm256_setr_epi32(4, 5, 0, 0, 0, 0, 0, 0);
    const __m256i ie2 = _mm256_setr_epi32(0, 0, 0, 1, 2, 3, 4, 5);
    size_t i = 0;
    for (; i + 32 <= npx; i += 32, s += 128, d += 96) {
        const __m256i a = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)s), sh), cp);
        const __m256i b =
            _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(s + 32)), sh), cp);
        const __m256i c =
            _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(s + 64)), sh), cp);
        const __m256i e =
            _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i*)(s + 96)), sh), cp);
        _mm256_stream_si256((__m256i*)d, _mm256_blend_epi32(a, _mm256_permutevar8x32_epi32(b, ib0), 0xC0));
        _mm256_stream_si256((__m256i*)(d + 32), _mm256_blend_epi32(_mm256_permutevar8x32_epi32(b, ib1),
                                                                   _mm256_permutevar8x32_epi32(c, ic1), 0xF0));
        _mm256_stream_si256((__m256i*)(d + 64), _mm256_blend_epi32(_mm256_permutevar8x32_epi32(c, ic2),
                                                                   _mm256_permutevar8x32_epi32(e, ie2), 0xFC));
    }
    _mm_sfence();
    for (; i < npx; i++, s += 4, d += 3) {
        d[0] = s[0];
        d[1] = s[1];
        d[2] = s[2];
    }
}
static void pack_rgb(uint8_t* d, const uint8_t* s, size_t npx)
{
    static const bool avx2 = __builtin_cpu_supports("avx2"), ssse3 = __builtin_cpu_supports("ssse3");
    if (avx2 && ((uintptr_t)d & 31) == 0) {
        pack_rgb_avx2(d, s, npx);
        return;
    }
    if (ssse3 && ((uintptr_t)d & 15) == 0) {
        pack_rgb_ssse3(d, s, npx);
        return;
    }
    for (size_t i = 0; i < npx; i++) {
        d[3 * i] = s[4 * i];
        d[3 * i + 1] = s[4 * i + 1];
        d[3 * i + 2] = s[4 * i + 2];
    }
}

// Is [p, p + n) page-locked host memory the DMA engines can read (hipHostMalloc
// or hipHostRegister)?  Then the address the agents use for p (the
// allocation's device pointer at p's offset: for registered memory it need not
// equal p), and such a frame goes to the engine directly, with no copy through
// the uploader's staging slot; else nullptr.
static const void* host_pinned(const void* p, size_t n)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // (pageable memory: not an error worth keeping)
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.hostPointer || !a.devicePointer) return nullptr;
    // the registration must cover the whole frame: its end must resolve too, to the same allocation
    hipPointerAttribute_t b;
    if (hipPointerGetAttributes(&b, (const uint8_t*)p + n - 1) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (b.type != hipMemoryTypeHost || b.hostPointer != a.hostPointer) return nullptr;
    return (const uint8_t*)a.devicePointer + ((const uint8_t*)p - (const uint8_t*)a.hostPointer);
}

int ctx_d2h_stream(zw_ctx* c, void* dst, const void* src, size_t bytes)
{
    if (bytes == 0) return ZW_OK;
    if (!c->copy_) HIPOK(hipStreamCreateWithFlags(&c->copy_, hipStreamNonBlocking));
    HIPOK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->copy_));
    // a blocking-sync event: the waiting thread sleeps instead of spinning on
    // the host CPUs (a 16-CPU quota on the box) the decode's parse needs
    // (1 024 1080p frames: 5 239-5 259 vs 4 928-5 290 decodes/s spinning)
    if (!c->copy_ev) HIPOK(hipEventCreateWithFlags(&c->copy_ev, hipEventBlockingSync | hipEventDisableTiming));
    HIPOK(hipEventRecord(c->copy_ev, c->copy_));
    HIPOK(hipEventSynchronize(c->copy_ev));
    return ZW_OK;
}

static void seam_trim(bool all);

extern "C" void zw_ctx_release_buffers(zw_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream_) (void)hipStreamSynchronize(c->stream_);  // nothing queued may still use them
    {
        std::lock_guard<std::mutex> lk(c->pipe1_mu);
        zw_pipe_destroy(c->pipe1);
        c->pipe1 = nullptr;
    }
    for (auto& v : c->dec_recs) std::vector<zw_ctx::RecBuf>().swap(v);
    zw_dec_pool_trim();  // the decoded-frame buffers callers have already freed
    seam_trim(false);    // the idle pipelines concurrent single-frame calls shared
    if (c->dscratch) (void)hipFree(c->dscratch);
    if (c->dscratch1) (void)hipFree(c->dscratch1);
    if (c->tok_) (void)hipStreamSynchronize(c->tok_);
    if (c->dscratch2) (void)hipFree(c->dscratch2);
    if (c->dscratch3) (void)hipFree(c->dscratch3);
    c->dscratch = c->dscratch1 = c->dscratch2 = c->dscratch3 = nullptr;
    c->dscratch2_cap = c->dscratch3_cap = 0;
    (void)hipDeviceSynchronize();  // queues may serve streams other than the context's
    for (auto& q : c->xmb_q)
        if (q.buf) (void)hipFree(q.buf);
    c->xmb_q.clear();
    c->dscratch_cap = c->dscratch1_cap = 0;
    for (int i = 0; i < 5; i++) {
        pinned_free(c->hpin[i]);
        c->hpin[i] = nullptr;
        c->hpin_cap[i] = 0;
    }
}

extern "C" void zw_ctx_destroy(zw_ctx* c)
{
    if (!c) return;
    zw_ctx_free_internal(c);
    if (g_ctx_alive.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        seam_trim(true);
        zw_dec_pool_trim();
    }
}

// Everything a context holds (the user contexts' zw_ctx_destroy, and the seam's
// internal contexts, which are not counted as alive).
void zw_ctx_free_internal(zw_ctx* c)
{
    (void)hipSetDevice(c->device);
    zw_pipe_destroy(c->pipe1);
    if (c->dscratch) (void)hipFree(c->dscratch);
    if (c->dscratch1) (void)hipFree(c->dscratch1);
    if (c->tok_) (void)hipStreamSynchronize(c->tok_);
    if (c->dscratch2) (void)hipFree(c->dscratch2);
    if (c->dscratch3) (void)hipFree(c->dscratch3);
    pinned_free(c->tok_total);
    for (auto& q : c->xmb_q)
        if (q.buf) (void)hipFree(q.buf);
    if (c->xmb_err) (void)hipHostFree((void*)c->xmb_err);
    for (hipEvent_t e : c->tok_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->dev_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->dev_ev1)
        if (e) (void)hipEventDestroy(e);
    for (void* h : c->hpin) pinned_free(h);
    if (c->stream_) (void)hipStreamDestroy(c->stream_);
    if (c->copy_) (void)hipStreamDestroy(c->copy_);
    if (c->copy_ev) (void)hipEventDestroy(c->copy_ev);
    if (c->tok_) (void)hipStreamDestroy(c->tok_);
    delete c;
}

extern "C" void zw_bytes_free(zw_bytes* b)
{
    if (b && b->data) {
        if (!zw_dec_pool_put(b->data)) free(b->data);
        b->data = nullptr;
        b->len = 0;
    }
}

// --------------------------------------------------------------------------
// Batch pipeline
//
// The frames of a pipe are split into up to ZW_PIPE_LANES lanes (default 4,
// the number of hardware queues HIP uses per process).  Each lane owns a HIP
// stream and runs the sequential per-frame flow on its slice:
//   rgb2yuv, analysis, segments, pass 1 -> pack + D2H -> host stats/probs ->
//   H2D -> pass 2 -> pack + D2H -> host token emission.
// Lanes run concurrently (one host thread each), so one lane's host stages
// overlap the other lanes' kernels and the GPU stays busy.
// --------------------------------------------------------------------------
// Pinned host array: copies to/from pageable memory are staged and can
// synchronise with unrelated device work, so every async copy of the pipeline
// goes through page-locked buffers.
template <class T>
struct Pinned {
    T* p = nullptr;
    size_t n = 0;
    bool alloc(size_t count)
    {
        free();
        if (hipHostMalloc((void**)&p, count * sizeof(T) + 64, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return false;
        }
        n = count;
        memset((void*)p, 0, count * sizeof(T));
        return true;
    }
    void free()
    {
        pinned_free(p);
        p = nullptr;
        n = 0;
    }
    T* data() { return p; }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    size_t size() const { return n; }
    ~Pinned() { free(); }
};

// Pinned landing buffers of packed MB streams fetched from the device.
struct FetchBuf {
    uint8_t* pack = nullptr;
    size_t cap = 0;
    Pinned<unsigned long long> finfo;  // [2*chunk] offset, bytes of each frame's packed stream
    Pinned<unsigned long long> total;  // [1] bytes of the chunk
    void release()
    {
        pinned_free(pack);
        pack = nullptr;
        cap = 0;
    }
};

struct PipeLane {
    int f0 = 0, n = 0;  // frame slice
    int chunk = 0;      // frames per chunk (kernels are launched per chunk)
    hipStream_t stream = nullptr;   // kernels of the lane
    hipStream_t stream2 = nullptr;  // packing + copies (runs beside the next chunk's kernels)
    std::vector<hipEvent_t> cev;    // per chunk: [p1 done, p2 done]
    hipEvent_t ev[8] = {};
    unsigned long long* d_ctr = nullptr;
    uint8_t* d_rows = nullptr;  // row-parallel encode scratch (small chunks), else null
    // [0] pass-1 records (host stats replay), [1], [2] pass-2 records of the
    // emission thread (chunk c in fb[1 + (c & 1)]: with pass 2 of two chunks in
    // one launch, both are copied out before either is emitted)
    FetchBuf fb[3];
    Pinned<ZwStatsOut> h_stats;          // [chunk] pass-1 statistics from k_stats
    float kms[4] = {0, 0, 0, 0};
    double hms[4] = {0, 0, 0, 0};  // host ms: fetch1, stats, fetch2, emit
    double emit_cpu_ms = 0;        // thread CPU ms of the emission workers per batch
    // Pass 2 in frame pairs (k_encode_pass2_fp: two frames a workgroup, so a
    // launch fills the CUs with two frames per CU): chunks 2k and 2k + 1 take
    // pass 2 in one launch, pass 1 and the statistics stay per chunk.
    bool pair2 = false;
    int p2_frames = 0;  // frames of the timed pass-2 launch (kms[3] is scaled to one chunk)
    bool pair1 = false;  // the same for pass 1 (k_encode_pass1_fp)
    int p1_frames = 0;
    int rc = 0;
    // Host-source streaming (zw_pipe_encode_host): the lane's uploader thread
    // copies batch b's frames into input buffer b & 1 on `ustream`, one event
    // per chunk (uev); the kernel stream waits for it before rgb2yuv and records
    // rev once rgb2yuv has read the buffer, which the upload of batch b + 2 waits for.
    // U uploaders per lane (frames i % U == u of every chunk), each with its own
    // stream and events uev[parity][u * nch + c]: a pageable copy costs its
    // calling thread about a millisecond per 1080p frame (pinning / staging).
    std::vector<hipStream_t> ustreams;
    std::vector<hipEvent_t> uev[2], rev[2];
    std::vector<long long> uploaded;  // per uploader: chunks issued (over all batches), under sync->mu
    long long p1_queued = 0;
    // DMA-engine uploads (the default when the HSA agents resolve): per uploader
    // two pinned frame slots and their completion signals.  HIP's own H2D of
    // large copies runs as a blit kernel, which waits for CUs the encode
    // launches hold, so it would not overlap them.
    std::vector<uint8_t*> ustage;      // [2 * U]
    std::vector<hsa_signal_t> usig;    // [2 * U]
    // Emission runs on its own thread, one batch behind the lane thread.
    // `fetched` counts the chunks whose pass-2 records it has copied out
    // (over all batches): pass 2 of the next batch may then reuse the chunk's
    // device buffers.  fetched = LLONG_MAX once the emitter failed.
    struct Sync {
        std::mutex mu;
        std::condition_variable cv;
        long long fetched = 0;
    };
    std::unique_ptr<Sync> sync = std::make_unique<Sync>();
};

struct zw_pipe {
    zw_ctx* ctx;
    int n, w, h, color, bpp, quality, method, mbw, mbh, nmb, qi, filter;
    size_t img_stride, ysz, csz;
    uint8_t *d_img = nullptr, *d_Y = nullptr, *d_U = nullptr, *d_V = nullptr;
    uint8_t *d_ry = nullptr, *d_ru = nullptr, *d_rv = nullptr, *d_alpha = nullptr;
    uint32_t* d_histo = nullptr;
    ZwFrameParams *d_tmpl = nullptr, *d_params = nullptr;
    ZwLevelCosts* d_lcost = nullptr;
    int8_t* d_derr = nullptr;
    ZwMbOut *d_out1 = nullptr, *d_out2 = nullptr;
    int* d_dbg = nullptr;  // optional pass-2 I4 dump
    ZwStatsOut* d_stats = nullptr;  // pass-1 statistics (zwk_stats)
    void* d_stats_tmp = nullptr;    // zwk_stats scratch (flags, stripe partials)
    bool host_stats = false;        // ZW_HOST_STATS=1: replay the statistics on the host instead
    // packed MB streams (zw_pack_kernels.hip)
    uint8_t* d_eobs = nullptr;
    uint32_t* d_sizes = nullptr;
    unsigned long long *d_finfo = nullptr, *d_finfo2 = nullptr;  // pass-1 / pass-2 packed streams
    uint8_t *d_pack = nullptr, *d_pack2 = nullptr;
    size_t pack_stride = 0;  // worst-case packed bytes per frame
    // Per-frame header state, two copies by batch parity: the statistics of
    // batch b+1 are built while batch b is still being emitted.
    Pinned<ZwFrameParams> h_params;  // [2][n]
    Pinned<ZwLevelCosts> h_lcost;
    std::vector<uint8_t> h_have_upd;  // [2][n]
    std::vector<uint8_t> h_upd;       // [2][n][4*8*3*11]
    int out_par = 0;                  // parity of the last emitted batch
    std::vector<std::vector<uint8_t>> bitstreams;
    // container output (zw_pipe_set_container): RIFF/VP8X per frame, the ALPH
    // chunk of an LA8 / RGBA8 frame encoded from its host copy
    bool container = false;
    std::vector<const uint8_t*> host_frames;
    int nparts = 1;  // token partitions per frame (zw_pipe_set_token_partitions)
    std::vector<PipeLane> lanes;
    // Cross-lane order of the pass-1 launches (lane_encode, ZW_P1_ORDER): lane
    // g's pass 1 of a batch waits for lane g - 1's statistics kernels of that
    // batch (lane 0: of the previous batch).  Otherwise a lane's statistics,
    // queued behind its own pass 1, wait for CUs until the other lane's whole
    // pass-1 launch ends, and its pass 2 after them (measured: ~30 ms of idle
    // GPU a step).  p1_stats[g]: batches whose statistics lane g has queued
    // (its event L.ev[6] recorded after them); INT64_MAX once the lane stopped.
    std::mutex p1_mu;
    std::condition_variable p1_cv;
    std::vector<long long> p1_stats;
    float kms[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    // emission workspaces (chunk_emit): one per concurrent group task at most
    std::mutex ews_mu;
    std::vector<std::unique_ptr<zwh::EmitWs>> ews;
    // Set when a run stops partway: k_segments' histograms and k_pack_scan's
    // counters, which the kernels clear themselves, may then be left nonzero,
    // so every later run of this pipe fails instead of reading them.
    bool broken = false;
    // zw_pipe_encode_host: second input buffer and the host frames of the call
    // (batch b, frame i at host_src[b * n + i]); null outside such a call
    uint8_t* d_img2 = nullptr;
    const uint8_t* const* host_src = nullptr;
    // RGBA frames staged as RGB (pack_rgb) and converted from that: set for a
    // zw_pipe_encode_host call on the DMA-staging path (ZW_UPLOAD_PACK=0: off)
    bool up_pack = false;
    uint8_t* img_buf(int parity) const { return parity ? d_img2 : d_img; }
};

static void pipe_free(zw_pipe* p)
{
    if (!p) return;
    // an upload DMA that timed out (the context is poisoned) may still write the
    // input buffers: they are leaked rather than handed back to the allocator
    if (p->ctx && p->ctx->poisoned.load(std::memory_order_acquire)) p->d_img = p->d_img2 = nullptr;
    void* ptrs[] = {p->d_img, p->d_img2, p->d_Y, p->d_U, p->d_V, p->d_ry, p->d_ru, p->d_rv, p->d_alpha, p->d_histo,
                    p->d_tmpl, p->d_params, p->d_lcost, p->d_derr, p->d_out1, p->d_out2, p->d_dbg,
                    p->d_eobs, p->d_sizes, p->d_finfo, p->d_pack, p->d_finfo2, p->d_pack2, p->d_stats, p->d_stats_tmp};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    for (PipeLane& L : p->lanes) {
        if (L.d_ctr) (void)hipFree(L.d_ctr);
        if (L.d_rows) (void)hipFree(L.d_rows);
        for (FetchBuf& b : L.fb) b.release();
        for (int i = 0; i < 8; i++)
            if (L.ev[i]) (void)hipEventDestroy(L.ev[i]);
        for (hipEvent_t e : L.cev)
            if (e) (void)hipEventDestroy(e);
        if (L.stream) (void)hipStreamDestroy(L.stream);
        if (L.stream2) (void)hipStreamDestroy(L.stream2);
        for (hipStream_t u : L.ustreams) (void)hipStreamDestroy(u);
        for (uint8_t* b : L.ustage) pinned_free(b);
        if (!g_dma_poisoned.load())
            for (hsa_signal_t sg : L.usig) (void)hsa_signal_destroy(sg);
        for (int k = 0; k < 2; k++) {
            for (hipEvent_t e : L.uev[k])
                if (e) (void)hipEventDestroy(e);
            for (hipEvent_t e : L.rev[k])
                if (e) (void)hipEventDestroy(e);
        }
    }
    delete p;
}

// Lanes: independent halves of the batch, each with its own kernel and copy
// streams.  Two lanes by default once each gets at least one full launch (one
// frame per CU): their launches overlap, so the CUs a launch's early frames
// free start the other lane's work instead of idling until its slowest frame
// ends (measured, 1024 1080p frames: 3 015 -> 3 087 encodes/s; three lanes no
// better).  ZW_PIPE_LANES overrides.
static int pipe_lanes_for(int n, int device, int mbw)
{
    const char* e = getenv("ZW_PIPE_LANES");
    int g;
    if (e && *e) {
        g = atoi(e);
    } else {
        hipDeviceProp_t prop;
        const int cus = hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0
                            ? prop.multiProcessorCount
                            : 256;
        // where the passes run in frame pairs a lane needs two chunks (two
        // frames per CU) for them: a second lane only from four chunks
        const bool fp = zwk_encode_fp(2, mbw, 2 * cus) != 0;
        g = n >= (fp ? 4 : 2) * cus ? 2 : 1;
    }
    if (g < 1) g = 1;
    if (g > 16) g = 16;
    while (g > 1 && n / g < 8) g--;  // keep >= 8 frames per lane
    return g;
}
// Frames per kernel launch inside a lane: one encode workgroup occupies a
// whole CU (768 threads x 168 VGPRs), so a launch of one frame per CU fills
// the device; the lane runs pass 1 of chunk c+1 while the host works on chunk c.
// (Pass 2 may take two chunks in one launch: PipeLane::pair2.)
static int pipe_chunk_for(int lane_frames, int device)
{
    const char* e = getenv("ZW_PIPE_CHUNK");
    int c = e ? atoi(e) : 0;
    if (c < 1) {
        hipDeviceProp_t prop;
        c = hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0
                ? prop.multiProcessorCount
                : 256;
    }
    return c > lane_frames ? lane_frames : c;
}
// Row-parallel encode kernels (one wave per MB row, spread over the CUs) for
// chunks too small to fill the device with one 12-wave workgroup per frame.
// ZW_ENC_ROWS=0/1 forces either shape.
static bool pipe_rows_for(int chunk, int mbw, int mbh, int device)
{
    static const int batch_max_mbw = zwk_encode_max_mbw(0);
    if (mbw > batch_max_mbw) return true;  // the batch shapes cannot hold the frame's rows in LDS
    const char* e = getenv("ZW_ENC_ROWS");
    if (e && *e) return atoi(e) != 0;
    hipDeviceProp_t prop;
    const int cus = hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0
                        ? prop.multiProcessorCount
                        : 256;
    return (long long)chunk * (mbh + 1) <= 12LL * cus;  // measured: rows win up to ~48 1080p frames
}

// encode_frame_lossy's dimension rule (vp8.rs:3143-3148): any u16, the header
// keeping the low 14 bits (vp8.rs:326-327; zwh::emit_frame does the same).
// Zero is refused (the reference has no meaningful zero-MB frame).  Frames
// wider than the batch kernels' LDS takes (zwk_encode_max_mbw(0), 1 568 MBs)
// run the row-parallel kernels, whose LDS holds any u16 width.
static bool encode_dims_ok(uint32_t width, uint32_t height)
{
    if (width == 0 || height == 0 || width > 65535 || height > 65535) return false;
    static const int max_mbw = zwk_encode_max_mbw(1);
    return (int)((width + 15) / 16) <= max_mbw;
}

extern "C" int zw_pipe_create(zw_ctx* ctx, int n, uint32_t width, uint32_t height, int color, uint8_t quality,
                              uint8_t method, zw_pipe** out)
{
    if (!ctx || !out || n <= 0) return ZW_EINVAL;
    *out = nullptr;
    if (!encode_dims_ok(width, height)) return ZW_EINVALID_DIMENSIONS;
    if (color < 0 || color > 3) return ZW_EINVAL;
    if (quality > 100) return ZW_EINVAL;
    HIPOK(hipSetDevice(ctx->device));
    zw_pipe* p = new zw_pipe();
    p->ctx = ctx;
    p->n = n;
    p->w = (int)width;
    p->h = (int)height;
    p->color = color;
    static const int bpp_of[4] = {1, 2, 3, 4};
    p->bpp = bpp_of[color];
    p->quality = quality;
    p->method = method > 6 ? 6 : method;
    p->mbw = (p->w + 15) / 16;
    p->mbh = (p->h + 15) / 16;
    p->nmb = p->mbw * p->mbh;
    p->img_stride = (size_t)p->w * p->h * p->bpp;
    p->ysz = (size_t)p->mbw * 16 * p->mbh * 16;
    p->csz = (size_t)p->mbw * 8 * p->mbh * 8;
    p->qi = zwh::quality_to_qi(quality);
    p->filter = zwh::filter_level_for(p->qi);
    p->pack_stride = (size_t)p->nmb * (1 + 8 + 25 + 800);
    const size_t N = (size_t)n;
    bool ok = hipMalloc(&p->d_img, N * p->img_stride + 64) == hipSuccess &&
              hipMalloc(&p->d_Y, N * p->ysz) == hipSuccess && hipMalloc(&p->d_U, N * p->csz) == hipSuccess &&
              hipMalloc(&p->d_V, N * p->csz) == hipSuccess && hipMalloc(&p->d_ry, N * p->ysz) == hipSuccess &&
              hipMalloc(&p->d_ru, N * p->csz) == hipSuccess && hipMalloc(&p->d_rv, N * p->csz) == hipSuccess &&
              hipMalloc(&p->d_alpha, N * p->nmb) == hipSuccess &&
              hipMalloc(&p->d_histo, N * 256 * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&p->d_tmpl, sizeof(ZwFrameParams)) == hipSuccess &&
              hipMalloc(&p->d_params, N * sizeof(ZwFrameParams)) == hipSuccess &&
              hipMalloc(&p->d_lcost, N * sizeof(ZwLevelCosts)) == hipSuccess &&
              hipMalloc(&p->d_derr, N * p->mbw * 4) == hipSuccess &&
              hipMalloc(&p->d_out1, N * p->nmb * sizeof(ZwMbOut)) == hipSuccess &&
              hipMalloc(&p->d_out2, N * p->nmb * sizeof(ZwMbOut)) == hipSuccess &&
              hipMalloc(&p->d_eobs, N * p->nmb * 25) == hipSuccess &&
              hipMalloc(&p->d_sizes, N * p->nmb * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&p->d_finfo, N * 2 * sizeof(unsigned long long)) == hipSuccess &&
              hipMalloc(&p->d_pack, N * p->pack_stride) == hipSuccess &&
              hipMalloc(&p->d_finfo2, N * 2 * sizeof(unsigned long long)) == hipSuccess &&
              hipMalloc(&p->d_pack2, N * p->pack_stride) == hipSuccess;
    // Pass-1 statistics are pre-aggregated on the device (zwk_stats) unless
    // ZW_HOST_STATS asks for the host replay of the packed records.
    // k_segments clears each frame's histogram after use; k_pack_scan resets its counters
    ok = ok && hipMemset(p->d_histo, 0, N * 256 * sizeof(uint32_t)) == hipSuccess;
    p->host_stats = getenv("ZW_HOST_STATS") != nullptr;
    ok = ok && (p->host_stats || (hipMalloc(&p->d_stats, N * sizeof(ZwStatsOut)) == hipSuccess &&
                                  hipMalloc(&p->d_stats_tmp, zw_stats_scratch_bytes(p->nmb, n)) == hipSuccess));
    const int G = pipe_lanes_for(n, ctx->device, p->mbw);
    p->lanes.resize(G);
    for (int g = 0; ok && g < G; g++) {
        PipeLane& L = p->lanes[g];
        L.f0 = (int)((long long)n * g / G);
        L.n = (int)((long long)n * (g + 1) / G) - L.f0;
        L.chunk = pipe_chunk_for(L.n, ctx->device);
        for (FetchBuf& b : L.fb) ok = ok && b.finfo.alloc(2 * (size_t)L.chunk) && b.total.alloc(1);
        ok = ok && (p->host_stats || L.h_stats.alloc((size_t)L.n));
        const int nch = (L.n + L.chunk - 1) / L.chunk;
        L.cev.assign(2 * (size_t)nch, nullptr);
        ok = ok && hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking) == hipSuccess &&
             hipStreamCreateWithFlags(&L.stream2, hipStreamNonBlocking) == hipSuccess &&
             hipMalloc(&L.d_ctr, 2 * (size_t)nch * ZW_PACK_CTR_WORDS * sizeof(unsigned long long)) == hipSuccess &&
             hipMemset(L.d_ctr, 0, 2 * (size_t)nch * ZW_PACK_CTR_WORDS * sizeof(unsigned long long)) == hipSuccess;
        if (ok && pipe_rows_for(L.chunk, p->mbw, p->mbh, ctx->device)) {
            const size_t rb = zwk_encode_rows_bytes(p->mbw, p->mbh, L.chunk);
            ok = hipMalloc(&L.d_rows, rb) == hipSuccess && hipMemset(L.d_rows, 0, rb) == hipSuccess;
            // test hook (ZW_ENC_FORCE_ERROR=1): pre-set the launch error word, as a
            // wave that gave up waiting would, so the host-side check is exercised
            if (ok && getenv("ZW_ENC_FORCE_ERROR")) ok = hipMemset(L.d_rows, 1, 1) == hipSuccess;
        }
        // pass 2 of chunks (2k, 2k + 1) in one launch where it runs in frame pairs
        L.pair2 = ok && !L.d_rows && nch >= 2 && zwk_encode_fp(2, p->mbw, 2 * L.chunk);
        L.pair1 = ok && !L.d_rows && nch >= 2 && zwk_encode_fp(1, p->mbw, 2 * L.chunk);
        for (int i = 0; ok && i < 8; i++) ok = hipEventCreate(&L.ev[i]) == hipSuccess;
        for (size_t i = 0; ok && i < L.cev.size(); i++)
            ok = hipEventCreateWithFlags(&L.cev[i], hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) {
        pipe_free(p);
        return ZW_ENOMEM;
    }
    if (!p->h_params.alloc(2 * N) || !p->h_lcost.alloc(N)) {
        pipe_free(p);
        return ZW_ENOMEM;
    }
    p->h_have_upd.assign(2 * N, 0);
    p->h_upd.assign(2 * N * 4 * 8 * 3 * 11, 0);
    p->bitstreams.resize(N);
    ZwFrameParams t;
    memset(&t, 0, sizeof t);
    t.width = p->w;
    t.height = p->h;
    t.mbw = p->mbw;
    t.mbh = p->mbh;
    t.method = p->method;
    t.do_trellis = p->method >= 4;
    t.base_qi = p->qi;
    t.filter_level = p->filter;
    t.skip_prob = 200;
    memcpy(t.probs, zwh::COEFF_PROBS, sizeof t.probs);
    if (hipMemcpy(p->d_tmpl, &t, sizeof t, hipMemcpyHostToDevice) != hipSuccess) {
        pipe_free(p);
        return ZW_EDEVICE;
    }
    *out = p;
    return ZW_OK;
}

extern "C" void zw_pipe_destroy(zw_pipe* p)
{
    if (p) (void)hipSetDevice(p->ctx->device);
    pipe_free(p);
}

extern "C" void* zw_pipe_input_device_ptr(zw_pipe* p) { return p ? p->d_img : nullptr; }

extern "C" int zw_pipe_set_container(zw_pipe* p, int enable, const uint8_t* const* host_frames)
{
    if (!p) return ZW_EINVAL;
    if (!enable) {
        p->container = false;
        p->host_frames.clear();
        return ZW_OK;
    }
    const bool has_alpha = p->color == ZW_COLOR_LA8 || p->color == ZW_COLOR_RGBA8;
    if (has_alpha) {
        // encode_alpha_lossless refuses > 16384 (api.rs:1187): InvalidDimensions
        // up front, not a VP8X file with an empty ALPH chunk
        if (p->w > 16384 || p->h > 16384) return ZW_EINVALID_DIMENSIONS;
        if (!host_frames) return ZW_EINVAL;
        for (int i = 0; i < p->n; i++)
            if (!host_frames[i]) return ZW_EINVAL;
        p->host_frames.assign(host_frames, host_frames + p->n);
    }
    p->container = true;
    return ZW_OK;
}

extern "C" int zw_pipe_set_token_partitions(zw_pipe* p, int nparts)
{
    if (!p || (nparts != 1 && nparts != 2 && nparts != 4 && nparts != 8)) return ZW_EINVAL;
    p->nparts = nparts;
    return ZW_OK;
}

extern "C" int zw_pipe_upload(zw_pipe* p, int frame, const uint8_t* data, size_t len)
{
    if (!p || frame < 0 || frame >= p->n || !data) return ZW_EINVAL;
    if (len != p->img_stride) return ZW_EINVALID_BUFFER_SIZE;
    HIPOK(hipMemcpy(p->d_img + (size_t)frame * p->img_stride, data, len, hipMemcpyHostToDevice));
    return ZW_OK;
}

static double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// CPU time the calling thread has run (ns)
static long long thread_cpu_ns()
{
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

// Zero the row-parallel kernels' per-frame tickets, progress and row state
// before a launch of n frames.  The launch header (error word) is not cleared:
// a wave that gave up waiting leaves it set, and rows_check fails the call.
static hipError_t rows_reset(zw_pipe* p, PipeLane& L, int n)
{
    if (!L.d_rows) return hipSuccess;
    const size_t hdr = zwk_encode_rows_bytes(p->mbw, p->mbh, 0);
    return hipMemsetAsync(L.d_rows + hdr, 0, zwk_encode_rows_bytes(p->mbw, p->mbh, n) - hdr, L.stream);
}
static int rows_check(zw_pipe* p, PipeLane& L)
{
    if (!L.d_rows) return ZW_OK;
    int err = 0;
    HIPOK(hipMemcpy(&err, L.d_rows, sizeof err, hipMemcpyDeviceToHost));
    return err ? ZW_EDEVICE : ZW_OK;
}

// ---- per-chunk stages (frames [fa, fa + na) of a lane) ----
// Pass 1 of frames [fa, fa + na): the encode launch alone (chunk_pass1 queues
// the steps before it; a paired lane launches two chunks' pass 1 at once).
static int chunk_pass1_encode(zw_pipe* p, PipeLane& L, int fa, int na, bool timed, bool write_recon = false)
{
    hipStream_t s = L.stream;
    const size_t F = (size_t)fa;
    if (timed) {
        HIPOK(hipEventRecord(L.ev[2], s));
        L.p1_frames = na;
    }
    HIPOK(rows_reset(p, L, na));
    HIPOK(zwk_encode(s, 1, p->d_Y + F * p->ysz, p->d_U + F * p->csz, p->d_V + F * p->csz, p->d_alpha + F * p->nmb,
                     p->d_params + F, nullptr, p->d_derr + F * p->mbw * 4, p->d_out1 + F * p->nmb,
                     write_recon ? p->d_ry + F * p->ysz : nullptr, write_recon ? p->d_ru + F * p->csz : nullptr,
                     write_recon ? p->d_rv + F * p->csz : nullptr, p->ysz, p->csz, p->mbw, p->mbh, na, nullptr,
                     L.d_rows));
    if (timed) HIPOK(hipEventRecord(L.ev[3], s));
    return ZW_OK;
}

static int chunk_pass1(zw_pipe* p, PipeLane& L, int fa, int na, bool timed, bool write_recon = false,
                       int parity = 0, hipEvent_t uploaded = nullptr, hipEvent_t read = nullptr, bool encode = true)
{
    hipStream_t s = L.stream;
    const size_t F = (size_t)fa;
    const int n = na;
    if (uploaded) HIPOK(hipStreamWaitEvent(s, uploaded, 0));
    if (timed) HIPOK(hipEventRecord(L.ev[0], s));
    const bool packed = uploaded && p->up_pack;  // (this chunk's frames arrived as RGB)
    HIPOK(zwk_rgb2yuv(s, p->img_buf(parity) + F * p->img_stride, p->w, p->h, packed ? 3 : p->bpp, p->mbw, p->mbh,
                      p->d_Y + F * p->ysz, p->d_U + F * p->csz, p->d_V + F * p->csz, p->img_stride, p->ysz, p->csz,
                      n));
    if (read) HIPOK(hipEventRecord(read, s));
    if (timed) HIPOK(hipEventRecord(L.ev[1], s));
    HIPOK(zwk_analysis(s, p->d_Y + F * p->ysz, p->d_U + F * p->csz, p->d_V + F * p->csz, p->mbw, p->mbh, p->ysz,
                       p->csz, p->d_alpha + F * p->nmb, p->d_histo + F * 256, n));
    HIPOK(zwk_segments(s, p->d_histo + F * 256, p->d_tmpl, p->d_params + F, n));
    if (!encode) return ZW_OK;
    return chunk_pass1_encode(p, L, fa, na, timed, write_recon);
}

// Pass 2 writes each MB's packed record size (EncArgs::sizes), so packing
// its records skips k_pack_size.  ZW_PASS2_SIZES=0 restores the separate kernel.
static bool pass2_sizes(const zw_pipe* p)
{
    static const bool on = []() {
        const char* e = getenv("ZW_PASS2_SIZES");
        return !(e && atoi(e) == 0);
    }();
    return on && p->d_sizes != nullptr;
}

// Pack the chunk's MB records on the kernel stream (right after the pass that
// produced them: the encode kernels occupy every CU, so a pack kernel queued
// elsewhere would wait for the next chunk's pass).  slot: 2*chunk + pass-1.
static int chunk_pack(zw_pipe* p, PipeLane& L, int fa, int na, const ZwMbOut* d_out, int slot)
{
    const size_t F = (size_t)fa;
    const bool p2 = slot & 1;  // pass-2 streams have their own buffers (a later batch's pass 1 may overwrite
                               // the pass-1 buffers while the host is still fetching pass-2 data)
    HIPOK(zwk_pack(L.stream, d_out + F * p->nmb, p->nmb, na, p->d_eobs + F * p->nmb * 25, p->d_sizes + F * p->nmb,
                   L.d_ctr + ZW_PACK_CTR_WORDS * slot, (p2 ? p->d_finfo2 : p->d_finfo) + 2 * F,
                   (p2 ? p->d_pack2 : p->d_pack) + F * p->pack_stride, p2 && pass2_sizes(p)));
    return ZW_OK;
}

// Copy a packed chunk into B once `ready` (recorded after chunk_pack) has
// fired.  B.finfo[2*i] = offset of frame fa+i in B.pack.
static int chunk_fetch(zw_pipe* p, PipeLane& L, FetchBuf& B, int fa, int na, int slot, hipEvent_t ready)
{
    const size_t F = (size_t)fa;
    HIPOK(hipEventSynchronize(ready));
    int r = ctx_d2h(p->ctx, B.total.data(), L.d_ctr + ZW_PACK_CTR_WORDS * slot + 2, sizeof(unsigned long long));
    const bool p2 = slot & 1;
    if (!r)
        r = ctx_d2h(p->ctx, B.finfo.data(), (p2 ? p->d_finfo2 : p->d_finfo) + 2 * F,
                    2 * (size_t)na * sizeof(unsigned long long));
    if (r) return r;
    const unsigned long long total = B.total[0];
    if (total > B.cap) {
        B.release();
        const size_t cap = (size_t)(total * 1.25) + 4096;
        if (hipHostMalloc((void**)&B.pack, cap, hipHostMallocDefault) != hipSuccess) return ZW_ENOMEM;
        B.cap = cap;
    }
    return ctx_d2h(p->ctx, B.pack, (p2 ? p->d_pack2 : p->d_pack) + F * p->pack_stride, total);
}

// Fetch the chunk's k_stats output (device pre-aggregated ProbaStats) once
// `ready` (recorded after zwk_stats) has fired.  h_stats[i] = frame fa+i.
static int chunk_fetch_stats(zw_pipe* p, PipeLane& L, int fa, int na, hipEvent_t ready)
{
    HIPOK(hipEventSynchronize(ready));
    return ctx_d2h(p->ctx, L.h_stats.data() + (fa - L.f0), p->d_stats + fa, (size_t)na * sizeof(ZwStatsOut));
}

// Header state of frame f in the batch-parity copy `par`.
static inline size_t hidx(const zw_pipe* p, int par, size_t f) { return (size_t)par * p->n + f; }

static int chunk_stats(zw_pipe* p, PipeLane& L, int fa, int na, int par)
{
    hipStream_t s = L.stream;
    const size_t F = (size_t)fa, n = (size_t)na;
    ZwFrameParams* hp = p->h_params.data() + hidx(p, par, F);
    // segment params of the chunk (written by k_segments before pass 1)
    {
        const int r = ctx_d2h(p->ctx, hp, p->d_params + F, n * sizeof(ZwFrameParams));
        if (r) return r;
    }
    parallel_for(na, [&](int i) {
        const size_t f = F + i, hf = hidx(p, par, f);
        zwh::Stats st;
        int sp;
        if (p->host_stats) {
            sp = zwh::replay_stats(st, L.fb[0].pack + L.fb[0].finfo[2 * i], p->mbw, p->mbh);
        } else {
            const ZwStatsOut& so = L.h_stats[f - L.f0];
            memcpy(st.s, so.s, sizeof st.s);
            sp = zwh::skip_prob(so.total_mbs, so.nonzero_mbs);
        }
        uint8_t* upd = p->h_upd.data() + hf * 4 * 8 * 3 * 11;
        bool have = zwh::updated_probs(st, (uint8_t(*)[8][3][11])upd);
        p->h_have_upd[hf] = have;
        ZwFrameParams& P = p->h_params[hf];
        P.skip_prob = sp;
        memcpy(P.probs, upd, sizeof P.probs);
        zwh::level_costs(p->h_lcost[f], (const uint8_t(*)[8][3][11])upd);
    });
    HIPOK(hipMemcpyAsync(p->d_params + F, hp, n * sizeof(ZwFrameParams), hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(p->d_lcost + F, p->h_lcost.data() + F, n * sizeof(ZwLevelCosts), hipMemcpyHostToDevice, s));
    return ZW_OK;
}

static int chunk_pass2(zw_pipe* p, PipeLane& L, int fa, int na, bool timed)
{
    hipStream_t s = L.stream;
    const size_t F = (size_t)fa;
    if (timed) {
        HIPOK(hipEventRecord(L.ev[4], s));
        L.p2_frames = na;
    }
    HIPOK(rows_reset(p, L, na));
    HIPOK(zwk_encode(s, 2, p->d_Y + F * p->ysz, p->d_U + F * p->csz, p->d_V + F * p->csz, p->d_alpha + F * p->nmb,
                     p->d_params + F, p->d_lcost + F, p->d_derr + F * p->mbw * 4, p->d_out2 + F * p->nmb,
                     p->d_ry + F * p->ysz, p->d_ru + F * p->csz, p->d_rv + F * p->csz, p->ysz, p->csz, p->mbw, p->mbh,
                     na, p->d_dbg ? p->d_dbg + F * p->nmb * 16 * 34 : nullptr, L.d_rows,
                     pass2_sizes(p) ? p->d_sizes + F * p->nmb : nullptr));
    if (timed) HIPOK(hipEventRecord(L.ev[5], s));
    return ZW_OK;
}

// One frame's VP8 bitstream from its pass-2 records.  With token partitions
// and a chunk of one frame (a single-frame call) the partitions are coded on
// their own threads; otherwise the frame's thread codes them in turn.
static void emit_vp8(zw_pipe* p, std::vector<uint8_t>& out, const uint8_t* rec, size_t hf, int na)
{
    const uint8_t(*upd)[8][3][11] = (const uint8_t(*)[8][3][11])(p->h_upd.data() + hf * 4 * 8 * 3 * 11);
    const ZwFrameParams& P = p->h_params[hf];
    if (p->nparts == 1) {
        zwh::emit_frame(out, P, rec, p->w, p->h, p->h_have_upd[hf] != 0, upd);
    } else if (na == 1) {
        zwh::emit_frame_parts(out, P, rec, p->w, p->h, p->h_have_upd[hf] != 0, upd, p->nparts,
                              [](int n, auto fn) { parallel_for(n, fn); });
    } else {
        zwh::emit_frame_parts(out, P, rec, p->w, p->h, p->h_have_upd[hf] != 0, upd, p->nparts, [](int n, auto fn) {
            for (int i = 0; i < n; i++) fn(i);
        });
    }
}

// ZW_DUMP_EMIT=<path>: the emission input of the pipe's frame 0 (its
// parameters, probability updates and packed records) for tools/emit_bench.cpp.
static void dump_emit_input(zw_pipe* p, const uint8_t* rec, size_t bytes, size_t hf)
{
    static const char* path = getenv("ZW_DUMP_EMIT");
    static std::atomic<int> done{0};
    if (!path || done.exchange(1)) return;
    FILE* fp = fopen(path, "wb");
    if (!fp) return;
    const uint32_t hdr[4] = {0x4d45575au, (uint32_t)sizeof(ZwFrameParams), (uint32_t)p->w, (uint32_t)p->h};
    const uint8_t have = p->h_have_upd[hf];
    const unsigned long long n = bytes;
    bool ok = fwrite(hdr, sizeof hdr, 1, fp) == 1 && fwrite(&p->h_params[hf], sizeof(ZwFrameParams), 1, fp) == 1 &&
              fwrite(&have, 1, 1, fp) == 1 && fwrite(p->h_upd.data() + hf * 4 * 8 * 3 * 11, 4 * 8 * 3 * 11, 1, fp) == 1 &&
              fwrite(&n, sizeof n, 1, fp) == 1 && fwrite(rec, 1, bytes, fp) == bytes;
    (void)ok;
    fclose(fp);
}

// cpu_ns: the workers' thread CPU time is added to it (the host budget per frame)
static int chunk_emit(zw_pipe* p, const FetchBuf& B, int fa, int na, int par, std::atomic<long long>& cpu_ns)
{
    const size_t F = (size_t)fa;
    const bool has_alpha = p->color == ZW_COLOR_LA8 || p->color == ZW_COLOR_RGBA8;
    if (fa == 0) dump_emit_input(p, B.pack + B.finfo[0], (size_t)B.finfo[1], hidx(p, par, 0));
    std::atomic<int> err{ZW_OK};
    // One token partition (the default): the frames go out in groups of up to
    // ZW_EMIT_GROUP (16 on a host with AVX-512: their boolean coders run as the
    // lanes of one vector coder, zwh::raw_code16; else 4, interleaved), in one
    // thread each (zwh::emit_frames); with token partitions, one frame per task.
    static const int group = [] {
        const char* e = getenv("ZW_EMIT_GROUP");
        const int g = e && *e ? atoi(e) : (zwh::have_code16() ? 16 : 4);
        return g < 1 ? 1 : (g > zwh::EmitWs::kMax ? zwh::EmitWs::kMax : g);
    }();
    // (small chunks -- the seam's batches -- in smaller groups, so that every worker has one)
    // (and very large frames in groups whose decision arenas stay within 1 GiB of
    // address space a worker)
    const int gmem = (int)std::max<size_t>(1, ((size_t)1 << 30) / zwh::emit_arena_bytes(p->mbw, p->mbh));
    const int G = p->nparts != 1
                      ? 1
                      : std::max(1, std::min({group, gmem, std::max(4, na / std::max(1, host_threads()))}));
    // workers per lane (ZW_EMIT_THREADS; default every host thread: with 8 a lane, the
    // two lanes' emissions used 2 % less CPU but the step was 2 % slower)
    static const int per_lane_env = [] { const char* e = getenv("ZW_EMIT_THREADS"); return e ? atoi(e) : 0; }();
    const int nt = per_lane_env > 0 ? per_lane_env : host_threads();
    parallel_for((na + G - 1) / G, [&](int g) {
        const long long c0 = thread_cpu_ns();
        // a workspace from the pipe's pool (its buffers stay allocated and faulted
        // in across chunks and batches; the workers are new threads per chunk)
        std::unique_ptr<zwh::EmitWs> ws;
        {
            std::lock_guard<std::mutex> lk(p->ews_mu);
            if (!p->ews.empty()) {
                ws = std::move(p->ews.back());
                p->ews.pop_back();
            }
        }
        if (!ws) ws.reset(new (std::nothrow) zwh::EmitWs);
        if (!ws) {
            int ok = ZW_OK;
            err.compare_exchange_strong(ok, ZW_ENOMEM);
            return;
        }
        struct Done {
            zw_pipe* p;
            std::unique_ptr<zwh::EmitWs>& ws;
            std::atomic<long long>& to;
            long long c0;
            ~Done()
            {
                {
                    std::lock_guard<std::mutex> lk(p->ews_mu);
                    p->ews.push_back(std::move(ws));
                }
                to.fetch_add(thread_cpu_ns() - c0, std::memory_order_relaxed);
            }
        } done{p, ws, cpu_ns, c0};
        const int i0 = g * G, K = std::min(G, na - i0);
        std::vector<uint8_t>* vp8 = ws->out;
        std::vector<uint8_t>& alph = ws->alph;
        std::vector<uint8_t>* outs[zwh::EmitWs::kMax];
        for (int k = 0; k < K; k++) {
            const size_t f = F + i0 + k;
            // WebPEncoder::encode with EncoderParams::lossy (api.rs:1291-1398) wraps
            // the VP8 frame (and for alpha inputs the ALPH chunk) in a container
            outs[k] = p->container ? &vp8[k] : &p->bitstreams[f];
            outs[k]->clear();
        }
        if (p->nparts == 1) {
            const ZwFrameParams* Pk[zwh::EmitWs::kMax];
            const uint8_t* rk[zwh::EmitWs::kMax];
            bool hk[zwh::EmitWs::kMax];
            const uint8_t(*uk[zwh::EmitWs::kMax])[8][3][11];
            for (int k = 0; k < K; k++) {
                const size_t hf = hidx(p, par, F + i0 + k);
                Pk[k] = &p->h_params[hf];
                rk[k] = B.pack + B.finfo[2 * (i0 + k)];
                hk[k] = p->h_have_upd[hf] != 0;
                uk[k] = (const uint8_t(*)[8][3][11])(p->h_upd.data() + hf * 4 * 8 * 3 * 11);
            }
            try {
                zwh::emit_frames(outs, Pk, rk, K, p->w, p->h, hk, uk, ws.get());
            } catch (const std::bad_alloc&) {  // (the worst-case decision arenas)
                int ok = ZW_OK;
                err.compare_exchange_strong(ok, ZW_ENOMEM);
                return;
            }
        } else {
            emit_vp8(p, *outs[0], B.pack + B.finfo[2 * i0], hidx(p, par, F + i0), na);
        }
        if (!p->container) return;
        for (int k = 0; k < K; k++) {
            const size_t f = F + i0 + k;
            std::vector<uint8_t>& out = p->bitstreams[f];
            alph.clear();
            out.clear();
            if (has_alpha) {
                if (const int r = zw_alph_encode(p->host_frames[f], p->img_stride, p->w, p->h, p->color, alph)) {
                    int ok = ZW_OK;
                    err.compare_exchange_strong(ok, r);
                    return;
                }
            }
            const zw_metadata md = {nullptr, 0, nullptr, 0, nullptr, 0};
            zw_webp_wrap(out, outs[k]->data(), outs[k]->size(), "VP8 ", has_alpha ? &alph : nullptr, has_alpha, p->w,
                         p->h, md);
        }
    }, nt);
    return err.load();
}

static void lane_times(PipeLane& L)
{
    for (int i = 0; i < 4; i++) L.kms[i] = 0.f;
    (void)hipEventElapsedTime(&L.kms[0], L.ev[0], L.ev[1]);  // rgb2yuv
    (void)hipEventElapsedTime(&L.kms[1], L.ev[1], L.ev[2]);  // analysis + segments
    (void)hipEventElapsedTime(&L.kms[2], L.ev[2], L.ev[3]);  // pass 1 (per chunk of frames)
    if (L.p1_frames > 0 && L.p1_frames != L.chunk) L.kms[2] *= (float)L.chunk / (float)L.p1_frames;
    (void)hipEventElapsedTime(&L.kms[3], L.ev[4], L.ev[5]);  // pass 2 (per chunk of frames)
    if (L.p2_frames > 0 && L.p2_frames != L.chunk) L.kms[3] *= (float)L.chunk / (float)L.p2_frames;
}

// Software-pipelined encode of one lane.  Per batch: pass 1 of every chunk is
// queued up front; then per chunk the lane thread fetches the pass-1
// statistics, builds the probabilities / level costs and queues pass 2.  The
// pass-2 records of the batch are fetched and emitted by an emission thread
// while the lane thread already works on the next batch (nb > 1):
//   GPU (stream):  P1(b,0) P1(b,1) P2(b,0) P2(b,1) P1(b+1,0) P1(b+1,1) P2(b+1,0) ..
//   lane thread:           S(b,0)  S(b,1)                   S(b+1,0)  S(b+1,1) ..
//   emitter:                               E(b,0)  E(b,1) ......
// so pass 2 of batch b+1 waits only for its own statistics, not for the
// emission of batch b.  The per-frame header state has one copy per batch
// parity, and pass 2 of (b+1, c) is queued only once the emitter has copied
// out the records of (b, c), whose device buffers it reuses.
static double g_trace_t0 = 0;
static bool g_trace = false;
static int lane_encode(zw_pipe* p, PipeLane& L, bool emit, int nb = 1)
{
    const int nch = (L.n + L.chunk - 1) / L.chunk;
    auto ca = [&](int c) { return L.f0 + c * L.chunk; };
    auto cn = [&](int c) { return std::min(L.chunk, L.n - c * L.chunk); };
    const bool host = p->host_src != nullptr;
    const long long FAILED = std::numeric_limits<long long>::max();
    int qb = 0;  // batch whose pass 1 queue_pass1 queues next
    // cross-lane order of the pass-1 launches (zw_pipe::p1_stats)
    static const bool p1_order_env = [] { const char* e = getenv("ZW_P1_ORDER"); return !e || atoi(e) != 0; }();
    const int G = (int)p->lanes.size();
    const int lane_id = (int)(&L - p->lanes.data());
    const bool p1_order = p1_order_env && G > 1 && emit;
    struct OrderGuard {  // a lane that stops releases the lanes waiting on it
        zw_pipe* p;
        int g;
        bool on;
        ~OrderGuard()
        {
            if (!on) return;
            {
                std::lock_guard<std::mutex> lk(p->p1_mu);
                p->p1_stats[g] = std::numeric_limits<long long>::max();
            }
            p->p1_cv.notify_all();
        }
    } order_guard{p, lane_id, p1_order};
    auto p1_order_wait = [&](int b) -> int {
        if (!p1_order) return ZW_OK;
        const int prev = (lane_id + G - 1) % G;
        const long long need = lane_id == 0 ? b : b + 1;
        if (need <= 0) return ZW_OK;
        {
            std::unique_lock<std::mutex> lk(p->p1_mu);
            p->p1_cv.wait(lk, [&] { return p->p1_stats[prev] >= need; });
            if (p->p1_stats[prev] == std::numeric_limits<long long>::max()) return ZW_OK;  // (it stopped)
        }
        HIPOK(hipStreamWaitEvent(L.stream, p->lanes[prev].ev[6], 0));
        return ZW_OK;
    };
    auto queue_pass1 = [&]() -> int {
        const int b = qb++;
        for (int c = 0; c < nch; c++) {
            // pass 1 of chunk c alone, or of chunks c and c + 1 in one launch (pair1)
            const int c1 = (L.pair1 && (c & 1) == 0 && c + 1 < nch) ? c + 1 : c;
            int r = ZW_OK;
            for (int k = c; k <= c1 && !r; k++) {
                hipEvent_t ue = nullptr, re = nullptr;
                if (host) {  // wait until every uploader has issued its copies of this chunk
                    std::unique_lock<std::mutex> lk(L.sync->mu);
                    const long long need = (long long)b * nch + k + 1;
                    L.sync->cv.wait(lk, [&] {
                        for (long long u : L.uploaded)
                            if (u < need) return false;
                        return true;
                    });
                    for (long long u : L.uploaded)
                        if (u == FAILED) return ZW_EDEVICE;
                    lk.unlock();
                    for (size_t u = 1; u < L.ustreams.size(); u++)
                        HIPOK(hipStreamWaitEvent(L.stream, L.uev[b & 1][u * nch + k], 0));
                    ue = L.uev[b & 1][k];
                    re = L.rev[b & 1][k];
                }
                // (the pre-pass kernels; an unpaired chunk also its pass 1, after the
                // cross-lane wait below for chunk 0)
                const bool enc = c1 == c && !(k == 0 && p1_order);
                r = chunk_pass1(p, L, ca(k), cn(k), k == 0, false, host ? (b & 1) : 0, ue, re, enc);
                if (!r && c1 == c && !enc) {
                    r = p1_order_wait(b);
                    if (!r) r = chunk_pass1_encode(p, L, ca(k), cn(k), k == 0);
                }
                if (host) {
                    {
                        std::lock_guard<std::mutex> lk(L.sync->mu);
                        L.p1_queued = r ? FAILED : L.p1_queued + 1;
                    }
                    L.sync->cv.notify_all();
                }
            }
            if (!r && c == 0 && c1 != c) r = p1_order_wait(b);
            if (!r && c1 != c) r = chunk_pass1_encode(p, L, ca(c), ca(c1) + cn(c1) - ca(c), c == 0);
            for (int k = c; k <= c1 && !r; k++) {
                if (p->host_stats) {
                    r = chunk_pack(p, L, ca(k), cn(k), p->d_out1, 2 * k);
                } else {
                    const size_t F = (size_t)ca(k);
                    HIPOK(zwk_stats(L.stream, p->d_out1 + F * p->nmb, p->mbw, p->mbh,
                                    (uint8_t*)p->d_stats_tmp + zw_stats_scratch_bytes(p->nmb, (int)F),
                                    p->d_stats + F, cn(k)));
                }
                if (!r) HIPOK(hipEventRecord(L.cev[2 * k], L.stream));
            }
            if (r) return r;
            c = c1;
        }
        if (p1_order) {  // this batch's statistics are queued: the next lane's pass 1 may follow
            HIPOK(hipEventRecord(L.ev[6], L.stream));
            {
                std::lock_guard<std::mutex> lk(p->p1_mu);
                p->p1_stats[lane_id] = b + 1;
            }
            p->p1_cv.notify_all();
        }
        return ZW_OK;
    };
    double fetch = 0, stats = 0, fetch2 = 0, tok = 0;
    std::atomic<long long> emit_cpu{0};
    int emit_rc = ZW_OK;
    {
        std::lock_guard<std::mutex> lk(L.sync->mu);
        L.sync->fetched = 0;
        L.uploaded.assign(host ? L.ustreams.size() : 0, 0);
        L.p1_queued = 0;
    }
    // host-source uploads: batch b's chunks into input buffer b & 1, each once
    // rgb2yuv of batch b - 2 has read that buffer's chunk (the copies of batch
    // b + 1 run while batch b's passes hold the GPU)
    std::atomic<int> up_rc{ZW_OK};
    std::vector<std::thread> up;
    if (host) {
        const int U = (int)L.ustreams.size();
        for (int u = 0; u < U; u++)
            up.emplace_back([&, u, U]() {  // (U by value: it goes out of scope before the threads end)
                (void)hipSetDevice(p->ctx->device);
                hipStream_t us = L.ustreams[u];
                for (int b = 0; b < nb && !up_rc; b++)
                    for (int c = 0; c < nch && !up_rc; c++) {
                        if (b >= 2) {
                            std::unique_lock<std::mutex> lk(L.sync->mu);
                            const long long need = (long long)(b - 2) * nch + c + 1;
                            L.sync->cv.wait(lk, [&] { return L.p1_queued >= need; });
                            if (L.p1_queued == FAILED) {
                                up_rc = ZW_EDEVICE;
                                L.uploaded[u] = FAILED;
                                lk.unlock();
                                L.sync->cv.notify_all();
                                return;
                            }
                        }
                        int r = ZW_OK;
                        uint8_t* dst = p->img_buf(b & 1) + (size_t)ca(c) * p->img_stride;
                        if (!L.ustage.empty()) {
                            // staged through the uploader's two pinned slots onto a DMA
                            // engine; the chunk is complete in HBM before it is published
                            if (b >= 2 && hipEventSynchronize(L.rev[b & 1][c]) != hipSuccess) r = ZW_EDEVICE;
                            bool busy[2] = {false, false};
                            int k = 0;
                            for (int i = u; i < cn(c) && !r; i += U, k++) {
                                const int sl = k & 1;
                                if (busy[sl] && (r = sdma_wait(p->ctx, L.usig[2 * u + sl]))) break;
                                const uint8_t* src = p->host_src[(size_t)b * p->n + ca(c) + i];
                                size_t bytes = p->img_stride;
                                if (p->up_pack) {  // RGBA -> RGB through the slot, pinned source or not
                                    pack_rgb(L.ustage[2 * u + sl], src, (size_t)p->w * p->h);
                                    src = L.ustage[2 * u + sl];
                                    bytes = (size_t)p->w * p->h * 3;
                                } else if (const void* dp = host_pinned(src, p->img_stride)) {
                                    src = (const uint8_t*)dp;
                                } else {  // pageable: through the slot
                                    memcpy(L.ustage[2 * u + sl], src, p->img_stride);
                                    src = L.ustage[2 * u + sl];
                                }
                                r = sdma_h2d_start(p->ctx, dst + (size_t)i * p->img_stride, src, bytes,
                                                   L.usig[2 * u + sl]);
                                busy[sl] = r == ZW_OK;
                            }
                            for (int sl = 0; sl < 2; sl++)
                                if (busy[sl]) {
                                    const int w = sdma_wait(p->ctx, L.usig[2 * u + sl]);
                                    if (!r) r = w;
                                }
                        } else {
                            if (b >= 2 && hipStreamWaitEvent(us, L.rev[b & 1][c], 0) != hipSuccess) r = ZW_EDEVICE;
                            for (int i = u; i < cn(c) && !r; i += U)
                                if (hipMemcpyAsync(dst + (size_t)i * p->img_stride,
                                                   p->host_src[(size_t)b * p->n + ca(c) + i], p->img_stride,
                                                   hipMemcpyHostToDevice, us) != hipSuccess)
                                    r = ZW_EDEVICE;
                        }
                        if (!r && hipEventRecord(L.uev[b & 1][u * nch + c], us) != hipSuccess) r = ZW_EDEVICE;
                        {
                            std::lock_guard<std::mutex> lk(L.sync->mu);
                            L.uploaded[u] = r ? FAILED : L.uploaded[u] + 1;
                        }
                        L.sync->cv.notify_all();
                        if (r) up_rc = r;
                    }
            });
    }
    auto join_up = [&]() {
        if (up.empty()) return;
        {  // a lane that stops early releases the uploaders' waits
            std::lock_guard<std::mutex> lk(L.sync->mu);
            if (L.p1_queued != FAILED && L.p1_queued < (long long)nb * nch) L.p1_queued = FAILED;
        }
        L.sync->cv.notify_all();
        for (auto& t : up) t.join();
        up.clear();
    };
    struct UpGuard {  // every return path joins the uploader
        decltype(join_up)& f;
        ~UpGuard() { f(); }
    } up_guard{join_up};
    // emission of batch b (runs on `em`)
    auto emitter = [&](int b) {
        for (int c = 0; c < nch; c++) {
            // the chunks of one pass-2 launch: copied out first (pass 2 of the
            // next batch may then reuse their device buffers), then emitted
            const int c1 = (L.pair2 && (c & 1) == 0 && c + 1 < nch) ? c + 1 : c;
            const double t0 = now_ms();
            for (int k = c; k <= c1; k++) {
                const int r = chunk_fetch(p, L, L.fb[1 + (k & 1)], ca(k), cn(k), 2 * k + 1, L.cev[2 * k + 1]);
                {
                    std::lock_guard<std::mutex> lk(L.sync->mu);
                    L.sync->fetched = r ? FAILED : L.sync->fetched + 1;
                }
                L.sync->cv.notify_all();
                if (r) {
                    emit_rc = r;
                    return;
                }
            }
            const double t1 = now_ms();
            for (int k = c; k <= c1; k++)
                if (const int re = chunk_emit(p, L.fb[1 + (k & 1)], ca(k), cn(k), b & 1, emit_cpu)) {
                    {  // the lane thread may wait for later chunks: release it
                        std::lock_guard<std::mutex> lk(L.sync->mu);
                        L.sync->fetched = FAILED;
                    }
                    L.sync->cv.notify_all();
                    emit_rc = re;
                    return;
                }
            tok += now_ms() - t1;
            fetch2 += t1 - t0;
            if (g_trace)
                fprintf(stderr, "  lane %d batch %d chunks %d-%d: p2 fetched %.1f emit done %.1f\n", L.f0, b, c, c1,
                        t1 - g_trace_t0, now_ms() - g_trace_t0);
            c = c1;
        }
    };
    std::thread em;
    auto join_emitter = [&]() {
        if (em.joinable()) em.join();
        return emit_rc;
    };
    auto fail = [&](int r) {
        join_emitter();
        return r;
    };
    int r = queue_pass1();
    if (r) return fail(r);
    for (int b = 0; b < nb; b++) {
        for (int c = 0; c < nch; c++) {
            // pass 2 of chunk c alone, or of chunks c and c + 1 in one launch (pair2)
            const int c1 = (L.pair2 && (c & 1) == 0 && c + 1 < nch) ? c + 1 : c;
            for (int k = c; k <= c1; k++) {
                const double t0 = now_ms();
                r = p->host_stats ? chunk_fetch(p, L, L.fb[0], ca(k), cn(k), 2 * k, L.cev[2 * k])
                                  : chunk_fetch_stats(p, L, ca(k), cn(k), L.cev[2 * k]);
                if (r) return fail(r);
                const double t1 = now_ms();
                if ((r = chunk_stats(p, L, ca(k), cn(k), b & 1))) return fail(r);
                stats += now_ms() - t1;
                fetch += t1 - t0;
                if (g_trace)
                    fprintf(stderr, "  lane %d batch %d chunk %d: p1 fetched %.1f stats done %.1f\n", L.f0, b, k,
                            t1 - g_trace_t0, now_ms() - g_trace_t0);
                if (emit && b > 0) {  // the emitter has copied out chunk k of batch b-1
                    std::unique_lock<std::mutex> lk(L.sync->mu);
                    const long long need = (long long)(b - 1) * nch + k + 1;
                    L.sync->cv.wait(lk, [&] { return L.sync->fetched >= need; });
                    if (L.sync->fetched == FAILED) {
                        lk.unlock();
                        const int re = join_emitter();
                        return re ? re : ZW_EDEVICE;
                    }
                }
            }
            r = chunk_pass2(p, L, ca(c), ca(c1) + cn(c1) - ca(c), c == 0);
            for (int k = c; k <= c1 && !r; k++) {
                if (emit) r = chunk_pack(p, L, ca(k), cn(k), p->d_out2, 2 * k + 1);
                if (!r && hipEventRecord(L.cev[2 * k + 1], L.stream) != hipSuccess) r = ZW_EDEVICE;
            }
            if (r) return fail(r);
            c = c1;
        }
        if (b + 1 < nb && (r = queue_pass1())) return fail(r);
        if (emit) {
            if ((r = join_emitter())) return r;
            em = std::thread([&, b]() {
                (void)hipSetDevice(p->ctx->device);
                // Emission is throughput work beside the lanes' latency-critical
                // steps (the statistics that release pass 2, the queueing): its
                // thread and the workers it spawns (they inherit the nice value)
                // yield the CPU to them.  Measured: the statistics of a chunk took
                // up to 45 ms instead of ~2 behind two lanes' emission workers,
                // with the GPU idle meanwhile.
                static const int nice_em = [] { const char* e = getenv("ZW_EMIT_NICE"); return e ? atoi(e) : 5; }();
                if (nice_em > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice_em);
                emitter(b);
            });
        }
    }
    if ((r = join_emitter())) return r;
    join_up();
    if (up_rc.load()) return up_rc.load();
    p->out_par = (nb - 1) & 1;
    HIPOK(hipStreamSynchronize(L.stream));
    if ((r = rows_check(p, L))) return r;
    L.hms[0] = fetch / nb;
    L.hms[1] = stats / nb;
    L.hms[2] = fetch2 / nb;
    L.hms[3] = tok / nb;
    L.emit_cpu_ms = 1e-6 * (double)emit_cpu.load() / nb;
    lane_times(L);
    return ZW_OK;
}

// Run fn(lane) for every lane concurrently; returns the first error.
template <class F>
static int run_lanes(zw_pipe* p, F fn)
{
    const int G = (int)p->lanes.size();
    if (G == 1) return fn(p->lanes[0]);
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++)
        th.emplace_back([&, g]() {
            (void)hipSetDevice(p->ctx->device);
            p->lanes[g].rc = fn(p->lanes[g]);
        });
    for (auto& t : th) t.join();
    for (PipeLane& L : p->lanes)
        if (L.rc) return L.rc;
    return ZW_OK;
}

static void pipe_collect_times(zw_pipe* p)
{
    // per-kernel: mean over lanes of each lane's launch duration; host: max over lanes
    // ms[8]: the emission workers' CPU ms per batch, summed over lanes
    for (int i = 0; i < 9; i++) p->kms[i] = 0.f;
    for (PipeLane& L : p->lanes) {
        for (int i = 0; i < 4; i++) {
            p->kms[i] += L.kms[i] / (float)p->lanes.size();
            p->kms[4 + i] = std::max(p->kms[4 + i], (float)L.hms[i]);
        }
        p->kms[8] += (float)L.emit_cpu_ms;
    }
}

extern "C" int zw_pipe_run_pass1(zw_pipe* p, int write_recon)
{
    if (!p) return ZW_EINVAL;
    if (p->broken) return ZW_EDEVICE;
    HIPOK(hipSetDevice(p->ctx->device));
    const int r = run_lanes(p, [&](PipeLane& L) -> int {
        for (int fa = L.f0; fa < L.f0 + L.n; fa += L.chunk) {
            int r = chunk_pass1(p, L, fa, std::min(L.chunk, L.f0 + L.n - fa), false, write_recon != 0);
            if (r) return r;
        }
        HIPOK(hipStreamSynchronize(L.stream));
        return rows_check(p, L);
    });
    if (r) p->broken = true;
    return r;
}

extern "C" int zw_pipe_run_device(zw_pipe* p)
{
    if (!p) return ZW_EINVAL;
    if (p->broken) return ZW_EDEVICE;
    HIPOK(hipSetDevice(p->ctx->device));
    int r = run_lanes(p, [&](PipeLane& L) -> int { return lane_encode(p, L, false); });
    pipe_collect_times(p);
    if (r) p->broken = true;
    return r;
}

static int pipe_encode(zw_pipe* p, int nb)
{
    if (!p || nb < 1) return ZW_EINVAL;
    if (p->broken) return ZW_EDEVICE;
    HIPOK(hipSetDevice(p->ctx->device));
    static const bool trace = getenv("ZW_PIPE_TRACE") != nullptr;
    const double T0 = now_ms();
    g_trace = trace;
    g_trace_t0 = T0;
    p->p1_stats.assign(p->lanes.size(), 0);
    int r = run_lanes(p, [&](PipeLane& L) -> int {
        const int q = lane_encode(p, L, true, nb);
        if (trace)
            fprintf(stderr, "lane f0=%d n=%d chunk=%d x%d: done %.1f ms (per batch: fetch %.1f stats %.1f fetch2 %.1f "
                            "emit %.1f) k: %.1f %.1f %.1f %.1f\n",
                    L.f0, L.n, L.chunk, nb, now_ms() - T0, L.hms[0], L.hms[1], L.hms[2], L.hms[3], L.kms[0], L.kms[1],
                    L.kms[2], L.kms[3]);
        return q;
    });
    pipe_collect_times(p);
    if (r) p->broken = true;
    return r;
}

extern "C" int zw_pipe_encode(zw_pipe* p) { return pipe_encode(p, 1); }

// nb batches whose frames are in host memory (frames[b * n + i], img_stride
// bytes each, any host memory): each lane's uploader thread copies batch b + 1
// into the second input buffer while batch b's passes run (the PCIe-inclusive
// form of zw_pipe_encode_repeat).  Outputs are those of the last batch.
extern "C" int zw_pipe_encode_host(zw_pipe* p, int nb, const uint8_t* const* frames)
{
    if (!p || nb < 1 || !frames) return ZW_EINVAL;
    if (p->broken) return ZW_EDEVICE;
    if (p->container) return ZW_EINVAL;  // (the ALPH coder reads the frames set by zw_pipe_set_container)
    for (size_t i = 0; i < (size_t)nb * p->n; i++)
        if (!frames[i]) return ZW_EINVAL;
    HIPOK(hipSetDevice(p->ctx->device));
    // uploaders per lane: ZW_UPLOAD_THREADS, else a quarter of the host threads
    // over the lanes (the rest code the bitstreams), at least one
    const char* ue = getenv("ZW_UPLOAD_THREADS");
    int U = ue ? atoi(ue) : host_threads() / (4 * (int)p->lanes.size());
    U = std::max(1, std::min(U, 16));
    for (PipeLane& L : p->lanes)
        if (!L.ustreams.empty() && (int)L.ustreams.size() != U) {  // a different count: rebuild the uev table
            for (int k = 0; k < 2; k++) {
                for (hipEvent_t e : L.uev[k]) (void)hipEventDestroy(e);
                L.uev[k].clear();
            }
            while ((int)L.ustreams.size() > U) {
                (void)hipStreamDestroy(L.ustreams.back());
                L.ustreams.pop_back();
            }
        }
    if (nb > 1 && !p->d_img2 && hipMalloc(&p->d_img2, (size_t)p->n * p->img_stride + 64) != hipSuccess)
        return ZW_ENOMEM;
    for (PipeLane& L : p->lanes) {
        const int nch = (L.n + L.chunk - 1) / L.chunk;
        while ((int)L.ustreams.size() < U) {
            hipStream_t st;
            HIPOK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            L.ustreams.push_back(st);
        }
        // DMA staging (ZW_UPLOAD_SDMA=0: HIP copies instead)
        const char* se = getenv("ZW_UPLOAD_SDMA");
        const bool want = !(se && atoi(se) == 0) && sdma_probe(p->ctx);
        if (!want || (int)L.ustage.size() != 2 * U) {
            for (uint8_t* b : L.ustage) pinned_free(b);
            for (hsa_signal_t sg : L.usig) (void)hsa_signal_destroy(sg);
            L.ustage.clear();
            L.usig.clear();
        }
        if (want && L.ustage.empty()) {
            for (int k = 0; k < 2 * U; k++) {
                void* b = nullptr;
                hsa_signal_t sg;
                if (hipHostMalloc(&b, p->img_stride, hipHostMallocDefault) != hipSuccess) return ZW_ENOMEM;
                if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) {
                    pinned_free(b);
                    return ZW_EDEVICE;
                }
                L.ustage.push_back((uint8_t*)b);
                L.usig.push_back(sg);
            }
        }
        for (int k = 0; k < 2; k++) {
            while ((int)L.uev[k].size() < U * nch) {
                hipEvent_t a = nullptr;
                HIPOK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
                L.uev[k].push_back(a);
            }
            while ((int)L.rev[k].size() < nch) {
                hipEvent_t a = nullptr;
                HIPOK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
                L.rev[k].push_back(a);
            }
        }
    }
    {
        const char* pe = getenv("ZW_UPLOAD_PACK");
        p->up_pack = p->bpp == 4 && !p->lanes.empty() && !p->lanes[0].ustage.empty() && !(pe && atoi(pe) == 0);
    }
    p->host_src = frames;
    const int r = pipe_encode(p, nb);
    p->host_src = nullptr;
    p->up_pack = false;
    return r;
}

extern "C" int zw_pipe_encode_repeat(zw_pipe* p, int n) { return pipe_encode(p, n); }

extern "C" int zw_host_threads(void) { return host_threads(); }

extern "C" int zw_pipe_launch_frames(zw_pipe* p) { return p && !p->lanes.empty() ? p->lanes[0].chunk : 0; }

extern "C" int zw_pipe_lanes(zw_pipe* p) { return p ? (int)p->lanes.size() : 0; }

extern "C" int zw_pipe_kernel_times(zw_pipe* p, float* ms, int n)
{
    if (!p || !ms) return ZW_EINVAL;
    for (int i = 0; i < n && i < 9; i++) ms[i] = p->kms[i];
    return ZW_OK;
}

extern "C" int zw_pipe_output(zw_pipe* p, int frame, zw_bytes* out)
{
    if (!p || !out || frame < 0 || frame >= p->n) return ZW_EINVAL;
    const std::vector<uint8_t>& b = p->bitstreams[frame];
    out->data = (uint8_t*)malloc(b.size() ? b.size() : 1);
    if (!out->data) return ZW_ENOMEM;
    memcpy(out->data, b.data(), b.size());
    out->len = b.size();
    return ZW_OK;
}

extern "C" int zw_pipe_read_planes(zw_pipe* p, int frame, int which, uint8_t* y, uint8_t* u, uint8_t* v)
{
    if (!p || frame < 0 || frame >= p->n) return ZW_EINVAL;
    HIPOK(hipSetDevice(p->ctx->device));
    uint8_t* Y = which ? p->d_ry : p->d_Y;
    uint8_t* U = which ? p->d_ru : p->d_U;
    uint8_t* V = which ? p->d_rv : p->d_V;
    if (y) HIPOK(hipMemcpy(y, Y + (size_t)frame * p->ysz, p->ysz, hipMemcpyDeviceToHost));
    if (u) HIPOK(hipMemcpy(u, U + (size_t)frame * p->csz, p->csz, hipMemcpyDeviceToHost));
    if (v) HIPOK(hipMemcpy(v, V + (size_t)frame * p->csz, p->csz, hipMemcpyDeviceToHost));
    return ZW_OK;
}

extern "C" int zw_pipe_read_mbinfo(zw_pipe* p, int frame, int pass, uint8_t* modes, int16_t* levels)
{
    if (!p || frame < 0 || frame >= p->n) return ZW_EINVAL;
    HIPOK(hipSetDevice(p->ctx->device));
    std::vector<ZwMbOut> tmp(p->nmb);
    HIPOK(hipMemcpy(tmp.data(), (pass == 1 ? p->d_out1 : p->d_out2) + (size_t)frame * p->nmb,
                    p->nmb * sizeof(ZwMbOut), hipMemcpyDeviceToHost));
    for (int i = 0; i < p->nmb; i++) {
        if (modes) {
            uint8_t* m = modes + (size_t)i * 20;
            m[0] = tmp[i].luma_mode;
            m[1] = tmp[i].chroma_mode;
            m[2] = tmp[i].skip;
            m[3] = tmp[i].segment;
            memcpy(m + 4, tmp[i].bpred, 16);
        }
        if (levels) memcpy(levels + (size_t)i * 400, tmp[i].levels, 800);
    }
    return ZW_OK;
}

extern "C" int zw_pipe_read_probs(zw_pipe* p, int frame, uint8_t* probs, int* skip_prob)
{
    if (!p || frame < 0 || frame >= p->n) return ZW_EINVAL;
    const ZwFrameParams& P = p->h_params[hidx(p, p->out_par, (size_t)frame)];
    if (probs) memcpy(probs, P.probs, sizeof P.probs);
    if (skip_prob) *skip_prob = P.skip_prob;
    return ZW_OK;
}

extern "C" int zw_pipe_read_segments(zw_pipe* p, int frame, int32_t* seg_qi)
{
    if (!p || frame < 0 || frame >= p->n || !seg_qi) return ZW_EINVAL;
    const ZwFrameParams& P = p->h_params[hidx(p, p->out_par, (size_t)frame)];
    for (int i = 0; i < 4; i++) seg_qi[i] = P.seg[i].quant_index;
    return ZW_OK;
}

extern "C" int zw_pipe_enable_debug(zw_pipe* p)
{
    if (!p) return ZW_EINVAL;
    if (p->d_dbg) return ZW_OK;
    HIPOK(hipSetDevice(p->ctx->device));
    const size_t b = (size_t)p->n * p->nmb * 16 * 34 * sizeof(int);
    if (hipMalloc(&p->d_dbg, b) != hipSuccess) return ZW_ENOMEM;
    HIPOK(hipMemset(p->d_dbg, 0, b));
    return ZW_OK;
}

extern "C" int zw_pipe_read_debug(zw_pipe* p, int frame, int32_t* out)
{
    if (!p || !p->d_dbg || frame < 0 || frame >= p->n || !out) return ZW_EINVAL;
    HIPOK(hipSetDevice(p->ctx->device));
    const size_t b = (size_t)p->nmb * 16 * 34 * sizeof(int);
    HIPOK(hipMemcpy(out, (uint8_t*)p->d_dbg + (size_t)frame * b, b, hipMemcpyDeviceToHost));
    return ZW_OK;
}

extern "C" int zw_pipe_read_alpha(zw_pipe* p, int frame, uint8_t* alpha)
{
    if (!p || frame < 0 || frame >= p->n || !alpha) return ZW_EINVAL;
    HIPOK(hipSetDevice(p->ctx->device));
    HIPOK(hipMemcpy(alpha, p->d_alpha + (size_t)frame * p->nmb, p->nmb, hipMemcpyDeviceToHost));
    return ZW_OK;
}

// --------------------------------------------------------------------------
// Single-image entry points
// --------------------------------------------------------------------------
static int check_encode_args(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                             uint8_t quality)
{
    if (!encode_dims_ok(width, height)) return ZW_EINVALID_DIMENSIONS;
    if (color < 0 || color > 3) return ZW_EINVAL;
    static const int bpp_of[4] = {1, 2, 3, 4};
    if ((uint64_t)width * height * bpp_of[color] != len || !data) return ZW_EINVALID_BUFFER_SIZE;
    if (quality > 100) return ZW_EINVAL;
    return ZW_OK;
}

extern "C" int zw_encode_batch(zw_ctx* ctx, int n, const zw_image* imgs, uint8_t quality, uint8_t method,
                               zw_bytes* outs)
{
    return zw_encode_batch_ex(ctx, n, imgs, quality, method, 1, outs);
}

extern "C" int zw_encode_batch_ex(zw_ctx* ctx, int n, const zw_image* imgs, uint8_t quality, uint8_t method,
                                  int token_partitions, zw_bytes* outs)
{
    if (!ctx || n <= 0 || !imgs || !outs) return ZW_EINVAL;
    if (token_partitions != 1 && token_partitions != 2 && token_partitions != 4 && token_partitions != 8)
        return ZW_EINVAL;
    for (int i = 0; i < n; i++) {
        outs[i].data = nullptr;
        outs[i].len = 0;
        int r = check_encode_args(imgs[i].data, imgs[i].len, imgs[i].width, imgs[i].height, imgs[i].color, quality);
        if (r) return r;
        if (imgs[i].width != imgs[0].width || imgs[i].height != imgs[0].height || imgs[i].color != imgs[0].color)
            return ZW_EINVAL;
    }
    zw_pipe* p = nullptr;
    int r;
    const int key[5] = {(int)imgs[0].width, (int)imgs[0].height, imgs[0].color, quality, method};
    const bool one = n == 1;
    if (one) {  // a one-frame pipeline of this shape from an earlier call, taken out for this call
        std::lock_guard<std::mutex> lk(ctx->pipe1_mu);
        if (ctx->pipe1 && !memcmp(key, ctx->pipe1_key, sizeof key)) {
            p = ctx->pipe1;
            ctx->pipe1 = nullptr;
        }
    }
    if (!p) {
        r = zw_pipe_create(ctx, n, imgs[0].width, imgs[0].height, imgs[0].color, quality, method, &p);
        if (r) return r;
    }
    r = zw_pipe_set_token_partitions(p, token_partitions);
    for (int i = 0; i < n && !r; i++) r = zw_pipe_upload(p, i, imgs[i].data, imgs[i].len);
    if (!r) r = zw_pipe_encode(p);
    for (int i = 0; i < n && !r; i++) r = zw_pipe_output(p, i, &outs[i]);
    if (one && !r) {  // kept for the next call of this shape (not after a failure)
        zw_pipe* old;
        {
            std::lock_guard<std::mutex> lk(ctx->pipe1_mu);
            old = ctx->pipe1;
            ctx->pipe1 = p;
            memcpy(ctx->pipe1_key, key, sizeof key);
        }
        zw_pipe_destroy(old);
    } else {
        zw_pipe_destroy(p);
    }
    return r;
}

extern "C" int zw_encode_webp_batch(zw_ctx* ctx, int n, const zw_image* imgs, uint8_t quality, uint8_t method,
                                    zw_bytes* outs)
{
    if (!ctx || n <= 0 || !imgs || !outs) return ZW_EINVAL;
    for (int i = 0; i < n; i++) {
        outs[i].data = nullptr;
        outs[i].len = 0;
        int r = check_encode_args(imgs[i].data, imgs[i].len, imgs[i].width, imgs[i].height, imgs[i].color, quality);
        if (r) return r;
        if (imgs[i].width != imgs[0].width || imgs[i].height != imgs[0].height || imgs[i].color != imgs[0].color)
            return ZW_EINVAL;
    }
    zw_pipe* p = nullptr;
    int r = zw_pipe_create(ctx, n, imgs[0].width, imgs[0].height, imgs[0].color, quality, method, &p);
    if (r) return r;
    std::vector<const uint8_t*> host(n);
    for (int i = 0; i < n; i++) host[i] = imgs[i].data;
    r = zw_pipe_set_container(p, 1, host.data());
    for (int i = 0; i < n && !r; i++) r = zw_pipe_upload(p, i, imgs[i].data, imgs[i].len);
    if (!r) r = zw_pipe_encode(p);
    for (int i = 0; i < n && !r; i++) r = zw_pipe_output(p, i, &outs[i]);
    zw_pipe_destroy(p);
    return r;
}

// --------------------------------------------------------------------------
// Seam batching of concurrent single-frame calls.  Callers of
// zw_encode_frame_lossy(_ex) on one device -- any contexts, any threads --
// queue their frame; up to SEAM_LEADERS of them at a time take the queue's
// front shape (size, colour, quality, method, partitions) and encode up to
// SEAM_MAX_BATCH queued frames of it as one pipeline batch (a power of two of
// them, so a few cached pipelines serve every load), then wake the callers whose
// frames they carried.  A frame's bitstream does not depend on the other
// frames of its batch, so every caller gets exactly what a call of its own
// returns, while concurrent callers share launches (one CU per frame) instead
// of each allocating a pipeline and queueing its own kernels.  Each leader slot
// has an internal context of its own (streams, scratch, cached pipelines); the
// last zw_ctx_destroy frees them.  ZW_SEAM=0: every call encodes on its own.
// --------------------------------------------------------------------------
namespace {
constexpr int SEAM_LEADERS = 8, SEAM_MAX_BATCH = 64, SEAM_PIPES = 6;
int seam_knob(const char* name, int def)
{
    const char* e = getenv(name);
    return e && *e ? atoi(e) : def;
}
struct SeamReq {
    const uint8_t* data;
    size_t len;
    int key[6];
    zw_bytes* out;
    int rc = ZW_OK;
    bool done = false;
};
struct SeamPipe {
    int key[6];
    int n;
    zw_pipe* p;
    uint64_t used;
};
struct SeamSlot {
    bool busy = false;
    zw_ctx* ctx = nullptr;
    std::vector<SeamPipe> pipes;  // idle pipelines by (shape, frames), LRU beyond SEAM_PIPES
};
struct Seam {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<SeamReq*> q;
    SeamSlot slot[SEAM_LEADERS];
    uint64_t clock = 0;
};
std::mutex g_seam_mu;
std::vector<std::pair<int, Seam*>> g_seams;  // by device; never freed (pointers stay valid)
// process-wide seam counters (zw_dbg_seam_stats): batches led, frames they held, the largest
std::atomic<uint64_t> g_seam_batches{0}, g_seam_frames{0}, g_seam_max{0};
Seam& seam_of(int device)
{
    std::lock_guard<std::mutex> g(g_seam_mu);
    for (auto& d : g_seams)
        if (d.first == device) return *d.second;
    g_seams.push_back({device, new Seam()});
    return *g_seams.back().second;
}
bool seam_enabled()
{
    static const bool on = [] {
        const char* e = getenv("ZW_SEAM");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
}  // namespace

// Frees the idle cached pipelines (all=true: and the internal contexts) of
// every device's seam; slots a leader holds are left alone.
static void seam_trim(bool all)
{
    std::vector<zw_pipe*> drop;
    std::vector<zw_ctx*> ctxs;
    {
        std::lock_guard<std::mutex> g(g_seam_mu);
        for (auto& d : g_seams) {
            Seam& S = *d.second;
            std::lock_guard<std::mutex> lk(S.mu);
            for (SeamSlot& sl : S.slot) {
                if (sl.busy) continue;
                for (SeamPipe& sp : sl.pipes) drop.push_back(sp.p);
                sl.pipes.clear();
                if (all && sl.ctx) {
                    ctxs.push_back(sl.ctx);
                    sl.ctx = nullptr;
                }
            }
        }
    }
    for (zw_pipe* p : drop) zw_pipe_destroy(p);
    for (zw_ctx* c : ctxs) zw_ctx_free_internal(c);
}

static int seam_encode(zw_ctx* ctx, const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                       uint8_t quality, uint8_t method, int nparts, zw_bytes* out)
{
    Seam& S = seam_of(ctx->device);
    SeamReq r{data, len, {(int)width, (int)height, color, quality, method, nparts}, out};
    std::unique_lock<std::mutex> lk(S.mu);
    S.q.push_back(&r);
    while (!r.done) {
        static const int leaders = std::max(1, std::min(SEAM_LEADERS, seam_knob("ZW_SEAM_LEADERS", 2)));
        static const bool pow2 = seam_knob("ZW_SEAM_POW2", 1) != 0;
        int k = 0;
        while (k < leaders && S.slot[k].busy) k++;
        if (k == leaders || S.q.empty()) {
            S.cv.wait(lk);
            continue;
        }
        // lead: the front shape's queued frames, a power of two of them
        SeamSlot& sl = S.slot[k];
        sl.busy = true;
        const int* key = S.q.front()->key;
        int avail = 0;
        for (SeamReq* x : S.q)
            if (!memcmp(x->key, key, sizeof x->key) && ++avail == SEAM_MAX_BATCH) break;
        int n = 1;
        while (2 * n <= avail) n *= 2;
        if (!pow2) n = avail;
        std::vector<SeamReq*> b;
        b.reserve(n);
        int kk[6];
        memcpy(kk, key, sizeof kk);
        for (auto it = S.q.begin(); it != S.q.end() && (int)b.size() < n;) {
            if (!memcmp((*it)->key, kk, sizeof kk)) {
                b.push_back(*it);
                it = S.q.erase(it);
            } else {
                ++it;
            }
        }
        zw_pipe* p = nullptr;
        for (size_t i = 0; i < sl.pipes.size(); i++)
            if (sl.pipes[i].n == n && !memcmp(sl.pipes[i].key, kk, sizeof kk)) {
                p = sl.pipes[i].p;
                sl.pipes.erase(sl.pipes.begin() + (long)i);
                break;
            }
        lk.unlock();
        int rc = ZW_OK;
        if (!sl.ctx) {
            sl.ctx = new zw_ctx();
            sl.ctx->device = ctx->device;
        }
        if (!p) rc = zw_pipe_create(sl.ctx, n, (uint32_t)kk[0], (uint32_t)kk[1], kk[2], (uint8_t)kk[3], (uint8_t)kk[4], &p);
        if (!rc) rc = zw_pipe_set_token_partitions(p, kk[5]);
        for (int i = 0; i < n && !rc; i++) rc = zw_pipe_upload(p, i, b[i]->data, b[i]->len);
        if (!rc) rc = zw_pipe_encode(p);
        std::vector<int> frc(n, rc);
        for (int i = 0; i < n && !rc; i++) frc[i] = zw_pipe_output(p, i, b[i]->out);
        zw_pipe* drop = nullptr;
        if (rc) {  // a pipeline that failed is not kept
            drop = p;
            p = nullptr;
        }
        g_seam_batches.fetch_add(1, std::memory_order_relaxed);
        g_seam_frames.fetch_add((uint64_t)n, std::memory_order_relaxed);
        for (uint64_t m = g_seam_max.load(); (uint64_t)n > m && !g_seam_max.compare_exchange_weak(m, (uint64_t)n);) {
        }
        lk.lock();
        if (sl.ctx && sl.ctx->poisoned.load()) {
            // an SDMA copy of this slot's context timed out: its pinned buffers may
            // still be written, so the context and its pipelines are leaked (the
            // poisoning policy) and the slot's next batch gets a fresh context
            // instead of failing every caller in it with ZW_EDEVICE
            sl.ctx = nullptr;
            sl.pipes.clear();
            p = nullptr;
            drop = nullptr;
        }
        if (p) {
            sl.pipes.push_back({{kk[0], kk[1], kk[2], kk[3], kk[4], kk[5]}, n, p, ++S.clock});
            if ((int)sl.pipes.size() > SEAM_PIPES) {
                size_t lru = 0;
                for (size_t i = 1; i < sl.pipes.size(); i++)
                    if (sl.pipes[i].used < sl.pipes[lru].used) lru = i;
                drop = sl.pipes[lru].p;
                sl.pipes.erase(sl.pipes.begin() + (long)lru);
            }
        }
        for (int i = 0; i < n; i++) {
            b[i]->rc = frc[i];
            b[i]->done = true;
        }
        sl.busy = false;
        S.cv.notify_all();
        if (drop) {
            lk.unlock();
            zw_pipe_destroy(drop);
            lk.lock();
        }
    }
    return r.rc;
}

// Test hook: the seam's process-wide counters (batches led, frames in them,
// the largest batch); reset = 1 clears them.
extern "C" int zw_dbg_seam_stats(uint64_t* out, int reset)
{
    if (!out) return ZW_EINVAL;
    out[0] = g_seam_batches.load();
    out[1] = g_seam_frames.load();
    out[2] = g_seam_max.load();
    if (reset) {
        g_seam_batches = 0;
        g_seam_frames = 0;
        g_seam_max = 0;
    }
    return ZW_OK;
}

extern "C" int zw_encode_frame_lossy(zw_ctx* ctx, const uint8_t* data, size_t len, uint32_t width, uint32_t height,
                                     int color, uint8_t quality, uint8_t method, zw_bytes* out)
{
    return zw_encode_frame_lossy_ex(ctx, data, len, width, height, color, quality, method, 1, out);
}

extern "C" int zw_encode_frame_lossy_ex(zw_ctx* ctx, const uint8_t* data, size_t len, uint32_t width,
                                        uint32_t height, int color, uint8_t quality, uint8_t method,
                                        int token_partitions, zw_bytes* out)
{
    if (!ctx || !out) return ZW_EINVAL;
    out->data = nullptr;
    out->len = 0;
    int r = check_encode_args(data, len, width, height, color, quality);
    if (r) return r;
    if (token_partitions != 1 && token_partitions != 2 && token_partitions != 4 && token_partitions != 8)
        return ZW_EINVAL;
    // Up to ZW_SEAM_SOLO calls in flight encode on their own (each context's
    // cached one-frame pipeline); calls beyond that join the seam.
    static std::atomic<int> inflight{0};
    static const int solo = seam_knob("ZW_SEAM_SOLO", 16);
    struct Count {
        Count() { inflight.fetch_add(1, std::memory_order_acq_rel); }
        ~Count() { inflight.fetch_sub(1, std::memory_order_acq_rel); }
    } count;
    if (seam_enabled() && inflight.load(std::memory_order_acquire) > solo)
        return seam_encode(ctx, data, len, width, height, color, quality, method, token_partitions, out);
    zw_image im = {data, len, width, height, color};
    return zw_encode_batch_ex(ctx, 1, &im, quality, method, token_partitions, out);
}

extern "C" int zw_encode_webp(zw_ctx* ctx, const uint8_t* data, size_t len, uint32_t width, uint32_t height,
                              int color, uint8_t quality, uint8_t method, zw_bytes* out)
{
    if (!ctx || !out) return ZW_EINVAL;
    // EncoderParams::lossy(quality) with the method set (api.rs:451-458)
    const zw_encoder_params p = {1, quality, method, 1};
    return zw_encode_webp_ex(ctx, data, len, width, height, color, &p, nullptr, out);
}

extern "C" int zw_rgb_to_yuv420(zw_ctx* ctx, const uint8_t* img, uint32_t width, uint32_t height, int bpp, uint8_t* y,
                                uint8_t* u, uint8_t* v)
{
    if (!ctx || !img || !y || !u || !v || width == 0 || height == 0 || width > 16383 || height > 16383) return ZW_EINVAL;
    if (bpp < 1 || bpp > 4) return ZW_EINVAL;
    HIPOK(hipSetDevice(ctx->device));
    const int mbw = ((int)width + 15) / 16, mbh = ((int)height + 15) / 16;
    const size_t isz = (size_t)width * height * bpp, ysz = (size_t)mbw * 16 * mbh * 16, csz = (size_t)mbw * 8 * mbh * 8;
    uint8_t *d_img = nullptr, *d_y = nullptr, *d_u = nullptr, *d_v = nullptr;
    hipStream_t s = ctx_stream(ctx);
    int rc = ZW_OK;
    if (hipMalloc(&d_img, isz) != hipSuccess || hipMalloc(&d_y, ysz) != hipSuccess || hipMalloc(&d_u, csz) != hipSuccess ||
        hipMalloc(&d_v, csz) != hipSuccess)
        rc = ZW_ENOMEM;
    if (!rc && hipMemcpyAsync(d_img, img, isz, hipMemcpyHostToDevice, s) != hipSuccess) rc = ZW_EDEVICE;
    if (!rc && zwk_rgb2yuv(s, d_img, (int)width, (int)height, bpp, mbw, mbh, d_y, d_u, d_v, isz, ysz, csz, 1) != hipSuccess)
        rc = ZW_EDEVICE;
    if (!rc && (hipMemcpyAsync(y, d_y, ysz, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(u, d_u, csz, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(v, d_v, csz, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess))
        rc = ZW_EDEVICE;
    (void)hipFree(d_img);
    (void)hipFree(d_y);
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    return rc;
}

// Kernel-level quantisation of n coefficient blocks (see zwebp.h).
extern "C" int zw_quant_blocks(zw_ctx* ctx, int n, const int32_t* coeffs, const uint8_t* ctx0, int ctype, int first,
                               int use_trellis, uint32_t lambda, int q_dc, int q_ac, int matrix_type,
                               const uint8_t* probs, int32_t* levels, int32_t* dequant)
{
    if (!ctx || n <= 0 || !coeffs || !ctx0 || !levels || !dequant) return ZW_EINVAL;
    if (ctype < 0 || ctype > 3 || (first != 0 && first != 1) || q_dc <= 0 || q_ac <= 0 || matrix_type < 0 ||
        matrix_type > 2)
        return ZW_EINVAL;
    for (int i = 0; i < n; i++)
        if (ctx0[i] > 2) return ZW_EINVAL;
    struct {
        ZwMatrix m;
        uint16_t sharpen[16];
        uint32_t lambda;
        int32_t ctype, first, trel, n;
    } a;
    memset(&a, 0, sizeof a);
    static const uint32_t bdc[3] = {96, 96, 110}, bac[3] = {110, 108, 115};
    a.m.q[0] = (uint32_t)q_dc;
    a.m.q[1] = (uint32_t)q_ac;
    for (int i = 0; i < 2; i++) {
        const uint32_t b = i ? bac[matrix_type] : bdc[matrix_type];
        a.m.iq[i] = (1u << 17) / a.m.q[i];
        a.m.bias[i] = ((b << 17) + 128) >> 8;
        a.m.zthresh[i] = ((1u << 17) - 1 - a.m.bias[i]) / a.m.iq[i];
    }
    if (matrix_type == 0)
        for (int i = 0; i < 16; i++)
            a.sharpen[i] = (uint16_t)(((uint32_t)zwh::VP8_FREQ_SHARPENING[i] * (i ? a.m.q[1] : a.m.q[0])) >> 11);
    a.lambda = lambda;
    a.ctype = ctype;
    a.first = first;
    a.trel = use_trellis == 2 ? 2 : use_trellis != 0;  // 2: the lane-parallel trellis
    a.n = n;
    uint8_t P[4][8][3][11];
    memcpy(P, probs ? probs : &zwh::COEFF_PROBS[0][0][0][0], sizeof P);
    ZwLevelCosts L;
    zwh::level_costs(L, P);
    HIPOK(hipSetDevice(ctx->device));
    const size_t cb = (size_t)n * 16 * sizeof(int32_t);
    const size_t o_c = 0, o_x = cb, o_l = (o_x + n + 255) & ~(size_t)255, o_p = o_l + sizeof(ZwLevelCosts);
    const size_t o_lv = (o_p + sizeof P + 255) & ~(size_t)255, o_dq = o_lv + cb, total = o_dq + cb;
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_c, coeffs, cb, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_x, ctx0, (size_t)n, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_l, &L, sizeof L, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_p, P, sizeof P, hipMemcpyHostToDevice, s));
    HIPOK(zwk_quant_blocks(s, (const int*)(d + o_c), d + o_x, (const ZwLevelCosts*)(d + o_l), d + o_p, &a,
                           (int*)(d + o_lv), (int*)(d + o_dq)));
    HIPOK(hipMemcpyAsync(levels, d + o_lv, cb, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(dequant, d + o_dq, cb, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return ZW_OK;
}

// ---------------------------------------------------------------------------
// Streaming DCT+quant pass (zw_xform_kernels.hip)
// ---------------------------------------------------------------------------
static int make_matrix(ZwMatrix& m, int q_dc, int q_ac, int matrix_type)
{
    if (q_dc <= 0 || q_ac <= 0 || q_dc > 2048 || q_ac > 2048 || matrix_type < 0 || matrix_type > 2) return ZW_EINVAL;
    static const uint32_t bdc[3] = {96, 96, 110}, bac[3] = {110, 108, 115};
    m.q[0] = (uint32_t)q_dc;
    m.q[1] = (uint32_t)q_ac;
    for (int i = 0; i < 2; i++) {
        const uint32_t b = i ? bac[matrix_type] : bdc[matrix_type];
        m.iq[i] = (1u << 17) / m.q[i];
        m.bias[i] = ((b << 17) + 128) >> 8;
        m.zthresh[i] = ((1u << 17) - 1 - m.bias[i]) / m.iq[i];
    }
    return ZW_OK;
}

static int device_cus(int device)
{
    hipDeviceProp_t prop;
    return hipGetDeviceProperties(&prop, device) == hipSuccess ? prop.multiProcessorCount : 256;
}

extern "C" int zw_transform_quant_blocks_device(zw_ctx* ctx, void* stream, size_t n, const void* d_src,
                                                const void* d_pred, int q_dc, int q_ac, int matrix_type, int first,
                                                void* d_levels, void* d_recon)
{
    if (!ctx || !d_src || !d_pred || !d_levels || !d_recon || (first != 0 && first != 1)) return ZW_EINVAL;
    ZwMatrix m;
    int r = make_matrix(m, q_dc, q_ac, matrix_type);
    if (r) return r;
    if (n == 0) return ZW_OK;
    static const int cus = device_cus(ctx->device);
    HIPOK(zwk_fdct_quant(stream ? (hipStream_t)stream : ctx_stream(ctx), d_src, d_pred, n, &m, first, d_levels, d_recon,
                         cus));
    return ZW_OK;
}

extern "C" int zw_transform_quant_blocks(zw_ctx* ctx, size_t n, const uint8_t* src, const uint8_t* pred, int q_dc,
                                         int q_ac, int matrix_type, int first, int16_t* levels, uint8_t* recon)
{
    if (!ctx || (n && (!src || !pred || !levels || !recon))) return ZW_EINVAL;
    if (n == 0) return ZW_OK;
    HIPOK(hipSetDevice(ctx->device));
    const size_t o_s = 0, o_p = n * 16, o_l = n * 32, o_r = n * 64, total = n * 80;
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_s, src, n * 16, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_p, pred, n * 16, hipMemcpyHostToDevice, s));
    int r = zw_transform_quant_blocks_device(ctx, s, n, d + o_s, d + o_p, q_dc, q_ac, matrix_type, first, d + o_l,
                                             d + o_r);
    if (r) return r;
    HIPOK(hipMemcpyAsync(levels, d + o_l, n * 32, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(recon, d + o_r, n * 16, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return ZW_OK;
}

// ---------------------------------------------------------------------------
// Streaming DCT+quant pass over per-MB records (zw_xmb_kernels.hip)
// ---------------------------------------------------------------------------
extern "C" size_t zw_xmb_seg_table_bytes(int nframes) { return nframes > 0 ? (size_t)nframes * zwk_xform_mb_seg_bytes() : 0; }

// Segment::init_matrices (types.rs:806) from each segment's quantizer index,
// as the encoder's seg_from_index: y2dc = 2*dc, y2ac = 155/100*ac (>= 8), uv
// uncapped (quirk A17).
extern "C" int zw_xmb_seg_table(int nframes, const int32_t* seg_qi, void* out)
{
    if (nframes <= 0 || !seg_qi || !out) return ZW_EINVAL;
    std::vector<ZwMatrix> m((size_t)nframes * 12);
    for (int i = 0; i < nframes * 4; i++) {
        const int qi = seg_qi[i];
        if (qi < 0 || qi > 127) return ZW_EINVAL;
        const int dc = zwh::DC_QUANT[qi], ac = zwh::AC_QUANT[qi];
        int y2ac = ac * 155 / 100;
        if (y2ac < 8) y2ac = 8;
        if (make_matrix(m[i * 3 + 0], dc, ac, 0) || make_matrix(m[i * 3 + 1], 2 * dc, y2ac, 1) ||
            make_matrix(m[i * 3 + 2], dc, ac, 2))
            return ZW_EINVAL;
    }
    zwk_xform_mb_pack_segs(m.data(), nframes, out);
    return ZW_OK;
}

static int xmb_variant()
{
    const char* e = getenv("ZW_XMB_VARIANT");  // 99: same loads and stores, no arithmetic (copy ceiling)
    return e ? atoi(e) : 0;
}

// Both source forms: src_bpp 0 = Y/U/V planes (d_y, d_u, d_v), 3 / 4 = RGB / RGBA
// pixels at d_y (frame stride img_stride, image w x h).
static int xmb_launch(zw_ctx* ctx, void* stream, int nframes, uint32_t mbw, uint32_t mbh, int src_bpp, uint32_t w,
                      uint32_t h, size_t img_stride, const void* d_y, const void* d_u, const void* d_v,
                      const void* d_recs, const void* d_segs, void* d_levels, void* d_ry, void* d_ru, void* d_rv)
{
    if (!ctx || nframes < 0 || mbw == 0 || mbh == 0 || mbw > 1024 || mbh > 1024) return ZW_EINVAL;
    if (nframes == 0) return ZW_OK;
    if (!d_y || (src_bpp == 0 && (!d_u || !d_v)) || !d_recs || !d_segs || !d_levels || !d_ry || !d_ru || !d_rv)
        return ZW_EINVAL;
    // 16-byte loads and stores: records, planes and levels must be 16-byte aligned (chroma rows 8)
    const uintptr_t a16 = (uintptr_t)d_recs | (uintptr_t)d_levels | (uintptr_t)d_ry | (src_bpp ? 0 : (uintptr_t)d_y);
    const uintptr_t a8 = (uintptr_t)d_ru | (uintptr_t)d_rv | (src_bpp ? 0 : ((uintptr_t)d_u | (uintptr_t)d_v));
    if ((a16 & 15) || (a8 & 7)) return ZW_EINVAL;
    HIPOK(hipSetDevice(ctx->device));
    // The I4 queue k_xform_mb fills and k_xform_mb_i4 drains: one per launch
    // stream, grow-only (a regrow frees the old buffer, which hipFree orders
    // after queued work).  The queue keeps one count per launch parity: a launch
    // appends to count qp and its drain zeroes count qp ^ 1 (the previous
    // launch's, drained earlier in stream order), so a launch pair leaves its own
    // count nonzero and the next launch, of the other parity, starts from zero.
    // A new buffer, or one whose last launch pair failed to queue, is reset on
    // the launch stream first.  So neither an overlapping launch on another
    // stream nor a launch that stopped partway can leave a stale count.
    // At most XMB_QUEUES streams keep a queue: a new stream takes the least
    // recently used idle one's entry (hipFree of its buffer waits for the
    // device); an entry whose launch another thread is queueing is never taken.
    // An overflow any launch reports through the context's host-visible error
    // word (k_xform_mb, never expected) fails this and every later call.
    const hipStream_t ls = stream ? (hipStream_t)stream : ctx_stream(ctx);
    const size_t qb = zwk_xform_mb_queue_bytes((int)mbw, (int)mbh, nframes);
    void* q = nullptr;
    zw_ctx::XmbQueue* qe = nullptr;
    int qp = 0;
    {
        std::lock_guard<std::mutex> lk(ctx->xmb_mu);
        if (!ctx->xmb_err) {
            void* h = nullptr;
            void* dp = nullptr;
            if (hipHostMalloc(&h, 64, hipHostMallocMapped) != hipSuccess) return ZW_ENOMEM;
            if (hipHostGetDevicePointer(&dp, h, 0) != hipSuccess) {
                (void)hipHostFree(h);
                return ZW_EDEVICE;
            }
            ctx->xmb_err = (volatile uint32_t*)h;
            ctx->xmb_err_dev = (uint32_t*)dp;
            *ctx->xmb_err = 0;
        }
        if (*ctx->xmb_err) return ZW_EDEVICE;
        constexpr size_t XMB_QUEUES = 8;
        zw_ctx::XmbQueue* e = nullptr;
        for (auto& x : ctx->xmb_q)
            if (x.stream == ls) e = &x;
        if (e && e->inflight && e->cap < qb) e = nullptr;  // (another thread queues on it: a new entry to regrow)
        if (!e && ctx->xmb_q.size() >= XMB_QUEUES) {
            for (auto& x : ctx->xmb_q)
                if (x.inflight == 0 && (!e || x.used < e->used)) e = &x;
            if (e) {
                if (e->buf) (void)hipFree(e->buf);
                *e = {ls, nullptr, 0};
            }
        }
        if (!e) {
            ctx->xmb_q.push_back({ls, nullptr, 0});
            e = &ctx->xmb_q.back();
        }
        e->used = ++ctx->xmb_clock;
        if (e->cap < qb) {
            if (e->buf) (void)hipFree(e->buf);
            e->buf = nullptr;
            e->cap = 0;
            if (hipMalloc(&e->buf, qb) != hipSuccess) return ZW_ENOMEM;
            e->cap = qb;
            e->dirty = true;
        }
        q = e->buf;
        qe = e;
        if (qe->dirty) HIPOK(hipMemsetAsync(q, 0, 16, ls));
        qe->dirty = true;
        qp = qe->parity;
        qe->inflight++;
        // test hook: a stale count past this launch's MBs, as a shared queue would leave
        if (getenv("ZW_XMB_FORCE_OVERFLOW")) {
            const uint32_t stale = (uint32_t)((size_t)nframes * mbw * mbh);
            HIPOK(hipMemcpyAsync((uint32_t*)q + qp, &stale, 4, hipMemcpyHostToDevice, ls));
            HIPOK(hipStreamSynchronize(ls));  // (the source is on this stack)
        }
    }
    const hipError_t le = zwk_xform_mb(ls, (const uint8_t*)d_y, (const uint8_t*)d_u, (const uint8_t*)d_v, src_bpp,
                                       (int)w, (int)h, img_stride, (const uint8_t*)d_recs, d_segs, (int)mbw, (int)mbh,
                                       nframes, (int16_t*)d_levels, (uint8_t*)d_ry, (uint8_t*)d_ru, (uint8_t*)d_rv,
                                       (uint32_t*)q, qp, ctx->xmb_err_dev, xmb_variant());
    {
        std::lock_guard<std::mutex> lk(ctx->xmb_mu);
        qe->inflight--;
        // both kernels queued: the pair leaves count qp ^ 1 zero for the next launch
        // (a failed launch leaves the entry dirty: reset before its next use)
        if (le == hipSuccess) {
            qe->dirty = false;
            qe->parity ^= 1;
        }
    }
    HIPOK(le);
    return ZW_OK;
}

extern "C" int zw_transform_quant_mbs_device(zw_ctx* ctx, void* stream, int nframes, uint32_t mbw, uint32_t mbh,
                                             const void* d_y, const void* d_u, const void* d_v, const void* d_recs,
                                             const void* d_segs, void* d_levels, void* d_ry, void* d_ru, void* d_rv)
{
    return xmb_launch(ctx, stream, nframes, mbw, mbh, 0, 0, 0, 0, d_y, d_u, d_v, d_recs, d_segs, d_levels, d_ry, d_ru,
                      d_rv);
}

extern "C" int zw_transform_quant_mbs_rgb_device(zw_ctx* ctx, void* stream, int nframes, uint32_t width,
                                                 uint32_t height, int bpp, const void* d_img, size_t img_stride,
                                                 const void* d_recs, const void* d_segs, void* d_levels, void* d_ry,
                                                 void* d_ru, void* d_rv)
{
    if (bpp != 3 && bpp != 4) return ZW_EINVAL;
    if (width == 0 || height == 0 || img_stride < (size_t)width * height * bpp) return ZW_EINVAL;
    return xmb_launch(ctx, stream, nframes, (width + 15) / 16, (height + 15) / 16, bpp, width, height, img_stride,
                      d_img, nullptr, nullptr, d_recs, d_segs, d_levels, d_ry, d_ru, d_rv);
}

extern "C" int zw_transform_quant_mbs(zw_ctx* ctx, int nframes, uint32_t mbw, uint32_t mbh, const uint8_t* y,
                                      const uint8_t* u, const uint8_t* v, const uint8_t* recs, const int32_t* seg_qi,
                                      int16_t* levels, uint8_t* ry, uint8_t* ru, uint8_t* rv)
{
    if (!ctx || nframes < 0 || mbw == 0 || mbh == 0 || mbw > 1024 || mbh > 1024) return ZW_EINVAL;
    if (nframes == 0) return ZW_OK;
    if (!y || !u || !v || !recs || !seg_qi || !levels || !ry || !ru || !rv) return ZW_EINVAL;
    HIPOK(hipSetDevice(ctx->device));
    const size_t F = (size_t)nframes, nmb = (size_t)mbw * mbh;
    const size_t ysz = nmb * 256 * F, csz = nmb * 64 * F, rb = nmb * ZW_XMB_RECORD_BYTES * F, lb = nmb * 800 * F;
    const size_t sb = zw_xmb_seg_table_bytes(nframes);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_y = 0, o_u = al(ysz), o_v = o_u + al(csz), o_r = o_v + al(csz), o_s = o_r + al(rb),
                 o_l = o_s + al(sb), o_ry = o_l + al(lb), o_ru = o_ry + al(ysz), o_rv = o_ru + al(csz),
                 total = o_rv + al(csz);
    std::vector<uint8_t> segs(sb);
    int r = zw_xmb_seg_table(nframes, seg_qi, segs.data());
    if (r) return r;
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_y, y, ysz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_u, u, csz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_v, v, csz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_r, recs, rb, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_s, segs.data(), sb, hipMemcpyHostToDevice, s));
    r = zw_transform_quant_mbs_device(ctx, s, nframes, mbw, mbh, d + o_y, d + o_u, d + o_v, d + o_r, d + o_s, d + o_l,
                                      d + o_ry, d + o_ru, d + o_rv);
    if (r) return r;
    HIPOK(hipMemcpyAsync(levels, d + o_l, lb, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(ry, d + o_ry, ysz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(ru, d + o_ru, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(rv, d + o_rv, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return *ctx->xmb_err ? ZW_EDEVICE : ZW_OK;
}

extern "C" int zw_transform_quant_mbs_rgb(zw_ctx* ctx, int nframes, uint32_t width, uint32_t height, int bpp,
                                          const uint8_t* img, const uint8_t* recs, const int32_t* seg_qi,
                                          int16_t* levels, uint8_t* ry, uint8_t* ru, uint8_t* rv)
{
    if (!ctx || nframes < 0 || width == 0 || height == 0 || (bpp != 3 && bpp != 4)) return ZW_EINVAL;
    const uint32_t mbw = (width + 15) / 16, mbh = (height + 15) / 16;
    if (mbw > 1024 || mbh > 1024) return ZW_EINVAL;
    if (nframes == 0) return ZW_OK;
    if (!img || !recs || !seg_qi || !levels || !ry || !ru || !rv) return ZW_EINVAL;
    HIPOK(hipSetDevice(ctx->device));
    const size_t F = (size_t)nframes, nmb = (size_t)mbw * mbh, fsz = (size_t)width * height * bpp;
    const size_t isz = fsz * F, ysz = nmb * 256 * F, csz = nmb * 64 * F, rb = nmb * ZW_XMB_RECORD_BYTES * F;
    const size_t lb = nmb * 800 * F, sb = zw_xmb_seg_table_bytes(nframes);
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_i = 0, o_r = al(isz), o_s = o_r + al(rb), o_l = o_s + al(sb), o_ry = o_l + al(lb),
                 o_ru = o_ry + al(ysz), o_rv = o_ru + al(csz), total = o_rv + al(csz);
    std::vector<uint8_t> segs(sb);
    int r = zw_xmb_seg_table(nframes, seg_qi, segs.data());
    if (r) return r;
    uint8_t* d = (uint8_t*)ctx_scratch(ctx, total);
    if (!d) return ZW_ENOMEM;
    hipStream_t s = ctx_stream(ctx);
    HIPOK(hipMemcpyAsync(d + o_i, img, isz, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_r, recs, rb, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d + o_s, segs.data(), sb, hipMemcpyHostToDevice, s));
    r = zw_transform_quant_mbs_rgb_device(ctx, s, nframes, width, height, bpp, d + o_i, fsz, d + o_r, d + o_s,
                                          d + o_l, d + o_ry, d + o_ru, d + o_rv);
    if (r) return r;
    HIPOK(hipMemcpyAsync(levels, d + o_l, lb, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(ry, d + o_ry, ysz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(ru, d + o_ru, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipMemcpyAsync(rv, d + o_rv, csz, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    return *ctx->xmb_err ? ZW_EDEVICE : ZW_OK;
}
