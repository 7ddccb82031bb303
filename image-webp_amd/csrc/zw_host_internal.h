// zw_host_internal.h -- state shared by the host translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <sched.h>
#include <algorithm>
#include <atomic>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

struct zw_ctx {
    int device;
    hipStream_t stream_ = nullptr;  // created on first use (hardware queues are scarce)
    hipStream_t copy_ = nullptr;    // decode downloads (ctx_d2h_stream), created on first use
    hipEvent_t copy_ev = nullptr;   // its completion, waited on without spinning
    // grow-only device scratch for the single-call decode / filter entry points
    void* dscratch = nullptr;
    size_t dscratch_cap = 0;
    void* dscratch1 = nullptr;  // second buffer of the pipelined decode batches
    void* dscratch2 = nullptr;  // decode batches: the device token parse's upload, snapshots and offsets
    size_t dscratch2_cap = 0;
    void* dscratch3 = nullptr;  // decode batches: the device token parse's records (sized by its count pass)
    size_t dscratch3_cap = 0;
    uint64_t* tok_total = nullptr;  // pinned: the count pass's record bytes
    hipStream_t tok_ = nullptr;  // the device token parse (runs beside the chunks' kernels), created on first use
    // [0] before stage 1, [1] the records written, [2] the count pass and scans done, [3] stage 1 done
    hipEvent_t tok_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // zw_transform_quant_mbs*_device: the I4 queue of k_xform_mb / k_xform_mb_i4,
    // one per launch stream (launches on different streams may overlap; launches
    // on one stream are ordered), its counters reset on that stream per launch
    struct XmbQueue {
        hipStream_t stream = nullptr;
        void* buf = nullptr;
        size_t cap = 0;
        bool dirty = true;  // counters not known to be zero: reset on the stream first
        int parity = 0;     // the count the next launch appends to (k_xform_mb's qp)
        uint64_t used = 0;  // xmb_clock at the last launch (LRU eviction past 8 streams)
        int inflight = 0;   // launches being queued on it (between the two locked sections): not evictable
    };
    std::deque<XmbQueue> xmb_q;  // (a deque: entries stay put while others are added)
    uint64_t xmb_clock = 0;
    volatile uint32_t* xmb_err = nullptr;  // host-mapped: k_xform_mb sets it on a queue overflow
    uint32_t* xmb_err_dev = nullptr;       // the same word as the device addresses it
    std::mutex xmb_mu;
    size_t dscratch1_cap = 0;
    // SDMA copy engine path (HSA) for device->host fetches: ROCclr's hipMemcpy
    // D2H runs as a blit kernel, which cannot be dispatched while an encode
    // kernel holds every CU; the DMA engines need no CU.
    // Probed once under sdma_mu (pipe lanes call ctx_d2h from several threads).
    std::atomic<int> sdma{-1};  // -1 unprobed, 0 unavailable, 1 ready
    std::mutex sdma_mu;
    // set when a DMA copy did not complete in time: the engine may still write
    // into its destination, so every later copy of this context fails
    std::atomic<bool> poisoned{false};
    hsa_agent_t gpu_agent{}, cpu_agent{};
    // grow-only pinned host staging (decode batch: MB records up, planes down)
    // [0] / [2]: the two upload buffers of the pipelined decode, [1] downloads,
    // [3] the row-parallel kernels' sync / error words, [4] the device token
    // parse's upload (modes, probabilities, token partitions)
    void* hpin[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t hpin_cap[5] = {0, 0, 0, 0, 0};
    // device time of the last decode batch: [0] k_dec_recon, [1] k_loopfilter,
    // [2] k_yuv2rgb (0 when the batch returned planes) (ms)
    // ([4], [5]: around k_dec_tokl when the device parses the tokens)
    hipEvent_t dev_ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    hipEvent_t dev_ev1[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // second buffer of the pipelined decode
    float dec_ms[3] = {0.f, 0.f, 0.f};
    float dec_tok_ms = 0.f;  // the device token parse of the last batch (0: the host parsed every frame)
    float dec_tok_stage_ms[3] = {0.f, 0.f, 0.f};  // its stage 1, count pass + offsets (+ the host's wait), record pass
    // measured rates for the host / device split of the token parse (dec_tok_split):
    // host chunk parse ms per frame (the whole chunk over all threads), device launch ms
    // per MB of a frame (the launch runs its frames side by side), 0 = not measured yet
    double dec_host_ms_per_frame = 0, dec_tok_ms_per_mb = 0;
    // host stages of the last decode batch, wall ms summed over its chunks:
    // [0] parse (bool decoder + records), [1] download, [2] fan-out / copy-out
    double dec_host_ms[3] = {0, 0, 0};
    // one-frame encode pipeline kept between encode_frame_lossy calls of the
    // same shape (dimensions, colour type, quality, method): its device buffers
    // and streams are reused instead of allocated per call
    // A call takes the cached pipe out under pipe1_mu and puts it back when it
    // succeeds, so two threads sharing a context never run on one pipe.
    struct zw_pipe* pipe1 = nullptr;
    int pipe1_key[5] = {0, 0, 0, 0, 0};
    std::mutex pipe1_mu;
    // decode: per-frame worst-case record buffers of the two pipelined buffer
    // sets, kept between chunks and calls (a parse touches only the pages it
    // writes; reallocating them per chunk cost page faults and unmaps)
    struct RecBuf {
        std::unique_ptr<uint8_t[]> p;  // uninitialised: untouched pages stay unbacked
        size_t cap = 0;
    };
    std::vector<RecBuf> dec_recs[2];
};

#define HIPOK(x)                                  \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) {                   \
            fprintf(stderr, "zwebp: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return ZW_EDEVICE;                    \
        }                                         \
    } while (0)


// Host worker threads per process (entropy coding, stats, decode parsing).
// ZW_HOST_THREADS overrides.  Default: this process's share of the CPUs it may
// run on -- the affinity mask divided by the ranks on this node
// (LOCAL_WORLD_SIZE, set by torch.distributed.run), capped by the job's
// per-process CPU share when one is declared (OMP_NUM_THREADS).
static inline int host_threads_default()
{
    cpu_set_t set;
    int cpus = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : 0;
    if (cpus <= 0) cpus = (int)std::thread::hardware_concurrency();
    const char* lw = getenv("LOCAL_WORLD_SIZE");
    const int ranks = lw && atoi(lw) > 0 ? atoi(lw) : 1;
    int n = cpus / ranks;
    const char* omp = getenv("OMP_NUM_THREADS");
    if (omp && atoi(omp) > 0 && atoi(omp) < n) n = atoi(omp);
    return n < 1 ? 1 : n;
}
static inline int host_threads()
{
    const char* e = getenv("ZW_HOST_THREADS");
    int n = e ? atoi(e) : 0;
    if (n <= 0) {
        static const int dflt = host_threads_default();
        n = dflt;
    }
    return n;
}

template <class F>
static inline void parallel_for(int n, F fn, int max_threads = 0)
{
    int nt = std::min(max_threads > 0 ? std::min(max_threads, host_threads()) : host_threads(), n);
    if (nt <= 1) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    std::atomic<int> next(0);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; t++)
        th.emplace_back([&]() {
            for (;;) {
                int i = next.fetch_add(1);
                if (i >= n) break;
                fn(i);
            }
        });
    for (auto& t : th) t.join();
}


// Device scratch `which` (0 or 1) of at least `bytes` owned by the context.
static inline void* ctx_scratch(zw_ctx* c, size_t bytes, int which = 0)
{
    void*& p = which ? c->dscratch1 : c->dscratch;
    size_t& cap = which ? c->dscratch1_cap : c->dscratch_cap;
    if (cap < bytes) {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        cap = bytes;
    }
    return p;
}

static inline void* ctx_scratch_rec(zw_ctx* c, size_t bytes)
{
    if (c->dscratch3_cap < bytes) {
        if (c->dscratch3) (void)hipFree(c->dscratch3);
        c->dscratch3 = nullptr;
        c->dscratch3_cap = 0;
        if (hipMalloc(&c->dscratch3, bytes) != hipSuccess) return nullptr;
        c->dscratch3_cap = bytes;
    }
    return c->dscratch3;
}

static inline void* ctx_scratch_tok(zw_ctx* c, size_t bytes)
{
    if (c->dscratch2_cap < bytes) {
        if (c->dscratch2) (void)hipFree(c->dscratch2);
        c->dscratch2 = nullptr;
        c->dscratch2_cap = 0;
        if (hipMalloc(&c->dscratch2, bytes) != hipSuccess) return nullptr;
        c->dscratch2_cap = bytes;
    }
    return c->dscratch2;
}

// The context's own stream (single-call entry points); created lazily so a
// context that only drives pipes does not hold a hardware queue.
// Device->host copy on the context's copy stream (HIP chooses the engine: a
// blit kernel for large copies, ≈57 GB/s on this box against ≈25 GB/s for one
// SDMA engine).  For the decode paths, whose kernels leave CUs free; the encode
// pipeline's fetches keep ctx_d2h (its kernels hold every CU).
int ctx_d2h_stream(zw_ctx* c, void* dst, const void* src, size_t bytes);

static inline hipStream_t ctx_stream(zw_ctx* c)
{
    if (!c->stream_) (void)hipStreamCreateWithFlags(&c->stream_, hipStreamNonBlocking);
    return c->stream_;
}

// Blocking device->host copy on a DMA engine (falls back to hipMemcpy when the
// HSA agents cannot be resolved).  `src` must have been released by the
// producing kernel (event-complete) before the call, and `dst` must be pinned
// (hipHostMalloc): the DMA engine cannot reach pageable memory.
int ctx_d2h(zw_ctx* c, void* dst, const void* src, size_t bytes);

// Decoded-frame buffer pool (zw_dec_host.cpp): takes back a buffer it handed
// out (returns false for any other pointer, which the caller frees).
bool zw_dec_pool_put(void* p);
// Frees the buffers the pool holds (zw_ctx_release_buffers).
void zw_dec_pool_trim();
// Is some zw_ctx alive (zw_host.cpp)?  The frame pool keeps buffers only then.
bool zw_ctx_any_alive();
// Frees a context's resources and the context (zw_ctx_destroy minus the count).
void zw_ctx_free_internal(zw_ctx* c);

// Set (process-wide) once an SDMA copy timed out with the engine possibly
// still writing its destination: from then on pinned host buffers, which are
// the destinations of those copies, are leaked instead of freed, so a late
// DMA write cannot land in memory the allocator has handed out again.
extern std::atomic<bool> g_dma_poisoned;
static inline void pinned_free(void* h)
{
    if (h && !g_dma_poisoned.load(std::memory_order_acquire)) (void)hipHostFree(h);
}

// Pinned host staging buffer `which` of at least `bytes` owned by the context.
static inline void* ctx_pinned(zw_ctx* c, int which, size_t bytes)
{
    if (c->hpin_cap[which] < bytes) {
        pinned_free(c->hpin[which]);
        c->hpin[which] = nullptr;
        c->hpin_cap[which] = 0;
        if (hipHostMalloc(&c->hpin[which], bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
        c->hpin_cap[which] = bytes;
    }
    return c->hpin[which];
}

// Host lossless coder and container writer (zw_host_lossless.cpp).
int zw_vp8l_encode(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color, bool predictor,
                   bool implicit_dims, std::vector<uint8_t>& out);
int zw_alph_encode(const uint8_t* data, size_t len, uint32_t width, uint32_t height, int color,
                   std::vector<uint8_t>& out);
void zw_webp_wrap(std::vector<uint8_t>& o, const uint8_t* frame, size_t flen, const char* tag,
                  const std::vector<uint8_t>* alph, bool has_alpha, uint32_t width, uint32_t height,
                  const zw_metadata& md);
