// mppi_readback.hip — sampled_traj_list's host read-back (control.py:135-145).
//
// The device re-roll writes fp32 (K, T, dx) states; the reference hands back fp64.  Widening on the device
// doubles what crosses the host link (134 MB instead of 67 MB at K = 65536, T = 64, ~2.5 ms at the link's
// ~54 GB/s).  fp32 -> fp64 is exact, so the widening can happen on either side with the same bits: here the
// fp32 states are DMA'd chunk by chunk into a page-locked ring, and a pool of host threads widens each chunk
// into the caller's fp64 array as soon as its copy has landed, while the next chunks are still in flight.
// The call is bound by the fp32 DMA plus the widening of the last chunk.
//
// Roles in one mppi_readback_run:
//   * the calling thread queues up to R chunk copies, alternating over S copy streams that first wait for the
//     caller's stream (the kernel that wrote the source): a copy's start-up overlaps the one before it instead of
//     leaving the link idle (one stream: ~15 us per copy, +1 ms at 1 MB chunks); it polls their events in order
//     and publishes `ready` = chunks landed;
//   * W workers (persistent, woken per call) widen their fixed slice of every landed chunk, streaming the
//     fp64 stores past the cache, and count themselves done per ring slot;
//   * the calling thread reuses a slot for chunk j + R only after all W workers are done with chunk j.
// The chunks are `chunk` floats, but the last three shrink to a half, a quarter and an eighth of it: the call
// ends with the widening of the last chunk, so the small ones shorten that tail.
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mppi_host.h"
#include "mppi_rocm.h"

namespace {
using mppi_host::fail;

constexpr int kMaxSlots = 16;
constexpr int kMaxWorkers = 64;
constexpr int kMaxStreams = 4;

struct alignas(64) SlotCount {
    std::atomic<int> done{0};
};

// fp32 -> fp64, exact.  AVX2 where the CPU has it: 8 values per iteration, the fp64 stores non-temporal (the
// destination is written once and read later by the caller: no read-for-ownership of 134 MB of lines).
__attribute__((target("avx2"))) void widen_avx2(double* d, const float* s, size_t n) {
    size_t i = 0;
    while (i < n && (reinterpret_cast<uintptr_t>(d + i) & 31)) {
        d[i] = (double)s[i];
        ++i;
    }
    for (; i + 8 <= n; i += 8) {
        const __m256 v = _mm256_loadu_ps(s + i);
        _mm256_stream_pd(d + i, _mm256_cvtps_pd(_mm256_castps256_ps128(v)));
        _mm256_stream_pd(d + i + 4, _mm256_cvtps_pd(_mm256_extractf128_ps(v, 1)));
    }
    for (; i < n; ++i) d[i] = (double)s[i];
    _mm_sfence();
}

void widen_scalar(double* d, const float* s, size_t n) {
    for (size_t i = 0; i < n; ++i) d[i] = (double)s[i];
}

}  // namespace

struct mppi_readback {
    int device = 0;
    int workers = 0;
    int slots = 0;
    int nstreams = 0;               // copy streams (0: the copies go on the caller's stream)
    size_t chunk = 0;               // floats per chunk (a multiple of 128)
    float* ring = nullptr;          // page-locked, slots x chunk floats
    hipEvent_t ev[kMaxSlots] = {};
    hipStream_t cs[kMaxStreams] = {};
    hipEvent_t start = nullptr;     // the caller's stream, before the copies
    bool avx2 = false;
    std::vector<std::thread> pool;

    // the job (written by the caller before the generation bump, read by the workers after it)
    std::mutex m;
    std::condition_variable cv;
    uint64_t gen = 0;
    bool quit = false;
    double* dst = nullptr;
    size_t n = 0;
    long long nchunks = 0;
    std::vector<size_t> off;        // chunk j is [off[j], off[j + 1])
    std::atomic<long long> ready{0};      // chunks landed in the ring (the caller's event polls); -1: abort
    std::atomic<int> finished{0};         // workers done with the whole job
    SlotCount count[kMaxSlots];

    void widen(double* d, const float* s, size_t len) const {
        if (avx2)
            widen_avx2(d, s, len);
        else
            widen_scalar(d, s, len);
    }

    // the chunk boundaries of n floats: `chunk` each, the last three chunk / 2, / 4, / 8 (the first takes the rest)
    void plan(size_t total) {
        off.clear();
        size_t end = total;
        std::vector<size_t> rev{end};
        for (int tail = 8; end > 0; tail = tail > 1 ? tail / 2 : 1) {
            const size_t len = chunk / tail;
            end = end > len ? end - len : 0;
            rev.push_back(end);
        }
        off.assign(rev.rbegin(), rev.rend());
        nchunks = (long long)off.size() - 1;
    }

    // worker w's slice of chunk j: [lo, hi) floats within the chunk, 16-float aligned
    void slice(long long j, int w, size_t* lo, size_t* hi) const {
        const size_t len = off[j + 1] - off[j];
        const size_t per = ((len + workers - 1) / workers + 15) & ~(size_t)15;
        *lo = (size_t)w * per < len ? (size_t)w * per : len;
        *hi = *lo + per < len ? *lo + per : len;
    }

    void worker(int w) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return quit || gen != seen; });
                if (quit) return;
                seen = gen;
            }
            for (long long j = 0; j < nchunks; ++j) {
                long long r;
                while ((r = ready.load(std::memory_order_acquire)) <= j && r >= 0) _mm_pause();
                if (r < 0) break;   // the copies failed: the caller reports it
                size_t lo, hi;
                slice(j, w, &lo, &hi);
                if (hi > lo) widen(dst + off[j] + lo, ring + (size_t)(j % slots) * chunk + lo, hi - lo);
                count[j % slots].done.fetch_add(1, std::memory_order_release);
            }
            finished.fetch_add(1, std::memory_order_release);
        }
    }
};

namespace {

int wait_event(hipEvent_t e) {
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return MPPI_OK;
        if (q != hipErrorNotReady) return fail(MPPI_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(q));
        _mm_pause();
    }
}

}  // namespace

extern "C" {

int mppi_readback_create(int device, int workers, int slots, long long chunk_floats, int copy_streams,
                         mppi_readback** out) {
    if (!out || workers < 1 || workers > kMaxWorkers || slots < 2 || slots > kMaxSlots || chunk_floats < 128 ||
        copy_streams < 0 || copy_streams > kMaxStreams)
        return fail(MPPI_E_ARG, "mppi_readback_create: workers 1..64, slots 2..16, chunk >= 128 floats, "
                                "copy streams 0..4");
    *out = nullptr;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    auto* rb = new mppi_readback();
    rb->device = device;
    rb->workers = workers;
    rb->slots = slots;
    rb->chunk = ((size_t)chunk_floats + 127) & ~(size_t)127;   // its eighth stays 16-float aligned
    rb->nstreams = copy_streams;
    rb->avx2 = __builtin_cpu_supports("avx2");
    e = hipHostMalloc((void**)&rb->ring, rb->chunk * slots * sizeof(float), hipHostMallocDefault);
    if (e != hipSuccess) {
        delete rb;
        return fail(MPPI_E_HIP, std::string("hipHostMalloc (read-back ring): ") + hipGetErrorString(e));
    }
    for (int s = 0; s < slots && e == hipSuccess; ++s) e = hipEventCreateWithFlags(&rb->ev[s], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&rb->start, hipEventDisableTiming);
    for (int s = 0; s < copy_streams && e == hipSuccess; ++s) e = hipStreamCreateWithFlags(&rb->cs[s], hipStreamNonBlocking);
    if (e != hipSuccess) {
        mppi_readback_destroy(rb);
        return fail(MPPI_E_HIP, std::string("mppi_readback_create: ") + hipGetErrorString(e));
    }
    rb->pool.reserve(workers);
    for (int w = 0; w < workers; ++w) rb->pool.emplace_back([rb, w] { rb->worker(w); });
    *out = rb;
    return MPPI_OK;
}

void mppi_readback_destroy(mppi_readback* rb) {
    if (!rb) return;
    {
        std::lock_guard<std::mutex> lk(rb->m);
        rb->quit = true;
    }
    rb->cv.notify_all();
    for (auto& t : rb->pool) t.join();
    for (int s = 0; s < rb->slots; ++s)
        if (rb->ev[s]) (void)hipEventDestroy(rb->ev[s]);
    if (rb->start) (void)hipEventDestroy(rb->start);
    for (int s = 0; s < rb->nstreams; ++s)
        if (rb->cs[s]) (void)hipStreamDestroy(rb->cs[s]);
    if (rb->ring) (void)hipHostFree(rb->ring);
    delete rb;
}

int mppi_readback_run(mppi_readback* rb, void* stream, const float* src_dev, double* dst_host, long long n) {
    if (!rb || n < 0 || (n > 0 && (!src_dev || !dst_host)))
        return fail(MPPI_E_ARG, "mppi_readback_run: null argument or negative length");
    if (n == 0) return MPPI_OK;
    hipError_t e = hipSetDevice(rb->device);
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    auto st = static_cast<hipStream_t>(stream);
    rb->plan((size_t)n);
    const long long nchunks = rb->nchunks;
    const int R = rb->slots;
    rb->dst = dst_host;
    rb->n = (size_t)n;
    if (rb->nstreams > 0) {
        e = hipEventRecord(rb->start, st);
        for (int s = 0; s < rb->nstreams && e == hipSuccess; ++s) e = hipStreamWaitEvent(rb->cs[s], rb->start, 0);
        if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("read-back start: ") + hipGetErrorString(e));
    }
    rb->ready.store(0, std::memory_order_relaxed);
    rb->finished.store(0, std::memory_order_relaxed);
    for (int s = 0; s < R; ++s) rb->count[s].done.store(0, std::memory_order_relaxed);

    auto issue = [&](long long j) -> int {
        const size_t off = rb->off[j], len = rb->off[j + 1] - off;
        float* slot = rb->ring + (size_t)(j % R) * rb->chunk;
        hipStream_t cs = rb->nstreams > 0 ? rb->cs[j % rb->nstreams] : st;
        hipError_t err = hipMemcpyAsync(slot, src_dev + off, len * sizeof(float), hipMemcpyDeviceToHost, cs);
        if (err == hipSuccess) err = hipEventRecord(rb->ev[j % R], cs);
        if (err != hipSuccess) return fail(MPPI_E_HIP, std::string("read-back copy: ") + hipGetErrorString(err));
        return MPPI_OK;
    };
    int rc = MPPI_OK;
    long long issued = 0;
    for (; issued < nchunks && issued < R && rc == MPPI_OK; ++issued) rc = issue(issued);
    {
        std::lock_guard<std::mutex> lk(rb->m);
        ++rb->gen;    // the workers start (they spin on `ready` until the first chunk lands)
    }
    rb->cv.notify_all();
    for (long long j = 0; j < nchunks && rc == MPPI_OK; ++j) {
        rc = wait_event(rb->ev[j % R]);
        if (rc != MPPI_OK) break;
        rb->ready.store(j + 1, std::memory_order_release);
        if (issued < nchunks) {
            // chunk `issued` reuses chunk j's slot (issued == j + R): every worker must be done with chunk j
            SlotCount& c = rb->count[j % R];
            while (c.done.load(std::memory_order_acquire) < rb->workers) _mm_pause();
            c.done.store(0, std::memory_order_relaxed);
            rc = issue(issued++);
        }
    }
    if (rc != MPPI_OK) rb->ready.store(-1, std::memory_order_release);   // the workers stop at their next chunk
    while (rb->finished.load(std::memory_order_acquire) < rb->workers) _mm_pause();
    if (rc != MPPI_OK) {   // no copy may still land in the ring
        for (int s = 0; s < rb->nstreams; ++s) (void)hipStreamSynchronize(rb->cs[s]);
        (void)hipStreamSynchronize(st);
    }
    return rc;
}

}  // extern "C"
