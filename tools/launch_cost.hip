// Host cost of one kernel launch call against the kernel-argument size, and the
// launch-to-start latency seen by a host spin on a host-mapped word (the
// drop-in tick's pattern).  Diagnostic only: tools/gpu_launch_cost.sh.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/launch_cost tools/launch_cost.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

template <int N>
struct Args {
    unsigned char pad[N];
};

// grid of G workgroups; workgroup 0 thread 0 publishes seq to host memory
template <int N>
__global__ void k_args(const Args<N> a, unsigned* host_word, unsigned seq) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned v = seq + (a.pad[N - 1] == 0x5A ? 1u : 0u);
        __hip_atomic_store(host_word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// busy for ~us microseconds (s_memrealtime at 100 MHz), one wave per workgroup
__global__ void k_busy(unsigned ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 1;                                                               \
        }                                                                           \
    } while (0)

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}
static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
static double p90(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() * 9 / 10];
}

// the rollout kernel's argument shape: 18 arguments, two of them structs
struct S120 { unsigned char b[120]; };
struct alignas(16) S1056 { unsigned char b[1056]; };
struct S96 { unsigned char b[96]; };
struct S16 { void* p; unsigned s; };
__global__ void k_many(const S120 c, const S1056 ss, const void* a0, const void* a1, double* a2, double* a3, double* a4,
                       unsigned* a5, double* a6, double* a7, void* a8, unsigned flags, const S96 xd, unsigned* a9,
                       unsigned* a10, float* a11, const S16 ho, unsigned long long* a12) {
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<unsigned*>(ho.p), ho.s + (ss.b[7] == 0x5A ? 1u : 0u), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

int run_many(hipStream_t s, unsigned* hw, int iters) {
    S120 c{};
    S1056 ss{};
    S96 xd{};
    std::vector<double> call, spin;
    unsigned seq = 1;
    for (int i = 0; i < iters + 50; ++i) {
        ++seq;
        const S16 ho{hw, seq};
        const auto t0 = clk::now();
        hipLaunchKernelGGL(k_many, dim3(256), dim3(256), 0, s, c, ss, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr, nullptr, 0u, xd, nullptr, nullptr, nullptr, ho, nullptr);
        const auto t1 = clk::now();
        while (__atomic_load_n(hw, __ATOMIC_ACQUIRE) != seq) {
        }
        const auto t2 = clk::now();
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        if (i >= 50) {
            call.push_back(us(t0, t1));
            spin.push_back(us(t0, t2));
        }
    }
    std::printf("18 arguments (rollout shape)  grid  256: launch call %6.2f us (p90 %6.2f)  call->published %6.2f us (p90 %6.2f)\n",
                med(call), p90(call), med(spin), p90(spin));
    return 0;
}

template <int N>
int run(hipStream_t s, unsigned* hw, int grid, int iters, int busy_us = 0) {
    Args<N> a{};
    std::vector<double> call, spin;
    unsigned seq = 1;
    for (int i = 0; i < iters + 50; ++i) {
        ++seq;
        if (busy_us) hipLaunchKernelGGL(k_busy, dim3(256), dim3(64), 0, s, (unsigned)(busy_us * 100));
        const auto t0 = clk::now();
        hipLaunchKernelGGL((k_args<N>), dim3(grid), dim3(256), 0, s, a, hw, seq);
        const auto t1 = clk::now();
        while (__atomic_load_n(hw, __ATOMIC_ACQUIRE) != seq) {
        }
        const auto t2 = clk::now();
        CHECK(hipStreamSynchronize(s));
        if (i >= 50) {
            call.push_back(us(t0, t1));
            spin.push_back(us(t0, t2));
        }
    }
    std::printf("%s", busy_us ? "behind a running kernel: " : "");
    std::printf("kernarg %5d B  grid %4d: launch call %6.2f us (p90 %6.2f)  call->published %6.2f us (p90 %6.2f)\n",
                (int)sizeof(Args<N>) + 12, grid, med(call), p90(call), med(spin), p90(spin));
    return 0;
}

#ifdef LAUNCH_COST_LIB
extern "C" int launch_cost_main() {
#else
int main() {
#endif
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned* hw = nullptr;
    CHECK(hipHostMalloc((void**)&hw, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *hw = 0;
    const int iters = 2000;
    for (int grid : {1, 256}) {
        if (run<16>(s, hw, grid, iters) || run<256>(s, hw, grid, iters) || run<512>(s, hw, grid, iters) ||
            run<1024>(s, hw, grid, iters) || run<1536>(s, hw, grid, iters) || run<2048>(s, hw, grid, iters) ||
            run<3072>(s, hw, grid, iters))
            return 1;
    }
    if (run_many(s, hw, iters)) return 1;
    std::printf("null stream:\n");
    if (run_many(nullptr, hw, iters) || run<16>(nullptr, hw, 256, iters)) return 1;
    hipStream_t sb;
    CHECK(hipStreamCreate(&sb));   // a blocking stream exists: the null stream must order against it
    std::printf("null stream, one blocking stream alive:\n");
    if (run_many(nullptr, hw, iters)) return 1;
    std::printf("blocking stream:\n");
    if (run_many(sb, hw, iters)) return 1;
    if (run<16>(s, hw, 256, iters, 20) || run<1536>(s, hw, 256, iters, 20)) return 1;
    CHECK(hipHostFree(hw));
    CHECK(hipStreamDestroy(s));
    return 0;
}
