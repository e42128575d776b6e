// The "armed launch" the round-3 verdict proposed for the drop-in tick, measured
// against the plain launch (diagnostic only, never the product):
//
//   plain: the call stages its step block (1 KiB) as a kernel argument and
//          launches a 256-workgroup grid; the host spins on a host-mapped word
//          until workgroup 0 publishes (the tick's pattern; the rollout itself is
//          left out, so the difference is what the critical path would lose);
//   armed: the grid of call n + 1 is launched at the end of call n and waits:
//          workgroup 0 polls a host-mapped "go" word (bounded), copies the step
//          block from pinned host memory into device memory and releases the
//          other workgroups through a device word; the call writes the block,
//          then "go", and spins on the same published word.
//   armed-all: every workgroup polls the host word itself (256 PCIe pollers); a
//          poller waits for go >= its call, since the host may already have
//          moved go on for the next call when a slow poller looks.
//
// Between two calls the host "works" for GAP us (the caller's plant step).
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/armed_launch tools/armed_launch.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }
static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
static double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
}

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e_ = (x);                                              \
        if (e_ != hipSuccess) {                                           \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            return 1;                                                     \
        }                                                                 \
    } while (0)

struct alignas(16) Block { unsigned char b[1024]; };
constexpr unsigned long long kPollTicks = 200000000ull;   // bound on every poll: 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// plain: the block arrives as the kernel argument
__global__ void k_plain(const Block blk, unsigned* out, unsigned seq, unsigned* sink) {
    if (threadIdx.x == 0 && blk.b[5] == 0xA5) sink[blockIdx.x] = 1;   // keep the argument live
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(out, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// armed: workgroup 0 waits for go == seq on the host word, copies the block and releases the others
__global__ void k_armed(const unsigned* go, const Block* hblk, Block* dblk, unsigned* dflag, unsigned* out, unsigned seq,
                        unsigned* sink, int all_poll) {
    __shared__ unsigned ok;
    if (all_poll || blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            const unsigned long long end = __builtin_amdgcn_s_memrealtime() + kPollTicks;
            bool in_time = true;
            while ((int)(ld_sys(go) - seq) < 0 && (in_time = __builtin_amdgcn_s_memrealtime() < end)) __builtin_amdgcn_s_sleep(1);
            ok = in_time;
        }
        __syncthreads();
        if (!all_poll) {
            if (threadIdx.x < 64) reinterpret_cast<uint4*>(dblk)[threadIdx.x] = reinterpret_cast<const uint4*>(hblk)[threadIdx.x];
            __syncthreads();
            if (threadIdx.x == 0) {
                __threadfence();
                __hip_atomic_store(dflag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    } else {
        if (threadIdx.x == 0) {
            const unsigned long long end = __builtin_amdgcn_s_memrealtime() + kPollTicks;
            bool in_time = true;
            while (__hip_atomic_load(dflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != seq &&
                   (in_time = __builtin_amdgcn_s_memrealtime() < end))
                __builtin_amdgcn_s_sleep(1);
            ok = in_time;
        }
        __syncthreads();
        if (threadIdx.x == 0 && ok && dblk->b[5] == 0xA5) sink[blockIdx.x] = 1;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(out, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// bounded host spin on the published word: a grid that never publishes ends the run with a message
static bool wait_pub(const unsigned* out, unsigned seq, const char* phase, int i) {
    const auto t0 = clk::now();
    while (__atomic_load_n(out, __ATOMIC_ACQUIRE) != seq) {
        if (us(t0, clk::now()) > 2e6) {
            std::printf("%s: call %d never published (seq %u, word %u)\n", phase, i, seq, *out);
            return false;
        }
    }
    return true;
}

static void host_work(double gap_us) {
    const auto t0 = clk::now();
    while (us(t0, clk::now()) < gap_us) {
    }
}

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    const double gap = argc > 2 ? atof(argv[2]) : 10.0;
    CHECK(hipSetDevice(0));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned *out, *go, *dflag, *sink;
    Block *hblk, *dblk;
    CHECK(hipHostMalloc(&out, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc(&go, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc(&hblk, sizeof(Block), hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipMalloc(&dblk, sizeof(Block)));
    CHECK(hipMalloc(&dflag, 64));
    CHECK(hipMalloc(&sink, 4096));
    CHECK(hipMemset(dflag, 0, 64));
    *out = 0;
    *go = 0;
    std::memset(hblk, 0, sizeof(Block));
    Block blk{};
    unsigned seq = 0;
    // plain
    std::vector<double> p_call, p_tot;
    for (int i = 0; i < iters + 100; ++i) {
        host_work(gap);
        ++seq;
        const auto t0 = clk::now();
        blk.b[0] = (unsigned char)seq;
        hipLaunchKernelGGL(k_plain, dim3(256), dim3(256), 0, s, blk, out, seq, sink);
        const auto t1 = clk::now();
        if (!wait_pub(out, seq, "plain", i)) {
            (void)hipStreamSynchronize(s);
            return 2;
        }
        const auto t2 = clk::now();
        if (i >= 100) {
            p_call.push_back(us(t0, t1));
            p_tot.push_back(us(t0, t2));
        }
    }
    CHECK(hipStreamSynchronize(s));
    std::printf("plain    : launch call %6.2f us, call -> published %6.2f us (p10 %6.2f p90 %6.2f)\n", med(p_call),
                med(p_tot), pct(p_tot, 0.1), pct(p_tot, 0.9));
    for (int all = 0; all < 2; ++all) {
        std::vector<double> a_tot, a_arm;
        // arm the first one
        ++seq;
        hipLaunchKernelGGL(k_armed, dim3(256), dim3(256), 0, s, go, hblk, dblk, dflag, out, seq, sink, all);
        for (int i = 0; i < iters + 100; ++i) {
            host_work(gap);
            const auto t0 = clk::now();
            hblk->b[0] = (unsigned char)seq;     // the step block, then go
            __atomic_store_n(go, seq, __ATOMIC_RELEASE);
            if (!wait_pub(out, seq, all ? "armed-all" : "armed", i)) {
                (void)hipStreamSynchronize(s);   // the grid's polls are bounded: let it drain before exiting
                return 2;
            }
            const auto t2 = clk::now();
            ++seq;   // arm the next call at the end of this one
            const auto t3 = clk::now();
            hipLaunchKernelGGL(k_armed, dim3(256), dim3(256), 0, s, go, hblk, dblk, dflag, out, seq, sink, all);
            const auto t4 = clk::now();
            if (i >= 100) {
                a_tot.push_back(us(t0, t2));
                a_arm.push_back(us(t3, t4));
            }
        }
        __atomic_store_n(go, seq, __ATOMIC_RELEASE);   // release the last armed grid
        CHECK(hipStreamSynchronize(s));
        std::printf("%s: go -> published %6.2f us (p10 %6.2f p90 %6.2f); arming launch call %6.2f us (off the path)\n",
                    all ? "armed-all" : "armed    ", med(a_tot), pct(a_tot, 0.1), pct(a_tot, 0.9), med(a_arm));
    }
    std::printf("(%d calls each, %.1f us of host work between calls)\n", iters, gap);
    return 0;
}
