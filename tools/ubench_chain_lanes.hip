// ubench_chain_lanes.hip — config 5's shard (K = 16384, T = 128, n = 7): four lanes per sample (the product's
// chain_horizon_q4) against eight, on the step's serial chain: the bias scans, the D' columns from broadcasts,
// the L D L^T factorization with its forward solve, the back solve, semi-implicit Euler and the new sincos —
// everything of a step but the noise, the window search and the cost (VERDICT r5 "Next round" item 6).
//
//   quad : lane p holds the link pair (2p, 2p+1) as f32x2 (packed math), broadcasts by DPP quad_perm;
//          K = 16384 samples x 4 lanes = 1024 waves: one wave per SIMD.
//   oct  : lane p holds link p (lane 7 a pad), scalar math, broadcasts within 8 lanes by
//          DPP quad_perm + row_half_mirror + a select (OCT_SWIZZLE=0) or one ds_swizzle (OCT_SWIZZLE=1);
//          8 lanes x 16384 = 2048 waves: two waves per SIMD.
// The arithmetic is the same in both (the same matrix, the same operations per element), so the two must agree
// to fp32 rounding; the time per step is what is compared.
//
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/_build/ubench_chain_lanes tools/ubench_chain_lanes.hip
// ./ubench_chain_lanes [K] [T] [reps]  ->  one JSON line
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <utility>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int N = 7;
constexpr int NT = 256;

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int Q>
__device__ __forceinline__ float qbc(float v) { return dpp<Q * 0x55>(v); }
__device__ __forceinline__ f32x2 splat(float x) { return f32x2{x, x}; }
template <int J>
__device__ __forceinline__ float elem(f32x2 v) { return (J & 1) ? v.y : v.x; }

template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// physical constants of a 7-link chain (per link): length, nu (mass moment), damping, diagonal and coupling terms
// (the pad link N: zero length and moment, unit diagonal, as the product's parameter block pads it)
__device__ __forceinline__ float cl(int a) { return a < N ? 0.30f + 0.02f * a : 0.f; }
__device__ __forceinline__ float cnu(int a) { return a < N ? 0.90f - 0.10f * a : 0.f; }
__device__ __forceinline__ float cdd(int a) { return a < N ? 2.0f - 0.15f * a : 1.f; }
__device__ __forceinline__ float cj(int a) { return a < N ? 0.05f + 0.01f * a : 0.f; }

// ------------------------------------------------------------------------------------------------ quad
__device__ __forceinline__ float q_excl_prefix(float x, float m1) {
#pragma clang fp contract(off)
    const float e = dpp<0x90>(x) * m1;
    const float f = e + dpp<0x90>(e);
    return f + dpp<0x40>(f);
}
__device__ __forceinline__ float q_excl_suffix(float x, float u1) {
#pragma clang fp contract(off)
    const float e = dpp<0xF9>(x) * u1;
    const float f = e + dpp<0xF9>(e);
    return f + dpp<0xFE>(f);
}

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) void quad_kernel(int K, int T, float* out) {
    const int tid = blockIdx.x * NT + threadIdx.x, sub = threadIdx.x & 3, k = tid >> 2;
    const int a0 = 2 * sub, a1 = a0 + 1;
    const float m1 = sub >= 1 ? 1.f : 0.f, u1 = sub <= 2 ? 1.f : 0.f;
    const f32x2 pad = {a0 < N ? 1.f : 0.f, a1 < N ? 1.f : 0.f};
    const f32x2 l2 = {cl(a0), cl(a1)}, nu2 = {cnu(a0), cnu(a1)}, damp2 = {0.1f, 0.1f};
    const float dt = 0.006f, g = 9.81f, dtr = dt * 0.15915494309189535f;
    f32x2 corr[N];
#pragma unroll
    for (int a = 0; a < N; ++a)
        corr[a] = f32x2{a0 == a ? cdd(a0) : (a0 == a + 1 ? -cj(a0) : 0.f), a1 == a ? cdd(a1) : (a1 == a + 1 ? -cj(a1) : 0.f)};
    f32x2 TH = f32x2{0.01f * (k & 63) + 0.1f * a0, 0.01f * (k & 63) + 0.1f * a1} * splat(0.15915494309189535f);
    f32x2 THD = {0.f, 0.f}, C, Sn;
    auto angles = [&]() {
        C = f32x2{__builtin_amdgcn_cosf(TH.x), __builtin_amdgcn_cosf(TH.y)};
        Sn = f32x2{__builtin_amdgcn_sinf(TH.x), __builtin_amdgcn_sinf(TH.y)};
    };
    angles();
    const f32x2 vin = f32x2{0.3f, -0.2f} * pad;
    for (int t = 0; t < T; ++t) {
        const f32x2 v = vin * splat(1.f + 1e-3f * (t & 7));
        const f32x2 w = THD * THD;
        const f32x2 lc = l2 * C, ls = l2 * Sn, vc = nu2 * C, vs = nu2 * Sn;
        const f32x2 wvc = w * vc, wvs = w * vs, wlc = w * lc, wls = w * ls;
        const float sC = q_excl_suffix(wvc.x + wvc.y, u1), sS = q_excl_suffix(wvs.x + wvs.y, u1);
        const float pC = q_excl_prefix(wlc.x + wlc.y, m1), pS = q_excl_prefix(wls.x + wls.y, m1);
        const f32x2 Cs = {wvc.y + sC, sC}, Ss = {wvs.y + sS, sS};
        const f32x2 Cp = {pC, wlc.x + pC}, Sp = {pS, wls.x + pS};
        const f32x2 X = __builtin_elementwise_fma(l2, Cs, nu2 * Cp);
        const f32x2 Y = __builtin_elementwise_fma(l2, Ss, nu2 * Sp);
        const float thd_prev = dpp<0x90>(THD.y) * m1;
        const f32x2 qd = THD - f32x2{thd_prev, THD.x};
        const f32x2 ve = __builtin_elementwise_fma(-damp2, qd, v);
        const float ve_next = dpp<0xF9>(ve.x) * u1;
        f32x2 r = {ve.x - ve.y, ve.y - ve_next};
        r = __builtin_elementwise_fma(C, Y, __builtin_elementwise_fma(-Sn, X, __builtin_elementwise_fma(splat(-g), vc, r)));
        f32x2 col[N];
        unroll_seq([&](auto a_c) {
            constexpr int a = decltype(a_c)::value;
            const float la = qbc<a / 2>(elem<a>(lc)), sa = qbc<a / 2>(elem<a>(ls));
            col[a] = __builtin_elementwise_fma(splat(la), vc, __builtin_elementwise_fma(splat(sa), vs, corr[a]));
        }, std::make_integer_sequence<int, N>{});
        float Ln[N][N], yn[N];
        unroll_seq([&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            const float nrd = __builtin_amdgcn_rcpf(-qbc<j / 2>(elem<j>(col[j])));
            yn[j] = qbc<j / 2>(elem<j>(r)) * nrd;
            r = __builtin_elementwise_fma(splat(yn[j]), col[j], r);
            unroll_seq([&](auto k_c) {
                constexpr int kk = decltype(k_c)::value;
                if constexpr (kk > j) {
                    Ln[kk][j] = qbc<kk / 2>(elem<kk>(col[j])) * nrd;
                    if constexpr (kk == N - 1) asm volatile("" : "+v"(Ln[kk][j]));
                    col[kk] = __builtin_elementwise_fma(splat(Ln[kk][j]), col[j], col[kk]);
                }
            }, std::make_integer_sequence<int, N>{});
        }, std::make_integer_sequence<int, N>{});
        float x[N];
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            float e = -yn[i];
#pragma unroll
            for (int kk = N - 1; kk > i; --kk) e = fmaf(Ln[kk][i], x[kk], e);
            x[i] = e;
        }
        auto xs = [&](int i) { return i < N ? x[i] : 0.f; };
        const bool b0 = sub & 1, b1 = sub & 2;
        const float xa = b1 ? (b0 ? xs(6) : xs(4)) : (b0 ? xs(2) : xs(0));
        const float xb = b1 ? (b0 ? xs(7) : xs(5)) : (b0 ? xs(3) : xs(1));
        THD = __builtin_elementwise_fma(f32x2{xa, xb}, splat(dt), THD);
        TH = __builtin_elementwise_fma(THD, splat(dtr), TH);
        angles();
    }
    // link a's angle: (lane a / 2, component a & 1)
    if (k < K) {
        if (a0 < N) out[(size_t)k * 8 + a0] = TH.x;
        if (a1 < N) out[(size_t)k * 8 + a1] = TH.y;
    }
}

// ------------------------------------------------------------------------------------------------ oct
#ifndef OCT_SWIZZLE
#define OCT_SWIZZLE 0
#endif
// lane Q of each group of 8
template <int Q>
__device__ __forceinline__ float obc(float v, bool upper) {
#if OCT_SWIZZLE
    (void)upper;
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x18 | (Q << 5)));   // and 0x18, or Q
#else
    const float a = qbc<Q & 3>(v);   // each quad: its lane Q & 3
    const float b = dpp<0x141>(a);   // row_half_mirror: the other quad's
    return ((Q < 4) != upper) ? a : b;
#endif
}
// exclusive prefix / suffix sums over the 8 lanes of a group: the shift by one, then Hillis-Steele strides 1, 2,
// 4 (row_shr / row_shl within the row of 16), the reads from the neighbouring group masked off
__device__ __forceinline__ float o_excl_prefix(float x, float m1, float m2, float m4) {
#pragma clang fp contract(off)
    float e = dpp<0x111>(x) * m1;          // row_shr:1: x_{p-1}
    e = e + dpp<0x111>(e) * m1;            // + e_{p-1}
    e = e + dpp<0x112>(e) * m2;            // row_shr:2
    return e + dpp<0x114>(e) * m4;         // row_shr:4
}
__device__ __forceinline__ float o_excl_suffix(float x, float u1, float u2, float u4) {
#pragma clang fp contract(off)
    float e = dpp<0x101>(x) * u1;          // row_shl:1: x_{p+1}
    e = e + dpp<0x101>(e) * u1;
    e = e + dpp<0x102>(e) * u2;            // row_shl:2
    return e + dpp<0x104>(e) * u4;         // row_shl:4
}

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void oct_kernel(int K, int T, float* out) {
    const int tid = blockIdx.x * NT + threadIdx.x, p = threadIdx.x & 7, k = tid >> 3;
    const bool upper = p >= 4;
    const float on = p < N ? 1.f : 0.f;
    const float m1 = p >= 1, m2 = p >= 2, m4 = p >= 4, u1 = p <= 6, u2 = p <= 5, u4 = p <= 3;
    const float l = cl(p), nu = cnu(p), damp = 0.1f;
    const float dt = 0.006f, g = 9.81f, dtr = dt * 0.15915494309189535f;
    float corr[N];
#pragma unroll
    for (int a = 0; a < N; ++a) corr[a] = p == a ? cdd(p) : (p == a + 1 ? -cj(p) : 0.f);
    float TH = (0.01f * (k & 63) + 0.1f * p) * 0.15915494309189535f, THD = 0.f, C, Sn;
    auto angles = [&]() {
        C = __builtin_amdgcn_cosf(TH);
        Sn = __builtin_amdgcn_sinf(TH);
    };
    angles();
    const float vin = ((p & 1) ? -0.2f : 0.3f) * on;
    for (int t = 0; t < T; ++t) {
        const float v = vin * (1.f + 1e-3f * (t & 7));
        const float w = THD * THD;
        const float lc = l * C, ls = l * Sn, vc = nu * C, vs = nu * Sn;
        const float sC = o_excl_suffix(w * vc, u1, u2, u4), sS = o_excl_suffix(w * vs, u1, u2, u4);
        const float pC = o_excl_prefix(w * lc, m1, m2, m4), pS = o_excl_prefix(w * ls, m1, m2, m4);
        // the quad's X / Y per link: link a0 = 2q takes (wvc_a1 + suffix past a1, prefix below a0) — the same sums
        const float X = fmaf(l, sC, nu * pC);
        const float Y = fmaf(l, sS, nu * pS);
        const float thd_prev = dpp<0x111>(THD) * m1;
        const float qd = THD - thd_prev;
        const float ve = fmaf(-damp, qd, v);
        const float ve_next = dpp<0x101>(ve) * u1;
        float r = ve - ve_next;
        r = fmaf(C, Y, fmaf(-Sn, X, fmaf(-g, vc, r)));
        float col[N];
        unroll_seq([&](auto a_c) {
            constexpr int a = decltype(a_c)::value;
            col[a] = fmaf(obc<a>(lc, upper), vc, fmaf(obc<a>(ls, upper), vs, corr[a]));
        }, std::make_integer_sequence<int, N>{});
        float Ln[N][N], yn[N];
        unroll_seq([&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            const float nrd = __builtin_amdgcn_rcpf(-obc<j>(col[j], upper));
            yn[j] = obc<j>(r, upper) * nrd;
            r = fmaf(yn[j], col[j], r);
            unroll_seq([&](auto k_c) {
                constexpr int kk = decltype(k_c)::value;
                if constexpr (kk > j) {
                    Ln[kk][j] = obc<kk>(col[j], upper) * nrd;
                    col[kk] = fmaf(Ln[kk][j], col[j], col[kk]);
                }
            }, std::make_integer_sequence<int, N>{});
        }, std::make_integer_sequence<int, N>{});
        float x[N];
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            float e = -yn[i];
#pragma unroll
            for (int kk = N - 1; kk > i; --kk) e = fmaf(Ln[kk][i], x[kk], e);
            x[i] = e;
        }
        float xp = 0.f;
#pragma unroll
        for (int a = 0; a < N; ++a) xp = p == a ? x[a] : xp;
        THD = fmaf(xp, dt, THD);
        TH = fmaf(THD, dtr, TH);
        angles();
    }
    if (k < K && p < N) out[(size_t)k * 8 + p] = TH;
}

// ------------------------------------------------------------------------------------------------ host
#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

template <class L>
static double time_ms(L launch, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int i = 0; i < reps + 3; ++i) {
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (i >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 16384, T = argc > 2 ? atoi(argv[2]) : 128;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    if (K < 1 || K % 64 || T < 1 || T > 4096) {
        fprintf(stderr, "K a multiple of 64, 1 <= T <= 4096\n");
        return 1;
    }
    float *oq, *oo;
    CHECK(hipMalloc(&oq, (size_t)K * 8 * sizeof(float)));
    CHECK(hipMalloc(&oo, (size_t)K * 8 * sizeof(float)));
    CHECK(hipMemset(oq, 0, (size_t)K * 8 * sizeof(float)));
    CHECK(hipMemset(oo, 0, (size_t)K * 8 * sizeof(float)));
    const int gq = K * 4 / NT, go = K * 8 / NT;
    const double tq = time_ms([&] { hipLaunchKernelGGL(quad_kernel, dim3(gq), dim3(NT), 0, 0, K, T, oq); }, reps);
    CHECK(hipGetLastError());
    const double to = time_ms([&] { hipLaunchKernelGGL(oct_kernel, dim3(go), dim3(NT), 0, 0, K, T, oo); }, reps);
    CHECK(hipGetLastError());
    std::vector<float> hq((size_t)K * 8), ho((size_t)K * 8);
    CHECK(hipMemcpy(hq.data(), oq, hq.size() * sizeof(float), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(ho.data(), oo, ho.size() * sizeof(float), hipMemcpyDeviceToHost));
    double maxd = 0.0;
    for (int k = 0; k < K; ++k)
        for (int a = 0; a < N; ++a) maxd = std::max(maxd, (double)fabsf(hq[(size_t)k * 8 + a] - ho[(size_t)k * 8 + a]));
    printf("{\"K\": %d, \"T\": %d, \"quad_ms\": %.4f, \"oct_ms\": %.4f, \"quad_ns_per_step\": %.1f, "
           "\"oct_ns_per_step\": %.1f, \"oct_swizzle\": %d, \"max_abs_diff_theta\": %.3g}\n",
           K, T, tq, to, tq * 1e6 / T, to * 1e6 / T, OCT_SWIZZLE, maxd);
    CHECK(hipFree(oq));
    CHECK(hipFree(oo));
    return 0;
}
