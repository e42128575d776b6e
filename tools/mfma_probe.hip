// Probe for a matrix-core window search (diagnostic tool, not product).
//
// The 30-slot window keys of 64 samples, key[slot][sample] = c'_slot - 2 p'_sample . r'_slot, form a
// [32 x 3] x [3 x 64] product.  This checks on the GPU, for v_mfma_f32_32x32x2_f32:
//   1. v_permlane32_swap_b32 semantics (which halves trade places);
//   2. the operand / result lane layout assumed below;
//   3. whether two chained MFMAs  D = mfma(A2, B2, mfma(A1, B1, 0))  with
//        A1 = (c', ry') B1 = (1, ay)   and   A2 = (rx', 0) B2 = (ax, -)
//      reproduce the VALU chain  fma(ax, rx', fma(ay, ry', c'))  bit for bit (they do if the
//      MFMA rounds each 2-term dot product + accumulator once);
//   4. the argmin (5-bit packed index, as mppi_device.h Search) against the VALU scan.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float f16v __attribute__((ext_vector_type(16)));

__device__ inline void swap32(float& a, float& b) {   // v_permlane32_swap_b32 a, b
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}

__global__ void swap_test(float* out) {
    const int l = threadIdx.x;
    float a = (float)l, b = (float)(100 + l);
    swap32(a, b);
    out[l] = a;
    out[64 + l] = b;
}

// keys: 32 slots {rx', ry', c', -} (slots 30, 31 padded with c' = 1e30); pts: p' per sample.
// out_m / out_f: [block][h][lane][r] keys from the MFMA / the VALU chain for the MFMA's (slot, sample)
// idx_m / idx_f: packed argmin per sample
__global__ __launch_bounds__(64) void probe(const float4* keys, const float2* pts, float* out_m, float* out_f,
                                            unsigned* idx_m, unsigned* idx_f) {
    const int l = threadIdx.x, hi = l >> 5, i = l & 31;
    const float4 kk = keys[i];
    const float A1 = hi ? kk.y : kk.z;   // k = 0: c', k = 1: ry'
    const float A2 = hi ? 0.f : kk.x;    // k = 0: rx', k = 1: 0
    const float2 p = pts[blockIdx.x * 64 + l];
    const float ax = -2.f * p.x, ay = -2.f * p.y;
    const float m = hi ? 1.f : 0.f, c1 = hi ? 0.f : 1.f;
    float X = ax, Y = ay;
    swap32(X, Y);   // assumed: X = [ax lo | ay lo], Y = [ax hi | ay hi]
    const float B1_0 = fmaf(X, m, c1), B1_1 = fmaf(ay, m, c1);
    const float B2_0 = ax, B2_1 = Y;
    const f16v z = {};
    const f16v D0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, B2_0, __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B1_0, z, 0, 0, 0), 0, 0, 0);
    const f16v D1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A2, B2_1, __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B1_1, z, 0, 0, 0), 0, 0, 0);
    float b0 = 3.0e38f, b1 = 3.0e38f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int slot = 8 * (r >> 2) + 4 * hi + (r & 3);
        const size_t o = (((size_t)blockIdx.x * 2 + 0) * 64 + l) * 16 + r;
        out_m[o] = D0[r];
        out_m[o + 64 * 16] = D1[r];
        // VALU reference for the same (slot, sample): sample j = 32 h + i
        const float4 ks = keys[slot];
        const float2 p0 = pts[blockIdx.x * 64 + i], p1 = pts[blockIdx.x * 64 + 32 + i];
        out_f[o] = fmaf(-2.f * p0.x, ks.x, fmaf(-2.f * p0.y, ks.y, ks.z));
        out_f[o + 64 * 16] = fmaf(-2.f * p1.x, ks.x, fmaf(-2.f * p1.y, ks.y, ks.z));
        b0 = fminf(b0, __uint_as_float((__float_as_uint(D0[r]) & ~31u) | (unsigned)slot));
        b1 = fminf(b1, __uint_as_float((__float_as_uint(D1[r]) & ~31u) | (unsigned)slot));
    }
    swap32(b0, b1);
    const float best = fminf(b0, b1);
    idx_m[blockIdx.x * 64 + l] = __float_as_uint(best) & 31u;
    // VALU scan of the sample's own 30 slots
    float bf = 3.0e38f;
    for (int s = 0; s < 30; ++s) {
        const float4 ks = keys[s];
        const float k = fmaf(ax, ks.x, fmaf(ay, ks.y, ks.z));
        bf = fminf(bf, __uint_as_float((__float_as_uint(k) & ~31u) | (unsigned)s));
    }
    idx_f[blockIdx.x * 64 + l] = __float_as_uint(bf) & 31u;
}

int main(int argc, char** argv) {
    const int nb = argc > 1 ? atoi(argv[1]) : 4096;
    float* d;
    hipMalloc(&d, 128 * 4);
    swap_test<<<1, 64>>>(d);
    float h[128];
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("permlane32_swap(a = lane, b = 100 + lane): a[0] %g a[31] %g a[32] %g a[63] %g | b[0] %g b[31] %g b[32] %g b[63] %g\n",
           h[0], h[31], h[32], h[63], h[64], h[95], h[96], h[127]);
    // window: 30 points on an arc of a radius-0.5 circle (xydq_circle-like spacing), centred coordinates
    float4 hk[32];
    double cx = 0, cy = 0;
    double wx[30], wy[30];
    for (int s = 0; s < 30; ++s) {
        const double th = 0.3 + 0.021 * s;
        wx[s] = 0.5 * cos(th) + 1.0;
        wy[s] = 0.5 * sin(th) + 0.2;
        cx += wx[s] / 30;
        cy += wy[s] / 30;
    }
    for (int s = 0; s < 32; ++s) {
        if (s < 30) {
            const float rx = (float)(wx[s] - cx), ry = (float)(wy[s] - cy);
            hk[s] = make_float4(rx, ry, rx * rx + ry * ry, 0.f);
        } else {
            hk[s] = make_float4(0.f, 0.f, 1e30f, 0.f);
        }
    }
    const size_t n = (size_t)nb * 64;
    float2* hp = (float2*)malloc(n * sizeof(float2));
    srand(7);
    for (size_t j = 0; j < n; ++j) {   // points around the window, some far
        const double u = (double)rand() / RAND_MAX, v = (double)rand() / RAND_MAX;
        const double sc = j % 8 == 0 ? 3.0 : 0.4;
        hp[j] = make_float2((float)((u - 0.5) * sc), (float)((v - 0.5) * sc));
    }
    float4* dk; float2* dp; float *dm, *df; unsigned *im, *jf;
    hipMalloc(&dk, sizeof(hk)); hipMalloc(&dp, n * sizeof(float2));
    const size_t nk = (size_t)nb * 2 * 64 * 16;   // keys: [block][h][lane][r]
    hipMalloc(&dm, nk * 4); hipMalloc(&df, nk * 4);
    hipMalloc(&im, n * 4); hipMalloc(&jf, n * 4);
    hipMemcpy(dk, hk, sizeof(hk), hipMemcpyHostToDevice);
    hipMemcpy(dp, hp, n * sizeof(float2), hipMemcpyHostToDevice);
    probe<<<nb, 64>>>(dk, dp, dm, df, im, jf);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    float* km = (float*)malloc(nk * 4); float* kf = (float*)malloc(nk * 4);
    unsigned* xm = (unsigned*)malloc(n * 4); unsigned* xf = (unsigned*)malloc(n * 4);
    hipMemcpy(km, dm, nk * 4, hipMemcpyDeviceToHost); hipMemcpy(kf, df, nk * 4, hipMemcpyDeviceToHost);
    hipMemcpy(xm, im, n * 4, hipMemcpyDeviceToHost); hipMemcpy(xf, jf, n * 4, hipMemcpyDeviceToHost);
    size_t bad = 0, ulp1 = 0, big = 0;
    for (size_t q = 0; q < nk; ++q) {
        unsigned a, b;
        memcpy(&a, &km[q], 4); memcpy(&b, &kf[q], 4);
        if (a != b) {
            ++bad;
            const long dd = labs((long)a - (long)b);
            if (dd <= 1) ++ulp1; else if (fabsf(km[q] - kf[q]) > 1e-3f * fabsf(kf[q]) + 1e-6f) ++big;
        }
    }
    size_t idx_bad = 0;
    for (size_t j = 0; j < n; ++j) idx_bad += xm[j] != xf[j];
    printf("keys: %zu of %zu differ in bits (%zu by 1 ulp, %zu beyond 1e-3 rel: layout wrong if nonzero)\n", bad, nk, ulp1, big);
    printf("argmin: %zu of %zu samples differ from the VALU scan\n", idx_bad, n);
    return 0;
}
