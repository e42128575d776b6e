// FETCH_SIZE / WRITE_SIZE calibration for the rollout's access pattern
// (diagnostic tool).  Reads NBUF rotating [T][K][2] fp32 noise buffers with the
// rollout kernel's pattern — lane k loads the 8-byte row element eps[t][k] for
// t = 0..T-1, 256-thread workgroups over k — and writes 4 bytes per thread.
// Known bytes per launch: read T*K*8, written K*4.  Run under
//   rocprofv3 --pmc FETCH_SIZE  --kernel-include-regex calib -- ./calib_fetch
//   rocprofv3 --pmc WRITE_SIZE  --kernel-include-regex calib -- ./calib_fetch
// and divide the counter (KB) by the known bytes.
// `./calib_fetch 4`: the chain kernel's pattern instead — 4-byte row elements
// eps[t][d][k], d < 7 (config 5's [T][n][K] layout), K = 131072, T = 16.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void calib_rows(const float2* __restrict__ noise, int K, int T, float* out) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
        const float2 e = noise[(size_t)t * K + k];
        acc += e.x * 0.5f + e.y;
    }
    out[k] = acc;
}

__global__ __launch_bounds__(256) void calib_rows4(const float* __restrict__ noise, int K, int T, float* out) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    float acc = 0.f;
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int d = 0; d < 7; ++d) acc = fmaf(acc, 0.5f, noise[((size_t)t * 7 + d) * K + k]);
    out[k] = acc;
}

static int chain_pattern() {
    const int K = 131072, T = 16, NBUF = 10, LAUNCHES = 20;
    const size_t bytes = (size_t)K * T * 7 * sizeof(float);
    float* buf[NBUF];
    float* out;
    for (int i = 0; i < NBUF; ++i) {
        hipMalloc(&buf[i], bytes);
        hipMemset(buf[i], 0, bytes);
    }
    hipMalloc(&out, K * sizeof(float));
    for (int i = 0; i < LAUNCHES; ++i)
        hipLaunchKernelGGL(calib_rows4, dim3((K + 255) / 256), dim3(256), 0, 0, buf[i % NBUF], K, T, out);
    hipDeviceSynchronize();
    printf("calib4: K=%d T=%d n=7 read %zu B, write %zu B per launch\n", K, T, bytes, (size_t)K * 4);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == '4') return chain_pattern();
    const int K = 65536, T = 64, NBUF = 10, LAUNCHES = 20;
    float2* buf[NBUF];
    float* out;
    for (int i = 0; i < NBUF; ++i) {
        hipMalloc(&buf[i], (size_t)K * T * sizeof(float2));
        hipMemset(buf[i], 0, (size_t)K * T * sizeof(float2));
    }
    hipMalloc(&out, K * sizeof(float));
    for (int i = 0; i < LAUNCHES; ++i)
        hipLaunchKernelGGL(calib_rows, dim3((K + 255) / 256), dim3(256), 0, 0, buf[i % NBUF], K, T, out);
    hipDeviceSynchronize();
    printf("calib: K=%d T=%d read %zu B, write %zu B per launch\n", K, T, (size_t)K * T * 8, (size_t)K * 4);
    return 0;
}
