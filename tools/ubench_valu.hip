// VALU issue-rate microbenchmark for gfx950 (diagnostic tool, not product).
// For each instruction: 8 independent chains per lane (inline asm), W waves per
// SIMD (W blocks of 256 threads per CU), N iterations.  Reports SIMD cycles per
// wave-instruction = clk * time / (instructions per wave * W), with the clock
// measured in-kernel (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHAIN8(INS)                                                              \
    asm volatile(INS : "+v"(a0) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a1) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a2) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a3) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a4) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a5) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a6) : "v"(b), "v"(c));                               \
    asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define CHAIN8T(INS, T)                                                          \
    asm volatile(INS : "+v"(d0) : "v"(db));                                      \
    asm volatile(INS : "+v"(d1) : "v"(db));                                      \
    asm volatile(INS : "+v"(d2) : "v"(db));                                      \
    asm volatile(INS : "+v"(d3) : "v"(db));                                      \
    asm volatile(INS : "+v"(d4) : "v"(db));                                      \
    asm volatile(INS : "+v"(d5) : "v"(db));                                      \
    asm volatile(INS : "+v"(d6) : "v"(db));                                      \
    asm volatile(INS : "+v"(d7) : "v"(db));

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void k(int iters, float* out, unsigned long long* clk) {
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float b = 0.999f, c = 0.001f;
    double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7, db = 1e-3;
    f2 p0 = {a0, a1}, p1 = {a1, a2}, p2 = {a2, a3}, p3 = {a3, a4}, p4 = {a4, a5}, p5 = {a5, a6}, p6 = {a6, a7}, p7 = {a7, a0}, pb = {b, c};
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { CHAIN8("v_fma_f32 %0, %1, %2, %0") }
        if (OP == 1) { CHAIN8("v_mul_f32 %0, %1, %0") }
        if (OP == 2) { CHAIN8("v_sin_f32 %0, %0") }
        if (OP == 3) { CHAIN8("v_rcp_f32 %0, %0") }
        if (OP == 4) { CHAIN8("v_and_or_b32 %0, %0, %1, %2") }
        if (OP == 5) { CHAIN8("v_min3_f32 %0, %0, %1, %2") }
        if (OP == 6) { asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d0) : "v"(a0)); asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d1) : "v"(a1));
                       asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d2) : "v"(a2)); asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d3) : "v"(a3));
                       asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d4) : "v"(a4)); asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d5) : "v"(a5));
                       asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d6) : "v"(a6)); asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(d7) : "v"(a7)); }
        if (OP == 7) { CHAIN8T("v_add_f64 %0, %0, %1", double) }
        if (OP == 8) { asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p0) : "v"(pb)); asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p1) : "v"(pb));
                       asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p2) : "v"(pb)); asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p3) : "v"(pb));
                       asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p4) : "v"(pb)); asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p5) : "v"(pb));
                       asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p6) : "v"(pb)); asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p7) : "v"(pb)); }
        if (OP == 9) { CHAIN8("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf") }
        if (OP == 10) { CHAIN8("v_fma_f32 %0, %0, %1, %2") }  // dependent chain per accumulator
        if (OP == 11) { CHAIN8("v_exp_f32 %0, %0") }
        if (OP == 12) { CHAIN8("v_cndmask_b32 %0, %0, %1, vcc") }
        if (OP == 13) { CHAIN8("v_add_u32 %0, %0, %1") }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 +
        (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7) + p0.x + p1.x + p2.x + p3.x + p4.y + p5.y + p6.y + p7.y;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP>
void run(const char* name, int W, float* out, unsigned long long* clk) {
    const int iters = 2000;
    dim3 grid(256 * W), block(256);
    hipLaunchKernelGGL(k<OP>, grid, block, 0, 0, 10, out, clk);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, grid, block, 0, 0, iters, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    const double instr = (double)iters * 8;   // per wave
    const double cyc = ms * 1e-3 * ghz * 1e9;
    printf("%-12s W=%d  %7.3f ms  clk %.2f GHz  SIMD cycles / wave-instr %.2f   (one wave: %.2f cyc/instr)\n", name, W, ms,
           ghz, cyc / (instr * W), (double)h[0] / instr);
}

int main() {
    float* out; unsigned long long* clk;
    hipMalloc(&out, 256 * 256 * 8 * sizeof(float)); hipMalloc(&clk, 16);
    for (int W : {1, 2, 4}) {
        run<0>("fma", W, out, clk);
        run<10>("fma(dep)", W, out, clk);
        run<1>("mul", W, out, clk);
        run<4>("and_or", W, out, clk);
        run<5>("min3", W, out, clk);
        run<13>("add_u32", W, out, clk);
        run<12>("cndmask", W, out, clk);
        run<9>("mov_dpp", W, out, clk);
        run<8>("pk_fma", W, out, clk);
        run<2>("sin", W, out, clk);
        run<11>("exp", W, out, clk);
        run<3>("rcp", W, out, clk);
        run<6>("cvt_f64_f32", W, out, clk);
        run<7>("add_f64", W, out, clk);
    }
    return 0;
}
