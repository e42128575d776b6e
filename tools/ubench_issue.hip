// Lone-wave issue cost of independent VALU streams on gfx950 (diagnostic tool, not product).
// Each iteration issues 16 instructions whose sources are loop-invariant registers and whose
// destinations are 16 distinct registers never read in the loop: no dependency between them.
// One workgroup of 64*W threads per CU... W waves per SIMD: W blocks of 256 threads per CU.
// Reports shader cycles per wave-instruction from s_memtime (one wave's view) and from the event time.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R16(INS) \
    asm volatile(INS : "=v"(o0) : "v"(b), "v"(c), "v"(d)); asm volatile(INS : "=v"(o1) : "v"(c), "v"(d), "v"(b)); \
    asm volatile(INS : "=v"(o2) : "v"(d), "v"(b), "v"(c)); asm volatile(INS : "=v"(o3) : "v"(b), "v"(d), "v"(c)); \
    asm volatile(INS : "=v"(o4) : "v"(b), "v"(c), "v"(d)); asm volatile(INS : "=v"(o5) : "v"(c), "v"(d), "v"(b)); \
    asm volatile(INS : "=v"(o6) : "v"(d), "v"(b), "v"(c)); asm volatile(INS : "=v"(o7) : "v"(b), "v"(d), "v"(c)); \
    asm volatile(INS : "=v"(o8) : "v"(b), "v"(c), "v"(d)); asm volatile(INS : "=v"(o9) : "v"(c), "v"(d), "v"(b)); \
    asm volatile(INS : "=v"(oa) : "v"(d), "v"(b), "v"(c)); asm volatile(INS : "=v"(ob) : "v"(b), "v"(d), "v"(c)); \
    asm volatile(INS : "=v"(oc) : "v"(b), "v"(c), "v"(d)); asm volatile(INS : "=v"(od) : "v"(c), "v"(d), "v"(b)); \
    asm volatile(INS : "=v"(oe) : "v"(d), "v"(b), "v"(c)); asm volatile(INS : "=v"(of) : "v"(b), "v"(d), "v"(c));

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void k(int iters, float* out, unsigned long long* clk) {
    float b = threadIdx.x * 0.5f, c = 0.999f, d = 0.001f;
    f2 pb = {b, c}, pc = {c, d}, pd = {d, b};
    float o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0, o7 = 0, o8 = 0, o9 = 0, oa = 0, ob = 0, oc = 0,
          od = 0, oe = 0, of = 0;
    f2 q0 = {}, q1 = {}, q2 = {}, q3 = {}, q4 = {}, q5 = {}, q6 = {}, q7 = {};
    float acc = 0.f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { R16("v_fma_f32 %0, %1, %2, %3") }
        if (OP == 1) { R16("v_and_or_b32 %0, %1, %2, %3") }
        if (OP == 2) { R16("v_min3_f32 %0, %1, %2, %3") }
        if (OP == 3) { R16("v_add_f32 %0, %1, %2 ; %3") }
        if (OP == 4) { R16("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf ; %2 %3") }
        if (OP == 5) { R16("v_cndmask_b32_e64 %0, %1, %2, s[0:1] ; %3") }
        if (OP == 6) { R16("v_sin_f32 %0, %1 ; %2 %3") }
        if (OP == 7) {   // packed: 8 independent v_pk_fma_f32 twice
#define PK(q) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(q) : "v"(pb), "v"(pc), "v"(pd));
            PK(q0) PK(q1) PK(q2) PK(q3) PK(q4) PK(q5) PK(q6) PK(q7) PK(q0) PK(q1) PK(q2) PK(q3) PK(q4) PK(q5) PK(q6) PK(q7)
        }
        if (OP == 8) {   // mix: pk_fma, fma alternating
#define PKF(q, o) PK(q) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(o) : "v"(b), "v"(c), "v"(d));
            PKF(q0, o0) PKF(q1, o1) PKF(q2, o2) PKF(q3, o3) PKF(q4, o4) PKF(q5, o5) PKF(q6, o6) PKF(q7, o7)
        }
        if (OP == 9) { R16("v_mul_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf ; %3") }
        if (OP == 10) {   // a dependent chain of 16 v_fma_f32 (latency)
            for (int j = 0; j < 16; ++j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(c), "v"(d));
        }
        if (OP == 11) { R16("s_nop 0 ; %0 %1 %2 %3") }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = o0 + o1 + o2 + o3 + o4 + o5 + o6 + o7 + o8 + o9 + oa + ob + oc + od + oe + of +
                                          q0.x + q1.x + q2.x + q3.x + q4.y + q5.y + q6.y + q7.y + acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
void run(const char* name, int W, float* out, unsigned long long* clk) {
    const int iters = 4000;
    dim3 grid(256 * W), block(256);
    hipLaunchKernelGGL(k<OP>, grid, block, 0, 0, 10, out, clk);
    hipLaunchKernelGGL(k<OP>, grid, block, 0, 0, iters, out, clk);
    hipDeviceSynchronize();
    unsigned long long h[1];
    hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
    printf("%-10s W=%d  %6.2f shader cycles per instruction (one wave's s_memtime)\n", name, W, (double)h[0] / (iters * 16.0));
}

int main() {
    float* out; unsigned long long* clk;
    hipMalloc(&out, 256 * 256 * 4 * sizeof(float)); hipMalloc(&clk, 16);
    for (int W : {1, 2}) {
        run<0>("fma", W, out, clk);
        run<3>("add", W, out, clk);
        run<1>("and_or", W, out, clk);
        run<2>("min3", W, out, clk);
        run<7>("pk_fma", W, out, clk);
        run<8>("pk+fma", W, out, clk);
        run<4>("mov_dpp", W, out, clk);
        run<9>("mul_dpp", W, out, clk);
        run<5>("cndmask", W, out, clk);
        run<6>("sin", W, out, clk);
        run<11>("s_nop0", W, out, clk);
        run<10>("fma dep", W, out, clk);
    }
    return 0;
}
