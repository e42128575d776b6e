// VALU issue rate of independent instruction streams on gfx950 (diagnostic tool, not product): the ceiling the
// rollout kernel's valu_roofline is priced against (bench.py reads profiles/ubench_issue.json).
//
// Each loop iteration issues 16 instructions whose sources are loop-invariant registers and whose destinations
// are distinct registers never read in the loop: no dependency between them.  Workgroups of 256 threads (4
// waves, one per SIMD) with a dynamic LDS allocation that lets exactly W workgroups share a CU, on a grid of
// 256 * W workgroups: W waves on every SIMD of the chip, as in the rollout launch (W = 1 at K = 65536).
//
// Reported per instruction class and W:
//   ns_per_inst_wave  = the launch's event time / (iterations * 16): nanoseconds between one wave's
//                       instructions, every SIMD of the chip busy (the clock the chip picks under this load);
//   memtime_ticks     = the same per instruction in s_memtime ticks of wave 0;
//   memtime_mhz       = s_memtime ticks per microsecond of s_memrealtime (100 MHz): the rate s_memtime counts at.
// The mix row approximates the c3 horizon loop's instruction mix per state-step (75 of 116.5 VALU are the
// window scan: 30 v_pk_fma_f32, 30 v_and_or_b32, 15 v_min3_f32; the rest fma / packed dynamics, 2 sin/cos
// pairs): per 16, 4 v_pk_fma_f32, 4 v_and_or_b32, 2 v_min3_f32, 5 v_fma_f32, 1 v_sin_f32.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <algorithm>
#include <vector>

#define I1(INS, o) asm volatile(INS : "=v"(o) : "v"(b), "v"(c), "v"(d));
#define R16(INS)                                                                                            \
    I1(INS, o0) I1(INS, o1) I1(INS, o2) I1(INS, o3) I1(INS, o4) I1(INS, o5) I1(INS, o6) I1(INS, o7)        \
    I1(INS, o8) I1(INS, o9) I1(INS, oa) I1(INS, ob) I1(INS, oc) I1(INS, od) I1(INS, oe) I1(INS, of)
#define PK(q) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(q) : "v"(pb), "v"(pc), "v"(pd));

typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(256) void k(int iters, float* out, unsigned long long* clk) {
    extern __shared__ float lds[];   // sized by the launch so that W workgroups fit a CU; touched once
    float b = threadIdx.x * 0.5f, c = 0.999f, d = 0.001f;
    f2 pb = {b, c}, pc = {c, d}, pd = {d, b};
    float o0 = 0, o1 = 0, o2 = 0, o3 = 0, o4 = 0, o5 = 0, o6 = 0, o7 = 0, o8 = 0, o9 = 0, oa = 0, ob = 0, oc = 0,
          od = 0, oe = 0, of = 0;
    f2 q0 = {}, q1 = {}, q2 = {}, q3 = {};
    if (threadIdx.x == 0) lds[0] = b;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if (OP == 0) { R16("v_fma_f32 %0, %1, %2, %3") }
        if (OP == 1) { R16("v_add_f32 %0, %1, %2 ; %3") }
        if (OP == 2) { PK(q0) PK(q1) PK(q2) PK(q3) PK(q0) PK(q1) PK(q2) PK(q3) PK(q0) PK(q1) PK(q2) PK(q3) PK(q0) PK(q1) PK(q2) PK(q3) }
        if (OP == 3) { R16("v_and_or_b32 %0, %1, %2, %3") }
        if (OP == 4) { R16("v_min3_f32 %0, %1, %2, %3") }
        if (OP == 5) { R16("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf ; %2 %3") }
        if (OP == 6) { R16("v_sin_f32 %0, %1 ; %2 %3") }
        if (OP == 7) {   // the c3 loop's mix (header)
            PK(q0) I1("v_and_or_b32 %0, %1, %2, %3", o0) I1("v_fma_f32 %0, %1, %2, %3", o1)
            PK(q1) I1("v_and_or_b32 %0, %1, %2, %3", o2) I1("v_min3_f32 %0, %1, %2, %3", o3)
            I1("v_fma_f32 %0, %1, %2, %3", o4) PK(q2) I1("v_and_or_b32 %0, %1, %2, %3", o5)
            I1("v_fma_f32 %0, %1, %2, %3", o6) I1("v_sin_f32 %0, %1 ; %2 %3", o7) PK(q3)
            I1("v_and_or_b32 %0, %1, %2, %3", o8) I1("v_min3_f32 %0, %1, %2, %3", o9)
            I1("v_fma_f32 %0, %1, %2, %3", oa) I1("v_fma_f32 %0, %1, %2, %3", ob)
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = o0 + o1 + o2 + o3 + o4 + o5 + o6 + o7 + o8 + o9 + oa + ob + oc + od + oe + of +
                                          q0.x + q1.x + q2.y + q3.y + lds[0];
    if ((threadIdx.x & 63) == 0) {   // per wave: loop start / end (s_memrealtime, s_memtime) and where it ran
        unsigned long long* w = clk + 8 * (blockIdx.x * 4 + threadIdx.x / 64);
        w[0] = r0;
        w[1] = r1;
        w[2] = t0;
        w[3] = t1;
        w[4] = ((unsigned long long)__builtin_amdgcn_s_getreg(0xF814) << 32) | __builtin_amdgcn_s_getreg(0xF804);
    }
}

template <int OP>
void run(const char* name, int W, float* out, unsigned long long* clk, bool json_first) {
    const int iters = 20000;
    const size_t lds = (size_t)(150 * 1024 / W);   // exactly W workgroups of this size fit the 160 KB of a CU
    dim3 grid(256 * W), block(256);
    hipFuncSetAttribute((const void*)k<OP>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k<OP>, grid, block, lds, 0, iters, out, clk);   // clock settle
    std::vector<float> ms;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(k<OP>, grid, block, lds, 0, iters, out, clk);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float t;
        hipEventElapsedTime(&t, e0, e1);
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const int nw = 256 * W * 4;
    std::vector<unsigned long long> h(8 * (size_t)nw);
    hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
    const double n = iters * 16.0;
    // per wave: realtime ns per instruction of its own loop; the launch's span of loop starts / ends; the most
    // waves whose loops overlap on one SIMD (key: XCC, SE, CU, SIMD from HW_ID)
    std::vector<double> per;
    unsigned long long s_min = ~0ull, s_max = 0, e_min = ~0ull, e_max = 0;
    double tick_ratio = 0;
    for (int i = 0; i < nw; ++i) {
        const unsigned long long* w = &h[8 * (size_t)i];
        per.push_back((w[1] - w[0]) * 10.0 / n);
        s_min = std::min(s_min, w[0]); s_max = std::max(s_max, w[0]);
        e_min = std::min(e_min, w[1]); e_max = std::max(e_max, w[1]);
        tick_ratio += (double)(w[3] - w[2]) / ((w[1] - w[0]) * 1e-2) / nw;
    }
    int max_overlap = 0;
    for (int i = 0; i < nw; ++i) {
        const unsigned long long* a = &h[8 * (size_t)i];
        const unsigned hw = (unsigned)a[4], xcc = (unsigned)(a[4] >> 32);
        int ov = 0;
        for (int j = 0; j < nw; ++j) {
            const unsigned long long* b = &h[8 * (size_t)j];
            const unsigned hwb = (unsigned)b[4], xccb = (unsigned)(b[4] >> 32);
            // HW_ID: SIMD_ID bits 5:4, CU_ID 11:8, SH_ID 12, SE_ID 15:13
            const bool same = (xcc & 15) == (xccb & 15) && ((hw >> 4) & 3) == ((hwb >> 4) & 3) &&
                              ((hw >> 8) & 0xFF) == ((hwb >> 8) & 0xFF);
            if (same && b[0] < a[1] && a[0] < b[1]) ++ov;
        }
        max_overlap = std::max(max_overlap, ov);
    }
    std::sort(per.begin(), per.end());
    printf("%s    {\"op\": \"%s\", \"waves_per_simd\": %d, \"event_ns_per_inst_wave\": %.4f, "
           "\"wave_ns_per_inst_p50\": %.4f, \"wave_ns_per_inst_min\": %.4f, \"wave_ns_per_inst_max\": %.4f, "
           "\"loop_start_spread_us\": %.2f, \"loop_end_spread_us\": %.2f, \"max_waves_overlapping_on_a_simd\": %d, "
           "\"memtime_mhz\": %.1f}",
           json_first ? "" : ",\n", name, W, ms[2] * 1e6 / n, per[nw / 2], per[0], per[nw - 1], (s_max - s_min) * 1e-2,
           (e_max - e_min) * 1e-2, max_overlap, tick_ratio);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 256 * 4 * sizeof(float));
    hipMalloc(&clk, 8 * 8 * 4096);
    printf("{\"tool\": \"tools/ubench_issue.hip\", \"rows\": [\n");
    bool first = true;
    for (int W : {1, 2, 4}) {
        run<7>("c3_mix", W, out, clk, first);
        first = false;
        run<0>("v_fma_f32", W, out, clk, false);
        run<1>("v_add_f32", W, out, clk, false);
        run<2>("v_pk_fma_f32", W, out, clk, false);
        run<3>("v_and_or_b32", W, out, clk, false);
        run<4>("v_min3_f32", W, out, clk, false);
        run<5>("v_mov_b32_dpp", W, out, clk, false);
        run<6>("v_sin_f32", W, out, clk, false);
    }
    printf("\n]}\n");
    return 0;
}
