// mppi_rocm.hip — MI355X (gfx950, CDNA4) MPPI rollout-and-reduce engine.
//
// The hot path of junofficial/mppi_RobotArm control.py:81-118 (K samples x T
// steps of: Gaussian control perturbation -> 2-link arm forward dynamics
// (_F, control.py:234-263) -> windowed nearest-waypoint stage cost (_c /
// _get_nearest_waypoint, control.py:174-232) + control cost (control.py:106)
// -> terminal cost (control.py:109) -> soft-min weights (control.py:297-314)
// -> weighted noise sum (control.py:115-118)), written for CDNA4 directly:
//
//  * rollout_kernel<LPS>: LPS lanes of a 64-wide wave per sample (1, 2, 4, 8 or 16).
//    The serial T loop runs per lane in fp32 registers; the 30-waypoint
//    argmin is split over the LPS lanes of a sample and closed with DPP
//    quad_perm min (no LDS, no MFMA: the work is element-wise VALU).  The
//    per-step noise row eps[t][k][:] is one coalesced 8-B-per-lane load,
//    prefetched four steps ahead.  S accumulates in fp64.
//  * the block epilogue turns its samples into a log-sum-exp partial
//    {rho_b, eta_b, N_b[T][2]} (only samples with non-zero weight are
//    visited) and publishes it write-through.  Default (grid co-resident):
//    tagged granules polled by workgroup 0, which merges every row directly
//    (or the first workgroup of each group of 16, then workgroup 0, when many
//    rows carry weight); larger grids: arrival counters and the last arriver
//    merges.  One launch covers control.py:81-118.  With MPPI_FLAG_FUSED_UPDATE
//    the merging workgroup also applies the median filter / update / shift of
//    control.py:122-149 into the ping-pong step block for the next launch.
//  * merge_kernel: the same merge over the all-gathered per-device partials
//    (multi-GPU), traj_kernel: trajectory re-roll (control.py:129-145),
//    philox_noise_kernel: counter-based Gaussian noise.
//
// C ABI: include/mppi_rocm.h.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <type_traits>

#include "mppi_device.h"
#include "mppi_host.h"
#include "mppi_rocm.h"

namespace {

using namespace mppi;

constexpr int kThreads = 256;

// The observed state and the window of a step: a kernel argument, by value
// (1 KiB of kernarg), so a control step stages its inputs without a copy call.
struct alignas(16) StepStatic {
    float4 win[kSlots];   // rx, ry, rdq1, rdq2 of window slot j (lookup after argmin)
    float4 key[kSlots];   // -2 rx', -2 ry', c' = rx'^2 + ry'^2 (centred), 0; pads c' = 1e30
    float4 x0;            // q1, q2, dq1, dq2
    float4 ctr;           // window centre (cx, cy), W, 0
};

// Device-resident nominal (ping-pong pair in the context): launch n reads one
// block and its fused update writes the next nominal into the other.
struct alignas(16) DevStep {
    float4 ua[kMaxT];     // u0, u1, a0, a1 (a = (gamma u_t)^T Sigma^-1), fp32
    double u[kMaxT][2];   // nominal control sequence, fp64 (device closed loop)
};

// Launch constants (kernel argument, by value).
struct KConst {
    int K_local, T, k_offset, k_exploit, nblocks, acquire;  // acquire: counter hand-off at > 1 workgroup/CU
    float dt, fk1, fk2;
    float A, B, D, E, P, Q;          // dynamics coefficients (see dyn_step)
    float sw[4], tw[4];              // stage / terminal weights x 10000
    double lambda, inv_lambda, gamma;
    double sig_inv[4];
};

// One semi-implicit Euler step of _F (control.py:234-263) in closed form:
//   M = [[A + B c2, D + E c2], [D + E c2, D]]   (M22 = m2 lc2^2 + l2 = D)
//   h = E s2,  G = [P c1 + Q c12, Q c12],  C dq = [-h dq2 (2 dq1 + dq2), h dq1^2]
//   ddq = M^-1 (v - C dq - G);  dq += ddq dt;  q += dq dt
// written on register pairs, so most of it issues as v_pk_* (two fp32 lanes
// per instruction):
//  * the joint angles are kept in revolutions (q / 2 pi), the unit of the
//    hardware v_sin_f32 / v_cos_f32, so no scaling per evaluation;
//  * c2/s2 come from the angle-difference identities of the cached (cos, sin)
//    of q1 and q1 + q2 — two packed ops — so a step evaluates exactly two
//    sincos (of the NEW q), shared by the next step's dynamics and this
//    step's kinematics;
//  * the constants live in VGPR pairs (DynK) so a packed op never needs a
//    second scalar operand moved in.
struct Arm {
    f32x2 Q;      // (q1, q2) / (2 pi)
    f32x2 dq;     // (dq1, dq2)
    f32x2 cs1;    // (cos q1, sin q1)
    f32x2 cs12;   // (cos(q1 + q2), sin(q1 + q2))
};

// Per-launch constants in VGPR pairs (made lane-opaque once, before the loop:
// as uniform values the compiler would keep them in SGPRs and move one into a
// VGPR at every packed use).
struct DynK {
    f32x2 zB, DA;      // (0, B), (D, A): (D, M11) = DA + zB c2
    f32x2 ED;          // (E, D): M12 = D + E c2, h = E s2
    f32x2 nP0, nQ;     // (-P, 0), (-Q, -Q): v - G
    f32x2 dt2;         // (dt, dt / (2 pi))
    f32x2 fk;          // (fk1, fk2)
    f32x2 ctr;         // window centre
    f32x2 w01, w23;    // stage weights x 10000
};

template <class V>
__device__ __forceinline__ V vgpr_opaque(V v) {
    asm volatile("" : "+v"(v));
    return v;
}

// One kernel-argument field as its own scalar: built straight from adjacent
// fields, the vector pairs below made LLVM copy (dt, fk1, fk2) into a private
// array that was then promoted to LDS — which costs the kernel a dispatch-packet
// read per wave and spread the workgroup starts over 13 us (measured).
__device__ __forceinline__ float arg_f(const float& f) {
    float x = f;
    asm volatile("" : "+s"(x));
    return x;
}

__device__ __forceinline__ DynK make_dynk(const KConst& c, float cx, float cy) {
    const float A = arg_f(c.A), B = arg_f(c.B), D = arg_f(c.D), E = arg_f(c.E), P = arg_f(c.P), Q = arg_f(c.Q);
    const float dt = arg_f(c.dt), fk1 = arg_f(c.fk1), fk2 = arg_f(c.fk2);
    DynK k;
    k.zB = vgpr_opaque(f32x2{0.f, B});
    k.DA = vgpr_opaque(f32x2{D, A});
    k.ED = vgpr_opaque(f32x2{E, D});
    k.nP0 = vgpr_opaque(f32x2{-P, 0.f});
    k.nQ = vgpr_opaque(f32x2{-Q, -Q});
    k.dt2 = vgpr_opaque(f32x2{dt, dt * 0.15915494309189535f});
    k.fk = vgpr_opaque(f32x2{fk1, fk2});
    k.ctr = vgpr_opaque(f32x2{cx, cy});
    k.w01 = vgpr_opaque(f32x2{arg_f(c.sw[0]), arg_f(c.sw[1])});
    k.w23 = vgpr_opaque(f32x2{arg_f(c.sw[2]), arg_f(c.sw[3])});
    return k;
}

__device__ __forceinline__ f32x2 splat(float x) { return f32x2{x, x}; }

// (cos, sin) of an angle given in revolutions
__device__ __forceinline__ f32x2 cossin_rev(float a) { return f32x2{__builtin_amdgcn_cosf(a), __builtin_amdgcn_sinf(a)}; }

__device__ __forceinline__ void arm_init(Arm& x, float4 x0) {
    x.Q = f32x2{x0.x, x0.y} * 0.15915494309189535f;
    x.dq = f32x2{x0.z, x0.w};
    x.cs1 = cossin_rev(x.Q.x);
    x.cs12 = cossin_rev(x.Q.x + x.Q.y);
}

// (c2, s2) = (c12 c1 + s12 s1, s12 c1 - c12 s1) from cs1 = (c1, s1), cs12 =
// (c12, s12): the swap and negation of cs12 are operand modifiers of the one
// v_pk_fma (op_sel / op_sel_hi pick the halves, neg_hi negates c12), which the
// compiler would otherwise build with a v_xor and two v_mov.
__device__ __forceinline__ f32x2 cos_sin_diff(f32x2 cs1, f32x2 cs12) {
    const f32x2 m = cs12 * splat(cs1.x);
    f32x2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
        : "=v"(r) : "v"(cs12), "v"(cs1), "v"(m));
    return r;
}

__device__ __forceinline__ void arm_step(Arm& x, f32x2 v, const DynK& k) {
    const float c1 = x.cs1.x, c12 = x.cs12.x;
    const f32x2 cs2 = cos_sin_diff(x.cs1, x.cs12);
    const float c2 = cs2.x, s2 = cs2.y;
    const f32x2 DM11 = __builtin_elementwise_fma(k.zB, splat(c2), k.DA);   // (D, M11)
    const float M12 = fmaf(k.ED.x, c2, k.ED.y);
    const float h = k.ED.x * s2;
    const f32x2 w = __builtin_elementwise_fma(k.nQ, splat(c12), __builtin_elementwise_fma(k.nP0, splat(c1), v));
    const float dq1 = x.dq.x, dq2 = x.dq.y;
    const float hd1 = h * dq1;
    const f32x2 r = {fmaf(h * dq2, fmaf(2.f, dq1, dq2), w.x), fmaf(-hd1, dq1, w.y)};
    const float det = fmaf(DM11.y, k.ED.y, -(M12 * M12));
    const float rdet = __builtin_amdgcn_rcpf(det);
    const f32x2 ddq = __builtin_elementwise_fma(splat(-M12), f32x2{r.y, r.x}, DM11 * r) * splat(rdet);
    x.dq = __builtin_elementwise_fma(ddq, splat(k.dt2.x), x.dq);
    x.Q = __builtin_elementwise_fma(x.dq, splat(k.dt2.y), x.Q);
    x.cs1 = cossin_rev(x.Q.x);
    x.cs12 = cossin_rev(x.Q.x + x.Q.y);
}

// end effector (control.py:178-179): (fk1 c1 + fk2 c12, fk1 s1 + fk2 s12)
__device__ __forceinline__ f32x2 arm_fk(const Arm& x, const DynK& k) {
    return __builtin_elementwise_fma(splat(k.fk.x), x.cs1, splat(k.fk.y) * x.cs12);
}

// stage / terminal cost (control.py:185-198, weights x 10000): e = (ex, ey), f = (e1, e2)
__device__ __forceinline__ float cost_pk(f32x2 e, f32x2 f, f32x2 w01, f32x2 w23) {
    const f32x2 s = __builtin_elementwise_fma(f * w23, f, (e * w01) * e);
    return s.x + s.y;
}

using Scratch = MergeScratch<2 * kMaxT>;

// Median filter (scipy.ndimage.median_filter(size=10, mode='reflect'),
// control.py:319-327, window [t-5, t+4], valid for T >= 5), u += w_eps
// (control.py:126), shift (control.py:148-149) and the fp32 per-step constants
// of the next launch.  Thread 2t + d produces the shifted element u_next[t][d]
// = u[src][d] + median(src, d) with src = min(t + 1, T - 1) straight from the
// filtered w_eps in sm.weps (no second barrier); u_src = cur->u[src][d], read
// at kernel entry (nominal_src).  The pair (t, 0), (t, 1) meets through DPP.
__device__ __forceinline__ double nominal_src(const DevStep* st, int tid, int T) {
    const int t = tid >> 1, src = t + 1 < T ? t + 1 : T - 1;
    return tid < 2 * T ? st->u[src][tid & 1] : 0.0;
}
// cur->u[0][d] for threads 0 and 1 (the element the shift drops), else 0
__device__ __forceinline__ double nominal_first(const DevStep* st, int tid) {
    return tid < 2 ? st->u[0][tid] : 0.0;
}

// Host-mapped outputs of a drop-in step (mppi_step_dropin): hout (device view
// of coherent pinned host memory, nullable) receives
//   [0] flag word (= seq once the rest is written), [2..3] u_new[0],
//   [4 .. 4 + 2T) the shifted nominal u_next[t][d],
// so the host reads the step's result without a copy or a stream synchronise.
struct HostOut {
    double* p;
    unsigned seq;
};

// upd (nullable): the updated, not yet shifted controls u_new[t] in fp32, the
// base of the optimal trajectory (control.py:129-134, mppi_optimal_traj):
// u_new[t + 1] is this thread's shifted element, u_new[0] one more median.
// Every thread of the workgroup must call it (it ends with a barrier when
// host outputs are requested).
template <int NT>
__device__ void nominal_update_block(DevStep* nxt, const KConst& c, Scratch& sm, double u_src, double u_first,
                                     float* upd, HostOut ho, bool publish = true) {
    const int tid = threadIdx.x;
    const int T = c.T;
    if (tid < ((2 * T + 63) & ~63)) {   // whole waves: the DPP pairs stay complete
        const int t = tid >> 1, d = tid & 1;
        const int src = t + 1 < T ? t + 1 : T - 1;
        const double un = tid < 2 * T ? u_src + median_at(sm, src, d, T, 2) : 0.0;
        const double other = dpp_f64<0xB1>(un);   // quad_perm [1,0,3,2]: the partner element
        if ((upd || ho.p) && tid < 2) {
            const double u0 = u_first + median_at(sm, 0, d, T, 2);
            if (upd) upd[d] = (float)u0;
            if (ho.p) ho.p[2 + d] = u0;
        }
        if (tid < 2 * T) {
            if (upd && t + 1 < T) upd[2 * (t + 1) + d] = (float)un;
            if (ho.p) ho.p[4 + tid] = un;
            nxt->u[t][d] = un;
            if (d == 0) {
                const double u0 = un, u1 = other;
                const double g0 = c.gamma * u0, g1 = c.gamma * u1;
                const double a0 = g0 * c.sig_inv[0] + g1 * c.sig_inv[2];
                const double a1 = g0 * c.sig_inv[1] + g1 * c.sig_inv[3];
                nxt->ua[t] = make_float4((float)u0, (float)u1, (float)a0, (float)a1);
            }
        }
    }
    if (ho.p) {
        __threadfence_system();   // this thread's host stores are out before the barrier
        if (!publish) return;     // the caller publishes (after the exchange's verdict)
        __syncthreads();
        if (tid == 0) __hip_atomic_store(reinterpret_cast<unsigned*>(ho.p), ho.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------------------ rollout kernel

constexpr int kPF = 4;  // noise rows in flight per lane

// POLL: the partial rows travel as tagged granules (see st_gran) to consumer
// workgroups that poll for them — the first workgroup of each group of kGroup
// merges its group, workgroup 0 merges the groups — so no
// workgroup drains its stores or waits on a counter, and the merges overlap the
// stragglers.  Needs every workgroup resident at once (the host enables it
// when the grid is at most one workgroup per CU); correctness does not depend
// on placement or order, every value is tag-checked.  Otherwise (!POLL) the
// last workgroup to arrive on a counter merges (arrive_last).
template <int LPS, int NT, bool POLL>
__global__ __launch_bounds__(NT) void rollout_kernel(
    const KConst c, const StepStatic ss, const DevStep* __restrict__ st, const float2* __restrict__ noise,
    double* __restrict__ S_out, double* __restrict__ slab, double* __restrict__ gslab,
    unsigned* __restrict__ counters, double* __restrict__ partial_out, double* __restrict__ w_eps_out,
    DevStep* __restrict__ nxt, unsigned flags, const XDesc xd, unsigned* __restrict__ epoch, unsigned* __restrict__ tmo,
    float* __restrict__ upd, const HostOut ho, unsigned long long* __restrict__ dbg) {
    __shared__ float4 s_win[kSlots];
    __shared__ float4 s_ua[kMaxT + kPF];   // per-step constants (u_t, a_t); rows >= T repeat row T - 1
    __shared__ double s_redd[NT / 64];
    __shared__ int s_cnt[NT / 64];
    __shared__ int s_k[NT];
    __shared__ double s_e[NT];
    __shared__ unsigned s_flag;
    __shared__ Scratch sm;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k_raw = (blockIdx.x * NT + tid) / LPS;
    const bool valid = k_raw < c.K_local;
    const int k = valid ? k_raw : c.K_local - 1;
    const float exf = (c.k_offset + k) < c.k_exploit ? 1.f : 0.f;  // control.py:98-101
    const int K = c.K_local, T = c.T;

    STAMP(0, NOW());
#ifdef MPPI_STAMPS
    STAMP(8, (unsigned long long)__builtin_amdgcn_s_getreg(0xF804));   // HW_ID
    STAMP(9, (unsigned long long)__builtin_amdgcn_s_getreg(0xF814));   // XCC_ID
#endif
    // The first noise rows go out first: they depend on nothing and come from
    // HBM, so every other prologue load (step block, keys) overlaps them.
    const float2* np = noise + k;
    float2 ring[kPF];   // noise rows eps[t][k] in flight
#pragma unroll
    for (int j = 0; j < kPF; ++j) ring[j] = np[(size_t)(j < T ? j : T - 1) * K];
    // this launch's granule tag (device epoch + 1), fetched now so its latency is hidden
    const unsigned tag_v = POLL ? __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    // nominal element for the fused update, fetched now so its latency is hidden
    const double u_cur = (flags & MPPI_FLAG_FUSED_UPDATE) ? nominal_src(st, tid, T) : 0.0;
    const double u_first = (flags & MPPI_FLAG_FUSED_UPDATE) ? nominal_first(st, tid) : 0.0;
    // window row for the LDS copy: loaded unconditionally (a load inside the
    // tid < kSlots branch would be waited for right there), stored before the barrier
    const float4 wrow = ss.win[tid & (kSlots - 1)];
    Search<LPS> sr;
    sr.load(ss.key, ss.ctr, tid & (LPS - 1));
    Arm x;
    arm_init(x, ss.x0);
    const DynK dk = make_dynk(c, sr.cx, sr.cy);
    // the per-step constants go to LDS: the ring reads them there, so no scalar
    // load shares lgkmcnt with the deferred row lookup below
    for (int i = tid; i < T + kPF; i += NT) s_ua[i] = st->ua[i < T ? i : T - 1];
    if (tid < kSlots) s_win[tid] = wrow;
    __syncthreads();
    float4 uring[kPF];  // per-step constants (u_t, a_t), uniform
#pragma unroll
    for (int j = 0; j < kPF; ++j) uring[j] = s_ua[j < T ? j : T - 1];

    // Horizon loop (control.py:95-109): v = u + eps -> _F -> end effector ->
    // nearest waypoint -> stage cost + control cost, S in fp64.
    //
    // Deferred cost: the LDS row of step t's nearest waypoint is consumed one
    // step later, after step t + 1's dynamics, so the lookup's latency is
    // hidden.  The costs are still added in step order and folded into fp64
    // every kPF steps (S4), so S is the sum of the same fp32 terms.
    double S = 0.0;
    // fp32 partial sums over one 4-step block, folded into fp64 S: the two lanes
    // of a pair accumulate (w0 ex^2 + w2 e1^2 + a0 v1, w1 ey^2 + w3 e2^2 + a1 v2),
    // each term one v_pk_fma into the running pair
    f32x2 S4 = {0.f, 0.f};
    f32x2 ee = {0.f, 0.f}, ef = {0.f, 0.f};   // (ex, ey), (e1, e2) of the last step added
    float4 pr = make_float4(0.f, 0.f, 0.f, 0.f);
    f32x2 pp = {0.f, 0.f}, pd = {0.f, 0.f};   // pending step: end effector, joint rates
    auto add_pending = [&]() {
        // the row is taken only once this step's dynamics are done (the asm
        // needs x.cs12, the step's last result): left free, the scheduler pulls
        // the cost up next to the lookup and waits on the LDS round trip there
        f32x4 r = {pr.x, pr.y, pr.z, pr.w};
        asm volatile("" : "+v"(r) : "v"(x.cs12));
        ee = pp - f32x2{r.x, r.y};
        ef = pd - f32x2{r.z, r.w};
        S4 = __builtin_elementwise_fma(ef * dk.w23, ef, __builtin_elementwise_fma(ee * dk.w01, ee, S4));
    };
    // uniform LDS byte offset of step t's row of s_ua, held in a VGPR (advanced
    // once per 4 steps; the ring's reads add compile-time offsets)
    int ua_off = vgpr_opaque(0);
    // `slot` (= t % kPF) is a compile-time constant at every call, so the rings
    // stay in registers (a runtime index sends them to scratch).  H: step t - 1
    // exists — 0 no, 1 yes, 2 test t > 0 at run time.  LPS = 1 peels the first
    // step so the unrolled loop body is one basic block (-2.9% at K = 65536);
    // the LPS > 1 kernels keep the test (+5% when peeled at K = 4096).
    auto dstep = [&](int t, auto slot_c, auto h_c) {
        constexpr int slot = decltype(slot_c)::value;
        constexpr int H = decltype(h_c)::value;
        const bool h = H == 2 ? t > 0 : H == 1;
        // The ring slot is fully consumed before its refill is issued: if the old
        // value outlived the new load, the two would need different registers and
        // the loop back-edge a v_mov of the refill — which waits for the load
        // (s_waitcnt vmcnt(0) each iteration: 1.86x the step time, measured).
        // The empty volatile asm takes the slot's values at this point of the
        // program (volatile asm keeps its order against the previous step's
        // PIN_LOADS): otherwise the scheduler hoists their uses towards the loop
        // top, where waiting for them means waiting for every load in flight.
        f32x2 e = {ring[slot].x, ring[slot].y};
        f32x4 ua = {uring[slot].x, uring[slot].y, uring[slot].z, uring[slot].w};
        asm volatile("" : "+v"(e), "+v"(ua));
        // u[t] + eps (exploit) or eps, control.py:99-101
        const f32x2 v = __builtin_elementwise_fma(splat(exf), f32x2{ua.x, ua.y}, e);
        // (gamma u^T Sigma^-1) v, control.py:106
        S4 = __builtin_elementwise_fma(f32x2{ua.z, ua.w}, v, S4);
        const int tl = t + kPF < T ? t + kPF : T - 1;
        ring[slot] = np[(size_t)tl * K];
        uring[slot] = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(s_ua) + ua_off +
                                                       (kPF + slot) * (int)sizeof(float4));
        if (slot == kPF - 1) ua_off += kPF * (int)sizeof(float4);   // slot == t % kPF at every call
        PIN_LOADS();
        arm_step(x, v, dk);
        if (h) {
            add_pending();   // step t - 1
            if (slot == 0) {
                S += (double)(S4.x + S4.y);
                S4 = f32x2{0.f, 0.f};
            }
        }
        pp = arm_fk(x, dk);   // control.py:178-179
        pd = x.dq;
        const f32x2 d = pp - dk.ctr;
        pr = s_win[sr.nearest_d(d.x, d.y)];
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    using H2 = std::integral_constant<int, 2>;
    static_assert(kPF == 4, "unrolled for a 4-deep ring");
    int t = 0;
    STAMP(12, NOW());
    if constexpr (LPS == 1) {
        dstep(0, I0{}, H0{});
        for (t = 1; t + kPF <= T; t += kPF) {   // slots 1, 2, 3, 0
            dstep(t, I1{}, H1{});
            dstep(t + 1, I2{}, H1{});
            dstep(t + 2, I3{}, H1{});
            dstep(t + 3, I0{}, H1{});
#ifdef MPPI_STAMPS
            if (t == 1) STAMP(13, NOW());
            if (t + kPF == T / 2 + 1) STAMP(14, NOW());
#endif
        }
        if (t < T) dstep(t, I1{}, H1{});          // remainder: t % kPF == 1, 2, 3 in order
        if (t + 1 < T) dstep(t + 1, I2{}, H1{});
        if (t + 2 < T) dstep(t + 2, I3{}, H1{});
    } else {
        for (; t + kPF <= T; t += kPF) {
            dstep(t, I0{}, H2{});
            dstep(t + 1, I1{}, H2{});
            dstep(t + 2, I2{}, H2{});
            dstep(t + 3, I3{}, H2{});
#ifdef MPPI_STAMPS
            if (t == 0) STAMP(13, NOW());
            if (t + kPF == T / 2) STAMP(14, NOW());
#endif
        }
        if (t < T) dstep(t, I0{}, H2{});          // remainder: t % kPF == 0, 1, 2 in order
        if (t + 1 < T) dstep(t + 1, I1{}, H2{});
        if (t + 2 < T) dstep(t + 2, I2{}, H2{});
    }
    add_pending();                       // step T - 1
    S += (double)(S4.x + S4.y);
    S += (double)cost_pk(ee, ef, f32x2{arg_f(c.tw[0]), arg_f(c.tw[1])}, f32x2{arg_f(c.tw[2]), arg_f(c.tw[3])});  // terminal cost, control.py:109

    STAMP(1, NOW());
    const bool owner = valid && sr.sub == 0;
    if (S_out && owner) S_out[k] = S;

    // ---- workgroup partial: rho_b, eta_b, N_b (control.py:112-118 over this block)
    const int stride = 2 + 2 * T;
    const RowGeo geo(2 * T);   // 2T + 1 merged columns <= NT: one column chunk (host keeps T <= 127 at NT = 256)
    const int nrows = c.nblocks;
    const int ngroups = (nrows + kGroup - 1) / kGroup;
    constexpr int kValBytes = POLL ? 16 : 8;
    const __amdgpu_buffer_rsrc_t slab_r = rows_rsrc(slab, nrows * stride * kValBytes);
    const __amdgpu_buffer_rsrc_t gslab_r = rows_rsrc(gslab, ngroups * stride * kValBytes);
    const unsigned tag = __builtin_amdgcn_readfirstlane(tag_v);
    auto publish = [&](int idx, double v) {
        if constexpr (POLL) st_gran(slab_r, idx, v, tag);
        else st_wt(slab_r, idx, v);
    };
    const double rho_b = block_min_f64<NT>(owner ? S : INFINITY, sm);
    if (tid == 0) publish(blockIdx.x * stride, rho_b);   // the merger's first need, out at once
    // weights below 2^-64 of the block's best are dropped (see kMergeFloor)
    // fp64, like the reference's weights; a wave whose samples all lie below the
    // floor (exp(-44.4) = 2^-64: the usual case, S spread >> lambda) skips the exp
    const double warg = (rho_b - S) * c.inv_lambda;
    double wgt = 0.0;
    if (__any(owner && warg >= -45.0)) wgt = owner ? exp(warg) : 0.0;
    const bool nz = wgt >= kMergeFloor;
    const unsigned long long bal = __ballot(nz);
    const double esum = wave_sum_f64(nz ? wgt : 0.0);
    if (lane == 0) {
        s_cnt[wave] = __popcll(bal);
        s_redd[wave] = esum;
    }
    __syncthreads();
    int off = 0, nl = 0;
    double eta_b = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        off += (w < wave) ? s_cnt[w] : 0;
        nl += s_cnt[w];
        eta_b += s_redd[w];
    }
    if (nz) {
        const int pos = off + lanes_below(bal);
        s_k[pos] = k;
        s_e[pos] = wgt;
    }
    __syncthreads();
    // eta_b leaves next (rho_b left right after the block minimum): a poll merger
    // learns the global minimum and which rows carry weight before the slowest
    // workgroup's gather is done
    if (tid == 0) publish(blockIdx.x * stride + 1, eta_b);
    STAMP(15, NOW());
    nl = __builtin_amdgcn_readfirstlane(nl);
    if (nl <= kSparseMax) {
        // few weighted samples (the usual case: S spread >> lambda): column
        // threads gather eps[t][k_l] for the listed samples, all loads of a
        // column issued together
        const float* nf = reinterpret_cast<const float*>(noise);
        for (int col = tid; col < 2 * T; col += NT) {
            const float* base = nf + (size_t)(col >> 1) * K * 2 + (col & 1);
            publish(blockIdx.x * stride + 2 + col, gather_col(base, 2, s_k, s_e, nl));
        }
    } else {
        // dense weights: each wave takes whole rows eps[t][k0 : k0 + NS] (coalesced),
        // lane l owns samples l, l + 64, ...; the loads of kRowBatch rows are in
        // flight together, then one DPP wave reduction per row and component
        constexpr int NS = NT / LPS;               // samples of this workgroup
        constexpr int PER = (NS + 63) / 64;
        constexpr int kRowBatch = 4;
        const int k0 = blockIdx.x * NS;
        if (tid < NS) s_e[tid] = 0.0;
        __syncthreads();
        if (nz) s_e[k - k0] = wgt;
        __syncthreads();
        double w[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int ks = lane + 64 * i;
            w[i] = (ks < NS && k0 + ks < K) ? s_e[ks] : 0.0;
        }
        for (int tb = wave * kRowBatch; tb < T; tb += (NT / 64) * kRowBatch) {
            float2 e[kRowBatch][PER];
#pragma unroll
            for (int r = 0; r < kRowBatch; ++r) {
                const int tr = min(tb + r, T - 1);
#pragma unroll
                for (int i = 0; i < PER; ++i)
                    e[r][i] = noise[(size_t)tr * K + min(k0 + lane + 64 * i, K - 1)];  // w = 0 past K
            }
#pragma unroll
            for (int r = 0; r < kRowBatch; ++r) {
                double ax = 0.0, ay = 0.0;
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    ax = fma(w[i], (double)e[r][i].x, ax);
                    ay = fma(w[i], (double)e[r][i].y, ay);
                }
                ax = wave_sum_f64(ax);
                ay = wave_sum_f64(ay);
                if (lane == 0 && tb + r < T) {
                    publish(blockIdx.x * stride + 2 + 2 * (tb + r), ax);
                    publish(blockIdx.x * stride + 3 + 2 * (tb + r), ay);
                }
            }
        }
    }
    STAMP(2, NOW());
    STAMP(5, (unsigned long long)nl);
    const int g = blockIdx.x / kGroup;
    const int gsz = min(kGroup, nrows - g * kGroup);
    if constexpr (POLL) {
        // ---- level 1: the group's first workgroup polls and merges its rows (the first
        // dispatched are the first done, so the merger is waiting when the last row lands)
        if ((int)blockIdx.x != g * kGroup) return;
        STAMP(3, NOW());
        if (ngroups == 1) {
            merge_rows_block<NT, 1, true, true>(slab_r, 0, gsz, geo, c.inv_lambda, sm, nullptr, 0, partial_out, w_eps_out, tag, tmo);
        } else if (blockIdx.x == 0 && nrows <= kDirectRows &&
                   direct_merge<NT, 1, true>(slab_r, nrows, geo, c.inv_lambda, sm, partial_out, w_eps_out, tag, tmo, dbg)) {
            // few weighted rows: finished straight from the workgroup rows
        } else {
            merge_rows_block<NT, 1, false, true>(slab_r, g * kGroup, gsz, geo, c.inv_lambda, sm, &gslab_r, g, nullptr, nullptr, tag,
                                                 tmo);
            STAMP(10, NOW());
            // ---- level 2: workgroup 0 polls and merges the group rows
            if (blockIdx.x != 0) return;
            STAMP(4, NOW());
            merge_rows_block<NT, 1, true, true>(gslab_r, 0, ngroups, geo, c.inv_lambda, sm, nullptr, 0, partial_out,
                                                w_eps_out, tag, tmo);
        }
        // every workgroup read the epoch before publishing, and all have published
        if (threadIdx.x == 0) __hip_atomic_store(epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        // ---- level 1: the last workgroup of each group of kGroup merges the group
        if (!arrive_last(counters + g, (unsigned)gsz, &s_flag, c.acquire != 0)) return;
        STAMP(3, NOW());
        merge_rows_block<NT, 1, false, false>(slab_r, g * kGroup, gsz, geo, c.inv_lambda, sm, &gslab_r, g, nullptr, nullptr,
                                              0u, nullptr);
        STAMP(10, NOW());
        // ---- level 2: the last group merges the group rows and finishes the step
        if (!arrive_last(counters + ngroups, (unsigned)ngroups, &s_flag, c.acquire != 0)) return;
        STAMP(4, NOW());
        // the same decision as the poll form (identical results either way)
        if (!(ngroups > 1 && nrows <= kDirectRows &&
              direct_merge<NT, 1, false>(slab_r, nrows, geo, c.inv_lambda, sm, partial_out, w_eps_out, 0u, nullptr)))
            merge_rows_block<NT, 1, true, false>(gslab_r, 0, ngroups, geo, c.inv_lambda, sm, nullptr, 0, partial_out,
                                                 w_eps_out, 0u, nullptr);
    }
    STAMP(11, NOW());
    STAMP(6, (unsigned long long)sm.nrel);
    if (flags & MPPI_FLAG_EXCHANGE) {
        // the update is computed while the ranks' statuses travel (exchange_send_merge / exchange_verdict):
        // it lands in the ping-pong block and outputs the host takes only after a good verdict; on a failed
        // exchange the host keeps its block and ignores them (check_timeout), so no rank applies the update
        const unsigned xtag = exchange_send_merge<NT, 1>(xd, geo, c.inv_lambda, sm, w_eps_out, tmo);
        if (flags & MPPI_FLAG_FUSED_UPDATE) nominal_update_block<NT>(nxt, c, sm, u_cur, u_first, upd, ho, false);
        exchange_verdict<NT>(xd, geo, xtag, tmo);   // a barrier: every thread's host stores are out
        if ((flags & MPPI_FLAG_FUSED_UPDATE) && ho.p && threadIdx.x == 0)   // the host's wait ends, then reads tmo
            __hip_atomic_store(reinterpret_cast<unsigned*>(ho.p), ho.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (flags & MPPI_FLAG_FUSED_UPDATE) {
        nominal_update_block<NT>(nxt, c, sm, u_cur, u_first, upd, ho);
    }
    STAMP(7, NOW());
}

// Merge of the all-gathered per-device rows (multi-GPU), plus the fused update.
template <int NT>
__global__ __launch_bounds__(NT) void merge_kernel(const KConst c, const double* parts, int n, double* w_eps_out,
                                                   const DevStep* cur, DevStep* nxt, unsigned flags, float* upd,
                                                   const HostOut ho) {
    __shared__ Scratch sm;
    const int tid = threadIdx.x;
    const double u_cur = (flags & MPPI_FLAG_FUSED_UPDATE) ? nominal_src(cur, tid, c.T) : 0.0;
    const double u_first = (flags & MPPI_FLAG_FUSED_UPDATE) ? nominal_first(cur, tid) : 0.0;
    const __amdgpu_buffer_rsrc_t r = rows_rsrc(parts, n * (2 + 2 * c.T) * 8);
    merge_rows_block<NT, 1, true, false>(r, 0, n, RowGeo(2 * c.T), c.inv_lambda, sm, nullptr, 0, nullptr, w_eps_out,
                                         0u, nullptr);
    if (flags & MPPI_FLAG_FUSED_UPDATE) nominal_update_block<NT>(nxt, c, sm, u_cur, u_first, upd, ho);
}

// Trajectory re-roll (control.py:129-145): control(t) = base[(t-1) mod T] (+ eps).
// The output is the reference's [K][T][4] order: a sample's states are
// contiguous, so a lane writing its own state each step would scatter 16 B per
// lane at a T * 16 B stride.  The states go through an LDS tile of kTrajTB steps
// instead, and each flush writes whole kTrajTB * 16 B runs per sample (eight
// steps = one 128 B line), lane-contiguous.
constexpr int kTrajTB = 8;
// base: the controls, float2 elements bstride apart (1: a plain [T][2] array;
// 2: the (u, a) float4 rows of a DevStep, read in place)
template <bool NOISE>
__global__ __launch_bounds__(kThreads) void traj_kernel(const KConst c, const StepStatic ss,
                                                        const float2* __restrict__ base, int bstride,
                                                        const float2* __restrict__ noise, int Kn,
                                                        float4* __restrict__ out) {
    __shared__ float4 tile[kTrajTB][kThreads];
    const int tid = threadIdx.x;
    const int k0 = blockIdx.x * kThreads;
    const int k = min(k0 + tid, Kn - 1);   // lanes past Kn recompute the last sample, never stored
    const int nk = min(kThreads, Kn - k0);
    const int T = c.T;
    const float exf = NOISE ? ((c.k_offset + k) < c.k_exploit ? 1.f : 0.f) : 1.f;
    Arm x;
    arm_init(x, ss.x0);
    const DynK dk = make_dynk(c, 0.f, 0.f);
    // the noise of a whole tile is loaded two tiles ahead (a lane's per-step load
    // would otherwise be waited for every step: one wave per SIMD hides nothing)
    auto load_tile = [&](int t0, float2 (&d)[kTrajTB]) {
#pragma unroll
        for (int j = 0; j < kTrajTB; ++j) {
            const int t = min(t0 + j, T - 1);
            const int ti = t == 0 ? T - 1 : t - 1;
            d[j] = NOISE ? noise[(size_t)ti * c.K_local + k] : make_float2(0.f, 0.f);
        }
    };
    // one tile: its 8 steps, the states into the LDS tile, one coalesced flush
    auto tile_steps = [&](const float2 (&cur)[kTrajTB], int t0) {
        const int nt = min(kTrajTB, T - t0);
#pragma unroll
        for (int j = 0; j < kTrajTB; ++j) {
            if (j >= nt) break;
            const int t = t0 + j;
            const int ti = t == 0 ? T - 1 : t - 1;
            const float2 b = base[ti * bstride];
            f32x2 v = {b.x, b.y};
            if (NOISE) v = __builtin_elementwise_fma(splat(exf), v, f32x2{cur[j].x, cur[j].y});
            arm_step(x, v, dk);
            const f32x2 q = x.Q * 6.283185307179586f;
            tile[j][tid] = make_float4(q.x, q.y, x.dq.x, x.dq.y);
        }
        __syncthreads();
        // flush: element i of the block's nk * nt states -> sample i / nt, step i % nt
        for (int i = tid; i < nk * nt; i += kThreads) {
            const int s = i / nt, j = i - s * nt;
            out[(size_t)(k0 + s) * T + t0 + j] = tile[j][s];
        }
        __syncthreads();
    };
    // three register tiles in rotation, compile-time slots: tile i + 2's noise
    // is issued before tile i is stepped (~2 tiles of dynamics ahead of its use)
    float2 ta[kTrajTB], tb[kTrajTB], tc[kTrajTB];
    load_tile(0, ta);
    load_tile(kTrajTB, tb);
    for (int t0 = 0; t0 < T; t0 += 3 * kTrajTB) {
        load_tile(t0 + 2 * kTrajTB, tc);
        tile_steps(ta, t0);
        if (t0 + kTrajTB >= T) break;
        load_tile(t0 + 3 * kTrajTB, ta);
        tile_steps(tb, t0 + kTrajTB);
        if (t0 + 2 * kTrajTB >= T) break;
        load_tile(t0 + 4 * kTrajTB, tb);
        tile_steps(tc, t0 + 2 * kTrajTB);
    }
}

// Diagnostics / tests (mppi_debug_nearest): the nearest window slot of every
// sample and step as the rollout evaluates it — the same dyn_step and
// Search<1>::nearest on the same inputs, so the same fp32 positions and slots —
// with the end-effector position: slot[k][t], pos[k][t] = (px, py).
__global__ __launch_bounds__(kThreads) void nearest_debug_kernel(const KConst c, const StepStatic ss,
                                                                 const DevStep* __restrict__ st,
                                                                 const float2* __restrict__ noise, int Kn,
                                                                 int* __restrict__ slot, float2* __restrict__ pos) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= Kn) return;
    const int T = c.T;
    const float exf = (c.k_offset + k) < c.k_exploit ? 1.f : 0.f;
    Search<1> sr;
    sr.load(ss.key, ss.ctr, 0);
    Arm x;
    arm_init(x, ss.x0);
    const DynK dk = make_dynk(c, sr.cx, sr.cy);
    for (int t = 0; t < T; ++t) {
        const float4 ua = st->ua[t];
        const float2 e = noise[(size_t)t * c.K_local + k];
        arm_step(x, __builtin_elementwise_fma(splat(exf), f32x2{ua.x, ua.y}, f32x2{e.x, e.y}), dk);
        const f32x2 p = arm_fk(x, dk);
        const f32x2 d = p - dk.ctr;
        slot[(size_t)k * T + t] = (int)sr.nearest_d(d.x, d.y);
        pos[(size_t)k * T + t] = make_float2(p.x, p.y);
    }
}

// Philox4x32-10 + Box-Muller (mppi_device.h); eps = L z, L = chol(Sigma) (the
// arguments carry L x kBoxMullerScale, box_muller's constant).
// Grid (ceil(K_local / kThreads), ceil(T / 2)): blockIdx.y is the step pair, so
// no 64-bit divide per thread (it was ~half the kernel's instructions).
__global__ __launch_bounds__(kThreads) void philox_noise_kernel(int K_local, int T, long long k_offset,
                                                                unsigned long long seed,
                                                                unsigned long long step, float L00,
                                                                float L10, float L11, float2* out) {
    const int k = (int)blockIdx.x * kThreads + (int)threadIdx.x;
    if (k >= K_local) return;
    const int t0 = 2 * (int)blockIdx.y;
    const unsigned long long kg = (unsigned long long)(k_offset + k);
    const uint4 ctr = make_uint4((unsigned)kg, (unsigned)(kg >> 32), (unsigned)t0, (unsigned)step);
    const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32) ^ (unsigned)(step >> 32));
    const uint4 r = philox4x32_10(ctr, key);
    const float2 za = box_muller(r.x, r.y), zb = box_muller(r.z, r.w);
    const float z0 = za.x, z1 = za.y, z2 = zb.x, z3 = zb.y;
    out[(size_t)t0 * K_local + k] = make_float2(L00 * z0, fmaf(L10, z0, L11 * z1));
    if (t0 + 1 < T) out[(size_t)(t0 + 1) * K_local + k] = make_float2(L00 * z2, fmaf(L10, z2, L11 * z3));
}

}  // namespace

// ================================================================ host side

struct mppi_ctx {
    mppi_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    int lps = 1, nt = 256, nblocks = 0;
    KConst kc;
    StepStatic stat{};          // x0 + window of the next launch (a kernel argument)
    DevStep* d_step = nullptr;  // [2] ping-pong nominal
    int cur = 0;
    DevStep* h_step = nullptr;  // pinned staging of an uploaded nominal
    hipEvent_t staged = nullptr;
    bool stage_pending = false;     // a staging copy may still be reading h_step
    // the current device nominal is the one the last MPPI_FLAG_HOST_OUT launch
    // published (h_dout): a drop-in step whose u equals it uploads nothing
    bool nominal_published = false;
    bool x_flipped = false;          // the last launch flipped the ping-pong and exchanged (undone on MPPI_E_EXCHANGE)
    double* h_dout = nullptr;       // coherent host-mapped drop-in outputs (HostOut layout)
    double* d_dout = nullptr;       // its device view
    unsigned dseq = 0;
    double dropin_us[6] = {};       // phase ends of the last mppi_step_dropin (mppi_debug_dropin_times)
    double* d_slab = nullptr;
    double* d_gslab = nullptr;
    unsigned* d_counter = nullptr;  // [ngroups + 1] arrival counters (counter hand-off), then the epoch word
    unsigned* d_epoch = nullptr;    // granule epoch (poll hand-off), inside the d_counter block
    bool poll = false;              // granule hand-off (grid <= one workgroup per CU)
    unsigned* h_tmo = nullptr;      // host-mapped: a bounded in-launch spin gave up
    unsigned* d_tmo = nullptr;
    double* d_weps = nullptr;
    double* h_buf = nullptr;    // pinned D2H staging, 2 * kMaxT doubles
    float2* d_base = nullptr;   // traj base controls
    float2* h_base = nullptr;   // pinned
    float2* d_upd = nullptr;    // updated, unshifted controls of the last fused update (optimal trajectory)
    bool upd_valid = false;
    double* h_out = nullptr;    // pinned: nominal (2T fp64) + optimal trajectory (4T fp32) of mppi_get_step_outputs
    mppi_dropin_binding bind{};  // mppi_dropin_bind
    bool bound = false;
    std::chrono::steady_clock::time_point tick_t0{};   // start of the current mppi_dropin_tick (phase times)
    bool in_tick = false;
    bool tick_launched = false;     // mppi_dropin_tick_launch done, mppi_dropin_tick_wait pending
    std::chrono::steady_clock::time_point step_t0{};   // start of the current drop-in step (phase times)
    double sig_inv[4];
    unsigned long long* d_dbg = nullptr;  // diagnostic stamp buffer (MPPI_STAMPS builds)
    // node-level exchange (mppi_exchange_*): inbox, this rank's row, epoch, peer mappings
    XDesc xd{};
    void* d_inbox = nullptr;
    double* d_xrow = nullptr;
    unsigned* d_xepoch = nullptr;
    int xworld_alloc = 0;
    void* xopened[kMaxWorld] = {};
};

namespace mppi_host {
namespace {
thread_local std::string g_err;
}
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
const char* last_error() { return g_err.c_str(); }
unsigned exchange_timeout_ticks() {
    const char* e = getenv("MPPI_EXCHANGE_TIMEOUT_US");
    const long v = e ? strtol(e, nullptr, 10) : 0;
    return v > 0 && v < 40000000 ? (unsigned)(v * 100) : 0u;   // s_memrealtime runs at 100 MHz
}
}  // namespace mppi_host

namespace {
using mppi_host::exchange_timeout_ticks;
using mppi_host::fail;

#define HIP_TRY(expr)                                                                 \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(MPPI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return MPPI_OK;
}

template <int L, int N>
int occupancy(int* per_cu) {
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, (const void*)rollout_kernel<L, N, true>, N, 0);
}

int check_timeout(mppi_ctx* c) {
    // tmo[0]: a local hand-off gave up (kTmoLocal); tmo[1]: the exchange's verdict bits (mppi_device.h)
    const unsigned v = c->h_tmo ? __atomic_load_n(c->h_tmo, __ATOMIC_ACQUIRE) | __atomic_load_n(c->h_tmo + 1, __ATOMIC_ACQUIRE)
                                : 0u;
    if (!v) return MPPI_OK;
    c->h_tmo[0] = c->h_tmo[1] = 0;
    if (v == kTmoExchange) {
        // every rank of the step reports it and none applied the update: back to the nominal before the launch
        if (c->x_flipped) c->cur ^= 1;
        c->x_flipped = false;
        c->upd_valid = false;
        c->nominal_published = false;
        return fail(MPPI_E_EXCHANGE, "multi-GPU exchange: a rank's row did not arrive within the bound on every "
                                     "rank of this step; no rank applied the update (run the step again)");
    }
    if (v & kTmoSplit)
        return fail(MPPI_E_HIP, "multi-GPU exchange: this rank had every row but not every rank's verdict within "
                                "the bound; other ranks may have applied the step, so it cannot be re-run");
    return fail(MPPI_E_HIP, "in-launch hand-off timed out (workgroups not co-resident?); results invalid");
}

int auto_lps(int K_local) {
    // Measured on MI355X (tools/ubench_valu.hip, tools/stamps.py): a lone wave
    // issues a VALU op every ~6-8 cycles, 2 waves/SIMD ~4.4, 4 waves ~3.0.
    // Splitting the window search over LPS lanes multiplies the instructions
    // per sample by ~1.6 (LPS=2) / ~2.7 (LPS=4); at K = 65536 (one wave per
    // SIMD) one lane per sample won (37 vs 45 us span), so split only while
    // the grid would leave SIMDs empty, up to one wave per SIMD
    // (tools/gpu_lps_sweep.sh, us per fused step, LPS 2 / 4 / 8:
    // K=2048 T=32 16.0 / 15.3 / 14.6; K=4096 T=32 17.3 / 15.7 / 15.5;
    // K=8192 T=64 23.4 / 20.1 / 20.4; K=16384 T=64 23.3 / 20.2 / 26.9;
    // K=32768 T=64 23.9 / 29.5 / 53.0; LPS 4 / 8 / 16: K=2048 T=32 15.2 / 14.7 /
    // 14.4; K=4096 T=32 15.3 / 15.2 / 15.5; K=4096 T=64 19.5 / 19.1 / 19.0;
    // K=8192 T=32 16.4 / 16.7 / 19.9).
    const long long waves1 = ((long long)K_local + 63) / 64;
    if (waves1 >= 1024) return 1;
    if (waves1 >= 512) return 2;
    if (waves1 >= 128) return 4;
    if (waves1 >= 64) return 8;
    return 16;
}
}  // namespace

extern "C" {

void mppi_config_init(mppi_config* cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->param_gamma = NAN;   // lambda (1 - alpha), control.py:45
    cfg->arm = mppi_arm_params{1.0, 1.0, 1.0, 1.0, 0.5, 0.5, 9.81, 1.0, 1.0};   // sys_params.py:1-13, control.py:55-56
}

const char* mppi_last_error(void) { return mppi_host::last_error(); }

int mppi_ctx_create(const mppi_config* cfg, int device, void* stream, mppi_ctx** out) {
    if (!cfg || !out) return fail(MPPI_E_ARG, "null argument");
    *out = nullptr;
    if (cfg->T < 1 || cfg->T > MPPI_MAX_T) return fail(MPPI_E_ARG, "T must be in [1, 128]");
    if (cfg->K_local < 1 || cfg->K_total < cfg->K_local || cfg->k_offset < 0 ||
        cfg->k_offset + (long long)cfg->K_local > cfg->K_total)
        return fail(MPPI_E_ARG, "bad sample geometry (K_local, K_total, k_offset)");
    const double* S = cfg->sigma;
    const double det = S[0] * S[3] - S[1] * S[2];
    if (det == 0.0 || !isfinite(det)) return fail(MPPI_E_SINGULAR, "Singular matrix");
    mppi_ctx* c = new mppi_ctx();
    c->cfg = *cfg;
    c->device = device;
    c->stream = (hipStream_t)stream;
    c->sig_inv[0] = S[3] / det;
    c->sig_inv[1] = -S[1] / det;
    c->sig_inv[2] = -S[2] / det;
    c->sig_inv[3] = S[0] / det;
    int lps = cfg->lanes_per_sample > 0 ? cfg->lanes_per_sample : auto_lps(cfg->K_local);
    if (lps != 1 && lps != 2 && lps != 4 && lps != 8 && lps != 16) {
        delete c;
        return fail(MPPI_E_ARG, "lanes_per_sample must be 0, 1, 2, 4, 8 or 16");
    }
    c->lps = lps;
    // 512-thread workgroups when the grid fills every CU with one of them (8 waves:
    // two per SIMD); 256 otherwise.  MPPI_BLOCK=256|512 overrides (diagnostics).
    const long long lanes = (long long)cfg->K_local * lps;
    c->nt = lanes >= 512LL * 256 ? 512 : 256;
    if (const char* ev = getenv("MPPI_BLOCK")) c->nt = atoi(ev) == 512 ? 512 : 256;
    // a workgroup's merge thread owns one column of the 2T + 1 merged columns
    if (2 * cfg->T + 1 > c->nt) c->nt = 512;
    c->nblocks = (int)((lanes + c->nt - 1) / c->nt);
    if (c->nblocks > 1024 * 1024) {
        delete c;
        return fail(MPPI_E_ARG, "too many samples");
    }
    const mppi_arm_params& a = cfg->arm;
    KConst& k = c->kc;
    memset(&k, 0, sizeof(k));
    k.K_local = cfg->K_local;
    k.T = cfg->T;
    k.k_offset = cfg->k_offset;
    {
        const double thr = (1.0 - cfg->param_exploration) * (double)cfg->K_total;  // control.py:98
        long long kx = thr <= 0.0 ? 0 : (long long)ceil(thr);
        if (kx > cfg->K_total) kx = cfg->K_total;
        k.k_exploit = (int)kx;
    }
    k.nblocks = c->nblocks;
    k.dt = (float)cfg->delta_t;
    k.fk1 = (float)a.fk_l1;
    k.fk2 = (float)a.fk_l2;
    k.A = (float)(a.m1 * a.lc1 * a.lc1 + a.l1 + a.m2 * (a.l1 * a.l1 + a.lc2 * a.lc2) + a.l2);
    k.B = (float)(2.0 * a.m2 * a.l1 * a.lc2);
    k.D = (float)(a.m2 * a.lc2 * a.lc2 + a.l2);
    k.E = (float)(a.m2 * a.l1 * a.lc2);
    k.P = (float)((a.m1 * a.lc1 + a.m2 * a.l1) * a.g);
    k.Q = (float)(a.m2 * a.lc2 * a.g);
    for (int i = 0; i < 4; ++i) {
        k.sw[i] = (float)(cfg->stage_cost_weight[i] * 10000.0);     // control.py:185
        k.tw[i] = (float)(cfg->terminal_cost_weight[i] * 10000.0);  // control.py:198
    }
    k.lambda = cfg->param_lambda;
    k.inv_lambda = 1.0 / cfg->param_lambda;
    // control.py:45 fixes gamma at construction; the caller passes it as given
    k.gamma = isnan(cfg->param_gamma) ? cfg->param_lambda * (1.0 - cfg->param_alpha) : cfg->param_gamma;
    for (int i = 0; i < 4; ++i) k.sig_inv[i] = c->sig_inv[i];

    auto cleanup_fail = [&](int rc) {
        mppi_ctx_destroy(c);
        return rc;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return cleanup_fail(fail(MPPI_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)));
    // hand-off form: tagged-granule polling when every workgroup is resident at
    // once (at most one per CU, the measured form); arrival counters otherwise,
    // with an agent acquire once workgroups share CUs.  MPPI_HANDOFF=counter
    // forces the counter form (tests).
    int ncu = 0, per_cu = 0;
    if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
        return cleanup_fail(fail(MPPI_E_HIP, std::string("device attributes: ") + hipGetErrorString(e)));
    {
        int rc = 0;
        if (c->nt == 512)
            rc = lps == 1 ? occupancy<1, 512>(&per_cu) : lps == 2 ? occupancy<2, 512>(&per_cu)
               : lps == 4 ? occupancy<4, 512>(&per_cu) : lps == 8 ? occupancy<8, 512>(&per_cu)
               : occupancy<16, 512>(&per_cu);
        else
            rc = lps == 1 ? occupancy<1, 256>(&per_cu) : lps == 2 ? occupancy<2, 256>(&per_cu)
               : lps == 4 ? occupancy<4, 256>(&per_cu) : lps == 8 ? occupancy<8, 256>(&per_cu)
               : occupancy<16, 256>(&per_cu);
        if (rc != 0) per_cu = 0;
    }
    c->poll = per_cu >= 1 && c->nblocks <= ncu;
    if (const char* ev = getenv("MPPI_HANDOFF")) {
        if (!strcmp(ev, "counter")) c->poll = false;
    }
    k.acquire = (!c->poll && c->nblocks > ncu) ? 1 : 0;
    const size_t val = c->poll ? 16 : sizeof(double);  // granule or plain fp64
    const size_t slab = (size_t)c->nblocks * (2 + 2 * cfg->T) * val;
    const int ngroups = (c->nblocks + kGroup - 1) / kGroup;
    const size_t gslab = (size_t)ngroups * (2 + 2 * cfg->T) * val;
    const size_t ctr_bytes = ((size_t)(ngroups + 2) * sizeof(unsigned) + 255) & ~(size_t)255;
    if ((e = hipMalloc(&c->d_step, 2 * sizeof(DevStep))) != hipSuccess ||
        (e = hipMalloc(&c->d_slab, slab)) != hipSuccess ||
        (e = hipMalloc(&c->d_gslab, gslab)) != hipSuccess ||
        (e = hipMalloc(&c->d_counter, ctr_bytes)) != hipSuccess ||
        (e = hipMalloc(&c->d_weps, 2 * kMaxT * sizeof(double))) != hipSuccess ||
        (e = hipMalloc(&c->d_base, kMaxT * sizeof(float2))) != hipSuccess ||
        (e = hipMalloc(&c->d_upd, kMaxT * sizeof(float2))) != hipSuccess ||
        (e = hipHostMalloc(&c->h_out, 2 * kMaxT * sizeof(double) + 4 * kMaxT * sizeof(float), hipHostMallocDefault)) !=
            hipSuccess ||
        (e = hipHostMalloc(&c->h_step, sizeof(DevStep), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_buf, 2 * kMaxT * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_base, kMaxT * sizeof(float2), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_tmo, 256, hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_dout, (4 + 2 * kMaxT) * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent)) !=
            hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->d_dout, c->h_dout, 0)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->d_tmo, c->h_tmo, 0)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->staged, hipEventDisableTiming)) != hipSuccess ||
        (e = hipMemset(c->d_counter, 0, ctr_bytes)) != hipSuccess ||
        (e = hipMemset(c->d_slab, 0, slab)) != hipSuccess ||
        (e = hipMemset(c->d_gslab, 0, gslab)) != hipSuccess ||
        (e = hipMemset(c->d_step, 0, 2 * sizeof(DevStep))) != hipSuccess ||
        (e = hipMemset(c->d_weps, 0, 2 * kMaxT * sizeof(double))) != hipSuccess ||
        (e = hipDeviceSynchronize()) != hipSuccess)
        return cleanup_fail(fail(MPPI_E_HIP, std::string("allocation: ") + hipGetErrorString(e)));
    memset(c->h_step, 0, sizeof(DevStep));
    memset(c->h_dout, 0, (4 + 2 * kMaxT) * sizeof(double));
    c->h_tmo[0] = c->h_tmo[1] = 0;
    c->d_epoch = c->d_counter + ngroups + 1;
    *out = c;
    return MPPI_OK;
}

void mppi_ctx_destroy(mppi_ctx* c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipDeviceSynchronize();
    (void)hipFree(c->d_step);
    (void)hipFree(c->d_slab);
    (void)hipFree(c->d_counter);
    (void)hipFree(c->d_gslab);
    (void)hipFree(c->d_weps);
    (void)hipFree(c->d_base);
    (void)hipFree(c->d_upd);
    if (c->h_out) (void)hipHostFree(c->h_out);
    for (void* p : c->xopened)
        if (p) (void)hipIpcCloseMemHandle(p);
    (void)hipFree(c->d_inbox);
    (void)hipFree(c->d_xrow);
    (void)hipFree(c->d_xepoch);
    if (c->h_step) (void)hipHostFree(c->h_step);
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->h_base) (void)hipHostFree(c->h_base);
    if (c->h_tmo) (void)hipHostFree(c->h_tmo);
    if (c->h_dout) (void)hipHostFree(c->h_dout);
    if (c->staged) (void)hipEventDestroy(c->staged);
    delete c;
}

int mppi_set_stream(mppi_ctx* c, void* stream) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    c->stream = (hipStream_t)stream;
    return MPPI_OK;
}

int mppi_ctx_info(const mppi_ctx* c, int* lps, int* blocks, int* threads) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    if (lps) *lps = c->lps;
    if (blocks) *blocks = c->nblocks;
    if (threads) *threads = c->nt;
    return MPPI_OK;
}

}  // extern "C"

namespace {

// Stage a step's inputs.  The observed state and the window (with its centred
// search keys, fp64 on the host then fp32) go into the host copy c->stat, which
// every launch passes by value: no copy call.  A nominal u, when given, is
// uploaded into the current ping-pong block (one stream-ordered copy from
// pinned staging) — unless `skip_same` and u is exactly the nominal the last
// drop-in launch published, which that launch already left on the device.
int stage_inputs(mppi_ctx* c, const double* x0, const double* window, int W, const double* u, bool skip_same) {
    if (!x0 || !window) return fail(MPPI_E_ARG, "null argument");
    if (W < 1 || W > MPPI_SEARCH_LEN) return fail(MPPI_E_ARG, "window rows must be in [1, 30]");
    StepStatic& h = c->stat;
    double cx = 0.0, cy = 0.0;
    for (int j = 0; j < W; ++j) {
        cx += window[4 * j];
        cy += window[4 * j + 1];
    }
    cx /= W;
    cy /= W;
    for (int j = 0; j < kSlots; ++j) {
        if (j < W) {
            const double* r = window + 4 * j;
            h.win[j] = make_float4((float)r[0], (float)r[1], (float)r[2], (float)r[3]);
            const double rx = r[0] - cx, ry = r[1] - cy;
            h.key[j] = make_float4((float)(-2.0 * rx), (float)(-2.0 * ry), (float)(rx * rx + ry * ry), 0.f);
        } else {
            h.win[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            h.key[j] = make_float4(0.f, 0.f, kPadKey, 0.f);
        }
    }
    h.x0 = make_float4((float)x0[0], (float)x0[1], (float)x0[2], (float)x0[3]);
    h.ctr = make_float4((float)cx, (float)cy, (float)W, 0.f);
    if (!u) return MPPI_OK;
    const int T = c->cfg.T;
    if (skip_same && c->nominal_published && !memcmp(u, c->h_dout + 4, 2 * (size_t)T * sizeof(double)))
        return MPPI_OK;
    if (c->stage_pending) HIP_TRY(hipEventSynchronize(c->staged));  // staging block free again
    DevStep* d = c->h_step;
    const KConst& k = c->kc;
    for (int t = 0; t < T; ++t) {
        const double u0 = u[2 * t], u1 = u[2 * t + 1];
        const double g0 = k.gamma * u0, g1 = k.gamma * u1;  // ((gamma u^T) Sigma^-1), control.py:106
        const double a0 = g0 * k.sig_inv[0] + g1 * k.sig_inv[2];
        const double a1 = g0 * k.sig_inv[1] + g1 * k.sig_inv[3];
        d->ua[t] = make_float4((float)u0, (float)u1, (float)a0, (float)a1);
        d->u[t][0] = u0;
        d->u[t][1] = u1;
    }
    HIP_TRY(hipMemcpyAsync(c->d_step + c->cur, d, sizeof(DevStep), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->staged, c->stream));
    c->stage_pending = true;
    c->nominal_published = false;
    c->upd_valid = false;
    return MPPI_OK;
}

int launch_rollout(mppi_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags,
                   HostOut ho);

// The host-mapped output block of the next launch (MPPI_FLAG_HOST_OUT): a fresh
// sequence number, never 0 (the flag word's initial value).
HostOut next_host_out(mppi_ctx* c, unsigned flags) {
    if (!(flags & MPPI_FLAG_HOST_OUT)) return HostOut{nullptr, 0u};
    if (++c->dseq == 0) ++c->dseq;
    return HostOut{c->d_dout, c->dseq};
}

// Wait until the last MPPI_FLAG_HOST_OUT launch has published its outputs: a spin
// on the coherent host-mapped flag word (no interrupt, no copy); the launch's own
// errors surface through hipStreamQuery.
int wait_host_out(mppi_ctx* c) {
    if (c->dseq == 0) return fail(MPPI_E_ARG, "no MPPI_FLAG_HOST_OUT launch to wait for");
    const unsigned seq = c->dseq;
    volatile unsigned* flag = reinterpret_cast<volatile unsigned*>(c->h_dout);
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned long long n = 0; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq; ++n) {
        if ((n & 1023) == 1023) {
            const hipError_t e = hipStreamQuery(c->stream);
            if (e != hipSuccess && e != hipErrorNotReady)
                return fail(MPPI_E_HIP, std::string("fused step: ") + hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq)
                return fail(MPPI_E_HIP, "fused step finished without publishing its outputs");
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
                return fail(MPPI_E_HIP, "fused step: no result after 30 s");
        }
        __builtin_ia32_pause();
    }
    c->stage_pending = false;   // the launch ran, so every staging copy before it did too
    if (int rc = check_timeout(c)) return rc;
    c->nominal_published = true;
    c->x_flipped = false;
    return MPPI_OK;
}

// _F (control.py:234-263) in fp64 on the host: the mass matrix as written, its
// closed-form 2x2 inverse (np.linalg.inv), semi-implicit Euler.  Used for the one
// optimal trajectory of a drop-in step (control.py:129-134), O(T) host work.
void host_F(const mppi_arm_params& a, double dt, double* x, double u1, double u2) {
    const double q1 = x[0], q2 = x[1], dq1 = x[2], dq2 = x[3];
    double s2, c2;
    sincos(q2, &s2, &c2);   // glibc: the same values as sin() and cos()
    const double M11 = a.m1 * a.lc1 * a.lc1 + a.l1 + a.m2 * (a.l1 * a.l1 + a.lc2 * a.lc2 + 2 * a.l1 * a.lc2 * c2) + a.l2;
    const double M22 = a.m2 * a.lc2 * a.lc2 + a.l2;
    const double M12 = a.m2 * a.l1 * a.lc2 * c2 + a.m2 * a.lc2 * a.lc2 + a.l2;
    const double h = a.m2 * a.l1 * a.lc2 * s2;
    const double c1 = cos(q1), c12 = cos(q1 + q2);   // each evaluated once (the reference evaluates them twice)
    const double g1 = a.m1 * a.lc1 * a.g * c1 + a.m2 * a.g * (a.lc2 * c12 + a.l1 * c1);
    const double g2 = a.m2 * a.lc2 * a.g * c12;
    const double r1 = u1 - ((-h * dq2) * dq1 + (-h * dq1 - h * dq2) * dq2) - g1;
    const double r2 = u2 - ((h * dq1) * dq1 + 0.0 * dq2) - g2;
    const double det = M11 * M22 - M12 * M12;
    const double ddq1 = (M22 * r1 - M12 * r2) / det;
    const double ddq2 = (-M12 * r1 + M11 * r2) / det;
    x[2] = dq1 + ddq1 * dt;
    x[3] = dq2 + ddq2 * dt;
    x[0] = q1 + x[2] * dt;
    x[1] = q2 + x[3] * dt;
}

}  // namespace

extern "C" {

int mppi_set_step_inputs(mppi_ctx* c, const double* x0, const double* window, int W, const double* u) {
    if (!c) return fail(MPPI_E_ARG, "null argument");
    return stage_inputs(c, x0, window, W, u, false);
}

int mppi_rollout(mppi_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags) {
    if (!c || !noise_dev) return fail(MPPI_E_ARG, "null argument");
    if ((flags & MPPI_FLAG_HOST_OUT) && !(flags & MPPI_FLAG_FUSED_UPDATE))
        return fail(MPPI_E_ARG, "MPPI_FLAG_HOST_OUT needs MPPI_FLAG_FUSED_UPDATE");
    return launch_rollout(c, noise_dev, S_dev, partial_dev, flags, next_host_out(c, flags));
}

}  // extern "C"

namespace {
int launch_rollout(mppi_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags,
                   HostOut ho) {
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    if (flags & MPPI_FLAG_EXCHANGE) {
        if (c->xd.world < 1) return fail(MPPI_E_ARG, "MPPI_FLAG_EXCHANGE before mppi_exchange_attach");
        if (partial_dev) return fail(MPPI_E_ARG, "MPPI_FLAG_EXCHANGE merges on device: no partial_out");
        partial_dev = c->d_xrow;
    }
    const DevStep* cur = c->d_step + c->cur;
    DevStep* nxt = c->d_step + (c->cur ^ 1);
    const float2* nz = reinterpret_cast<const float2*>(noise_dev);
#define MPPI_LAUNCH(L, NTH, P)                                                                                   \
    hipLaunchKernelGGL((rollout_kernel<L, NTH, P>), dim3(c->nblocks), dim3(NTH), 0, c->stream, c->kc, c->stat, cur, nz, \
                       S_dev, c->d_slab, c->d_gslab, c->d_counter, partial_dev, c->d_weps, nxt, flags, c->xd,          \
                       c->d_epoch, c->d_tmo, reinterpret_cast<float*>(c->d_upd), ho, c->d_dbg)
#define MPPI_LAUNCH_P(L, NTH)                \
    do {                                     \
        if (c->poll) MPPI_LAUNCH(L, NTH, true);  \
        else MPPI_LAUNCH(L, NTH, false);     \
    } while (0)
    if (c->nt == 512) {
        if (c->lps == 1) MPPI_LAUNCH_P(1, 512);
        else if (c->lps == 2) MPPI_LAUNCH_P(2, 512);
        else if (c->lps == 4) MPPI_LAUNCH_P(4, 512);
        else if (c->lps == 8) MPPI_LAUNCH_P(8, 512);
        else MPPI_LAUNCH_P(16, 512);
    } else {
        if (c->lps == 1) MPPI_LAUNCH_P(1, 256);
        else if (c->lps == 2) MPPI_LAUNCH_P(2, 256);
        else if (c->lps == 4) MPPI_LAUNCH_P(4, 256);
        else if (c->lps == 8) MPPI_LAUNCH_P(8, 256);
        else MPPI_LAUNCH_P(16, 256);
    }
#undef MPPI_LAUNCH_P
#undef MPPI_LAUNCH
    const int rc = launch_check("rollout_kernel");
    if (rc == MPPI_OK && (flags & MPPI_FLAG_FUSED_UPDATE)) {
        c->cur ^= 1;
        c->upd_valid = true;
        c->nominal_published = false;   // until wait_host_out sees this launch's outputs
        c->x_flipped = (flags & MPPI_FLAG_EXCHANGE) != 0;   // undone if the exchange fails (check_timeout)
    }
    return rc;
}
}  // namespace

extern "C" {

int mppi_exchange_handle(mppi_ctx* c, int world, void* handle_out) {
    if (!c || !handle_out || world < 1 || world > kMaxWorld) return fail(MPPI_E_ARG, "bad argument");
    if (c->d_inbox && c->xworld_alloc != world) return fail(MPPI_E_ARG, "inbox already sized for another world");
    const int stride = 2 + 2 * c->cfg.T;
    if (!c->d_inbox) {
        const size_t bytes = (size_t)2 * world * (stride + 1) * 16;   // rows and statuses, two parities
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipExtMallocWithFlags(&c->d_inbox, bytes, hipDeviceMallocUncached));
        HIP_TRY(hipMemset(c->d_inbox, 0, bytes));
        HIP_TRY(hipMalloc(&c->d_xrow, stride * sizeof(double)));
        HIP_TRY(hipMalloc(&c->d_xepoch, 256));
        HIP_TRY(hipMemset(c->d_xepoch, 0, 256));
        HIP_TRY(hipDeviceSynchronize());
        c->xworld_alloc = world;
        c->xd.bytes = (int)bytes;
    }
    HIP_TRY(hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle_out), c->d_inbox));
    return MPPI_OK;
}

int mppi_exchange_attach(mppi_ctx* c, int rank, int world, const void* handles) {
    if (!c || !handles || world < 1 || rank < 0 || rank >= world) return fail(MPPI_E_ARG, "bad argument");
    if (!c->d_inbox || c->xworld_alloc != world) return fail(MPPI_E_ARG, "call mppi_exchange_handle(world) first");
    if (c->xd.world) return fail(MPPI_E_ARG, "already attached");
    HIP_TRY(hipSetDevice(c->device));
    const hipIpcMemHandle_t* h = static_cast<const hipIpcMemHandle_t*>(handles);
    for (int p = 0; p < world; ++p) {
        if (p == rank) {
            c->xd.peer[p] = c->d_inbox;
            continue;
        }
        void* ptr = nullptr;
        HIP_TRY(hipIpcOpenMemHandle(&ptr, h[p], hipIpcMemLazyEnablePeerAccess));
        c->xopened[p] = ptr;
        c->xd.peer[p] = ptr;
    }
    c->xd.row = c->d_xrow;
    c->xd.epoch = c->d_xepoch;
    c->xd.rank = rank;
    c->xd.world = world;
    c->xd.timeout_ticks = exchange_timeout_ticks();
    return MPPI_OK;
}

int mppi_merge_partials(mppi_ctx* c, const double* partials_dev, int n, unsigned flags) {
    if (!c || !partials_dev || n < 1) return fail(MPPI_E_ARG, "bad argument");
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    if ((flags & MPPI_FLAG_HOST_OUT) && !(flags & MPPI_FLAG_FUSED_UPDATE))
        return fail(MPPI_E_ARG, "MPPI_FLAG_HOST_OUT needs MPPI_FLAG_FUSED_UPDATE");
    const DevStep* cur = c->d_step + c->cur;
    DevStep* nxt = c->d_step + (c->cur ^ 1);
    const HostOut ho = next_host_out(c, flags);
    // one workgroup, one thread per merged column (2T + 1 <= 256 up to T = 127)
    if (2 * c->cfg.T + 1 <= 256)
        hipLaunchKernelGGL(merge_kernel<256>, dim3(1), dim3(256), 0, c->stream, c->kc, partials_dev, n, c->d_weps,
                           cur, nxt, flags, reinterpret_cast<float*>(c->d_upd), ho);
    else
        hipLaunchKernelGGL(merge_kernel<512>, dim3(1), dim3(512), 0, c->stream, c->kc, partials_dev, n, c->d_weps,
                           cur, nxt, flags, reinterpret_cast<float*>(c->d_upd), ho);
    const int rc = launch_check("merge_kernel");
    if (rc == MPPI_OK && (flags & MPPI_FLAG_FUSED_UPDATE)) {
        c->cur ^= 1;
        c->upd_valid = true;
        c->nominal_published = false;   // until wait_host_out sees this launch's outputs
    }
    return rc;
}

int mppi_get_weighted_noise(mppi_ctx* c, double* w_eps_host) {
    if (!c || !w_eps_host) return fail(MPPI_E_ARG, "null argument");
    const size_t bytes = 2 * (size_t)c->cfg.T * sizeof(double);
    HIP_TRY(hipMemcpyAsync(c->h_buf, c->d_weps, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    memcpy(w_eps_host, c->h_buf, bytes);
    return check_timeout(c);
}

int mppi_get_nominal(mppi_ctx* c, double* u_host) {
    if (!c || !u_host) return fail(MPPI_E_ARG, "null argument");
    const size_t bytes = 2 * (size_t)c->cfg.T * sizeof(double);
    HIP_TRY(hipMemcpyAsync(c->h_buf, (const char*)(c->d_step + c->cur) + offsetof(DevStep, u), bytes,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    memcpy(u_host, c->h_buf, bytes);
    return MPPI_OK;
}

int mppi_rollout_traj(mppi_ctx* c, const double* base_u, const float* noise_dev, int K, float* out_dev) {
    if (!c || !out_dev || K < 1 || K > c->cfg.K_local) return fail(MPPI_E_ARG, "bad argument");
    const DevStep* cur = c->d_step + c->cur;
    const float2* base;
    int bstride = 1;
    if (base_u) {
        HIP_TRY(hipEventSynchronize(c->staged));
        for (int t = 0; t < c->cfg.T; ++t) c->h_base[t] = make_float2((float)base_u[2 * t], (float)base_u[2 * t + 1]);
        HIP_TRY(hipMemcpyAsync(c->d_base, c->h_base, c->cfg.T * sizeof(float2), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->staged, c->stream));
        base = c->d_base;
    } else {
        // the current nominal in place: ua[t].xy, every other float2 (stream order
        // keeps the next launch's write of this block behind the re-roll)
        base = reinterpret_cast<const float2*>(reinterpret_cast<const char*>(cur) + offsetof(DevStep, ua));
        bstride = 2;
    }
    const int blocks = (K + kThreads - 1) / kThreads;
    if (noise_dev)
        hipLaunchKernelGGL(traj_kernel<true>, dim3(blocks), dim3(kThreads), 0, c->stream, c->kc, c->stat, base, bstride,
                           reinterpret_cast<const float2*>(noise_dev), K, reinterpret_cast<float4*>(out_dev));
    else
        hipLaunchKernelGGL(traj_kernel<false>, dim3(blocks), dim3(kThreads), 0, c->stream, c->kc, c->stat, base,
                           bstride, (const float2*)nullptr, K, reinterpret_cast<float4*>(out_dev));
    return launch_check("traj_kernel");
}

int mppi_optimal_traj(mppi_ctx* c, float* out_dev) {
    if (!c || !out_dev) return fail(MPPI_E_ARG, "null argument");
    if (!c->upd_valid) return fail(MPPI_E_ARG, "mppi_optimal_traj needs a preceding MPPI_FLAG_FUSED_UPDATE launch");
    hipLaunchKernelGGL(traj_kernel<false>, dim3(1), dim3(kThreads), 0, c->stream, c->kc, c->stat, c->d_upd, 1,
                       (const float2*)nullptr, 1, reinterpret_cast<float4*>(out_dev));
    return launch_check("traj_kernel");
}

int mppi_get_step_outputs(mppi_ctx* c, double* u_host, const float* traj_dev, float* traj_host) {
    if (!c || !u_host || (traj_dev && !traj_host)) return fail(MPPI_E_ARG, "bad argument");
    const int T = c->cfg.T;
    const size_t ub = 2 * (size_t)T * sizeof(double), tb = 4 * (size_t)T * sizeof(float);
    float* h_traj = reinterpret_cast<float*>(c->h_out + 2 * kMaxT);
    HIP_TRY(hipMemcpyAsync(c->h_out, (const char*)(c->d_step + c->cur) + offsetof(DevStep, u), ub,
                           hipMemcpyDeviceToHost, c->stream));
    if (traj_dev) HIP_TRY(hipMemcpyAsync(h_traj, traj_dev, tb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    memcpy(u_host, c->h_out, ub);
    if (traj_dev) memcpy(traj_host, h_traj, tb);
    return check_timeout(c);
}

int mppi_optimal_traj_host(const mppi_ctx* c, const double* x0, const double* u_new, double* traj_out) {
    if (!c || !x0 || !u_new || !traj_out) return fail(MPPI_E_ARG, "null argument");
    // control.py:129-134: x_{t+1} = _F(x_t, u_new[t - 1]), u_new[-1] = u_new[T - 1]
    const int T = c->cfg.T;
    double x[4] = {x0[0], x0[1], x0[2], x0[3]};
    for (int t = 0; t < T; ++t) {
        const double* ut = u_new + 2 * (t == 0 ? T - 1 : t - 1);
        host_F(c->cfg.arm, c->cfg.delta_t, x, ut[0], ut[1]);
        memcpy(traj_out + 4 * t, x, sizeof(x));
    }
    return MPPI_OK;
}

int mppi_wait_outputs(mppi_ctx* c, const double* x0, double* u_out, double* traj_out) {
    if (!c || !u_out || (traj_out && !x0)) return fail(MPPI_E_ARG, "bad argument");
    if (int rc = wait_host_out(c)) return rc;
    const int T = c->cfg.T;
    memcpy(u_out, c->h_dout + 4, 2 * (size_t)T * sizeof(double));
    if (traj_out) {
        // u_new[0] from the flag block, u_new[t] = shifted[t - 1] for t >= 1
        double un[2 * kMaxT];
        un[0] = c->h_dout[2];
        un[1] = c->h_dout[3];
        memcpy(un + 2, c->h_dout + 4, 2 * (size_t)(T - 1) * sizeof(double));
        return mppi_optimal_traj_host(c, x0, un, traj_out);
    }
    return MPPI_OK;
}

}  // extern "C"

namespace {
// The launch half of mppi_step_dropin: stage, fused launch, next noise queued.
int dropin_launch(mppi_ctx* c, const double* x0, const double* window, int W, const double* u, const float* noise_dev,
                  double* S_dev, float* next_noise_dev, unsigned long long seed, unsigned long long next_step) {
    if (!c || !x0 || !window || !noise_dev) return fail(MPPI_E_ARG, "null argument");
    if (c->cfg.T < 5) return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    using clk = std::chrono::steady_clock;
    const auto t0 = c->in_tick ? c->tick_t0 : clk::now();   // a tick's phases include its waypoint update
    c->in_tick = false;
    c->step_t0 = t0;
    auto mark = [&](int i) { c->dropin_us[i] = std::chrono::duration<double, std::micro>(clk::now() - t0).count(); };
    if (int rc = stage_inputs(c, x0, window, W, u, true)) return rc;
    mark(0);
    // with an exchange attached the launch also trades rows with the other ranks
    const unsigned fl = MPPI_FLAG_FUSED_UPDATE | MPPI_FLAG_HOST_OUT | (c->xd.world >= 1 ? MPPI_FLAG_EXCHANGE : 0u);
    if (int rc = launch_rollout(c, noise_dev, S_dev, nullptr, fl, next_host_out(c, fl))) return rc;
    mark(1);
    // the next step's noise, queued behind this step's rollout (stream order: the
    // draw starts after the rollout has read the buffer); issuing it now hides the
    // launch call under the rollout, and the draw overlaps the host's remaining work
    if (next_noise_dev)
        if (int rc = mppi_noise_philox(c, seed, next_step, next_noise_dev)) return rc;
    mark(2);
    return MPPI_OK;
}

// The wait half: the launch's published outputs, then the host trajectory.
int dropin_finish(mppi_ctx* c, const double* x0, double* u_out, double* traj_out) {
    if (!u_out) return fail(MPPI_E_ARG, "null argument");
    using clk = std::chrono::steady_clock;
    auto mark = [&](int i) {
        c->dropin_us[i] = std::chrono::duration<double, std::micro>(clk::now() - c->step_t0).count();
    };
    if (int rc = wait_host_out(c)) return rc;
    mark(3);
    if (int rc = mppi_wait_outputs(c, x0, u_out, traj_out)) return rc;   // already published: copies + trajectory
    mark(4);
    return MPPI_OK;
}
}  // namespace

extern "C" {

int mppi_step_dropin(mppi_ctx* c, const double* x0, const double* window, int W, const double* u,
                     const float* noise_dev, double* S_dev, float* next_noise_dev, unsigned long long seed,
                     unsigned long long next_step, double* u_out, double* traj_out) {
    if (!u_out) return fail(MPPI_E_ARG, "null argument");
    if (int rc = dropin_launch(c, x0, window, W, u, noise_dev, S_dev, next_noise_dev, seed, next_step)) return rc;
    return dropin_finish(c, x0, u_out, traj_out);
}

int mppi_dropin_bind(mppi_ctx* c, const mppi_dropin_binding* b) {
    if (!c || !b) return fail(MPPI_E_ARG, "null argument");
    if (!b->path || b->rows < 1 || b->stride < 4 || !b->x0 || !b->idx || !b->u || !b->noise_dev)
        return fail(MPPI_E_ARG, "binding: path (rows >= 1, stride >= 4), x0, idx, u and noise_dev are required");
    c->bind = *b;
    c->bound = true;
    return MPPI_OK;
}

int mppi_dropin_tick(mppi_ctx* c, unsigned long long next_step) {
    if (int rc = mppi_dropin_tick_launch(c, next_step)) return rc;
    return mppi_dropin_tick_wait(c);
}

int mppi_dropin_tick_wait(mppi_ctx* c) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    if (!c->tick_launched) return fail(MPPI_E_ARG, "mppi_dropin_tick_wait without a launched tick");
    c->tick_launched = false;
    return dropin_finish(c, c->bind.x0, c->bind.u, c->bind.traj);
}

int mppi_dropin_tick_launch(mppi_ctx* c, unsigned long long next_step) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    if (!c->bound) return fail(MPPI_E_ARG, "mppi_dropin_tick before mppi_dropin_bind");
    if (c->tick_launched) return fail(MPPI_E_ARG, "a launched tick was not waited for (mppi_dropin_tick_wait)");
    const mppi_dropin_binding& b = c->bind;
    c->tick_t0 = std::chrono::steady_clock::now();
    c->in_tick = true;
    // _get_nearest_waypoint(x0[0], x0[1], update_prev_idx=True), control.py:200-232, in the
    // reference's fp64 operations (NumPy's float64 cos/sin are the C library's)
    const double q1 = b.x0[0], q2 = b.x0[1];
    const double x = b.fk_l1 * cos(q1) + b.fk_l2 * cos(q1 + q2);
    const double y = b.fk_l1 * sin(q1) + b.fk_l2 * sin(q1 + q2);
    const long long prev = b.idx[0];
    if (prev < 0 || prev >= b.rows) {
        c->in_tick = false;
        return fail(MPPI_E_ARG, "prev_waypoints_idx outside ref_path");
    }
    const int n = (int)std::min<long long>(MPPI_SEARCH_LEN, b.rows - prev);
    int best = 0;
    double dmin = 0.0;
    for (int j = 0; j < n; ++j) {   // min(d) then d.index(min_d) (control.py:213-215): d[0], replaced on a strict '<'
        const double* r = b.path + (prev + j) * (long long)b.stride;
        const double dx = x - r[0], dy = y - r[1];
        const double d = (dx * dx + dy * dy) * 100;
        if (j == 0 || d < dmin) {
            dmin = d;
            best = j;
        }
    }
    const long long idx = prev + best;
    b.idx[1] = prev;
    b.idx[0] = idx;
    if (idx >= b.rows - 1) {
        c->in_tick = false;
        return fail(MPPI_E_PATH_END, "Reached the end of the reference path.");
    }
    // the window ref_path[idx : idx + 30, 0:4] (control.py:203-204, slice-truncated)
    const int W = (int)std::min<long long>(MPPI_SEARCH_LEN, b.rows - idx);
    double win[4 * MPPI_SEARCH_LEN];
    for (int j = 0; j < W; ++j) memcpy(win + 4 * j, b.path + (idx + j) * (long long)b.stride, 4 * sizeof(double));
    const int rc = dropin_launch(c, b.x0, win, W, b.u, b.noise_dev, b.S_dev, b.next_noise_dev, b.seed, next_step);
    c->tick_launched = rc == MPPI_OK;
    return rc;
}

int mppi_noise_philox(mppi_ctx* c, unsigned long long seed, unsigned long long step, float* out_dev) {
    if (!c || !out_dev) return fail(MPPI_E_ARG, "null argument");
    const double* S = c->cfg.sigma;
    // Cholesky of the symmetric part (np.random.multivariate_normal expects SPD Sigma)
    const double s01 = 0.5 * (S[1] + S[2]);
    if (!(S[0] > 0.0)) return fail(MPPI_E_ARG, "Sigma not positive definite");
    const double L00 = sqrt(S[0]), L10 = s01 / L00, d = S[3] - L10 * L10;
    if (!(d >= 0.0)) return fail(MPPI_E_ARG, "Sigma not positive semi-definite");
    const double L11 = sqrt(d);
    constexpr double bm = kBoxMullerScale;   // box_muller's constant, folded into L
    const dim3 grid((unsigned)((c->cfg.K_local + kThreads - 1) / kThreads), (unsigned)((c->cfg.T + 1) / 2));
    hipLaunchKernelGGL(philox_noise_kernel, grid, dim3(kThreads), 0, c->stream, c->cfg.K_local,
                       c->cfg.T, (long long)c->cfg.k_offset, seed, step, (float)(L00 * bm), (float)(L10 * bm), (float)(L11 * bm),
                       reinterpret_cast<float2*>(out_dev));
    return launch_check("philox_noise_kernel");
}

int mppi_debug_set_buffer(mppi_ctx* c, void* dbg_dev) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    c->d_dbg = (unsigned long long*)dbg_dev;
    return MPPI_OK;
}

int mppi_debug_nearest(mppi_ctx* c, const float* noise_dev, int K, int* slot_dev, float* pos_dev) {
    if (!c || !noise_dev || !slot_dev || !pos_dev || K < 1 || K > c->cfg.K_local) return fail(MPPI_E_ARG, "bad argument");
    hipLaunchKernelGGL(nearest_debug_kernel, dim3((K + kThreads - 1) / kThreads), dim3(kThreads), 0, c->stream, c->kc,
                       c->stat, c->d_step + c->cur, reinterpret_cast<const float2*>(noise_dev), K, slot_dev,
                       reinterpret_cast<float2*>(pos_dev));
    return launch_check("nearest_debug_kernel");
}

int mppi_debug_dropin_times(const mppi_ctx* c, double* us_out) {
    if (!c || !us_out) return fail(MPPI_E_ARG, "null argument");
    memcpy(us_out, c->dropin_us, 5 * sizeof(double));
    return MPPI_OK;
}

int mppi_sync(mppi_ctx* c) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return check_timeout(c);
}

int mppi_ctx_handoff(const mppi_ctx* c, int* poll) {
    if (!c || !poll) return fail(MPPI_E_ARG, "null argument");
    *poll = c->poll ? 1 : 0;
    return MPPI_OK;
}

}  // extern "C"
