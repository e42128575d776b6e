// mppi_rocm.hip — MI355X (gfx950, CDNA4) MPPI rollout-and-reduce engine.
//
// The hot path of junofficial/mppi_RobotArm control.py:81-118 (K samples x T
// steps of: Gaussian control perturbation -> 2-link arm forward dynamics
// (_F, control.py:234-263) -> windowed nearest-waypoint stage cost (_c /
// _get_nearest_waypoint, control.py:174-232) + control cost (control.py:106)
// -> terminal cost (control.py:109) -> soft-min weights (control.py:297-314)
// -> weighted noise sum (control.py:115-118)), written for CDNA4 directly:
//
//  * rollout_kernel<LPS>: LPS lanes of a 64-wide wave per sample (1, 2 or 4).
//    The serial T loop runs per lane in fp32 registers; the 30-waypoint
//    argmin is split over the LPS lanes of a sample and closed with DPP
//    quad_perm min (no LDS, no MFMA: the work is element-wise VALU).  The
//    per-step noise row eps[t][k][:] is one coalesced 8-B-per-lane load,
//    prefetched two steps ahead.  S accumulates in fp64.
//  * the block epilogue turns its samples into a log-sum-exp partial
//    {rho_b, eta_b, N_b[T][2]} (only samples with non-zero weight are
//    visited), publishes it with an agent-scope release + arrival counter,
//    and the last-arriving workgroup merges every partial (agent acquire),
//    so one launch covers control.py:81-118.  With MPPI_FLAG_FUSED_UPDATE
//    that workgroup also applies the median filter / update / shift of
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

#include <string>
#include <type_traits>

#include "mppi_rocm.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxT = MPPI_MAX_T;
constexpr int kSlots = 32;  // window slots (>= MPPI_SEARCH_LEN), index fits 5 bits
constexpr float kPadKey = 1.0e30f;

// Device-resident per-step parameter block (ping-pong pair in the context).
struct alignas(16) DevStep {
    float4 win[kSlots];   // rx, ry, rdq1, rdq2 of window slot j (lookup after argmin)
    float4 key[kSlots];   // rx', ry', c' = rx'^2 + ry'^2 (centred), 0; pads c' = 1e30
    float4 x0;            // q1, q2, dq1, dq2
    float4 ctr;           // window centre (cx, cy), W, unused
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

// ------------------------------------------------------------------ helpers

// Hardware v_sin_f32 / v_cos_f32 (argument pre-scaled by 1/(2 pi)): 30 % faster
// rollouts than OCML's sincosf at K=65536 T=64, parity unchanged (S rel-err
// budget 5e-5 in tests/test_gpu_parity.py).  -DMPPI_ACCURATE_TRIG selects sincosf.
__device__ __forceinline__ void sincos_f32(float x, float* s, float* c) {
#ifdef MPPI_ACCURATE_TRIG
    sincosf(x, s, c);
#else
    __sincosf(x, s, c);
#endif
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ int lanes_below(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// v from lane l as a wave-uniform (scalar) value
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ float readlane_f32(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Whole-wave reductions (all 64 lanes active), result wave-uniform: DPP
// quad_perm xor 1 / xor 2, row_half_mirror, row_mirror reduce each row of 16
// in registers, then the four row results are combined from v_readlane — no
// LDS round trips (a ds_bpermute butterfly costs six of them).  The combine
// order is fixed, so sums are deterministic.
template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
    if constexpr (sizeof(T) == 8) {
        v = op(v, dpp_f64<0xB1>(v));
        v = op(v, dpp_f64<0x4E>(v));
        v = op(v, dpp_f64<0x141>(v));
        v = op(v, dpp_f64<0x140>(v));
        return op(op(readlane_f64(v, 0), readlane_f64(v, 16)), op(readlane_f64(v, 32), readlane_f64(v, 48)));
    } else {
        v = op(v, dpp_f32<0xB1>(v));
        v = op(v, dpp_f32<0x4E>(v));
        v = op(v, dpp_f32<0x141>(v));
        v = op(v, dpp_f32<0x140>(v));
        return op(op(readlane_f32(v, 0), readlane_f32(v, 16)), op(readlane_f32(v, 32), readlane_f32(v, 48)));
    }
}
struct OpMin { __device__ double operator()(double a, double b) const { return fmin(a, b); } };
struct OpAdd {
    template <class T> __device__ T operator()(T a, T b) const { return a + b; }
};
__device__ __forceinline__ double wave_min_f64(double v) { return wave_reduce(v, OpMin{}); }
__device__ __forceinline__ double wave_sum_f64(double v) { return wave_reduce(v, OpAdd{}); }
__device__ __forceinline__ float wave_sum_f32(float v) { return wave_reduce(v, OpAdd{}); }

// One semi-implicit Euler step of _F (control.py:234-263) in closed form:
//   M = [[A + B c2, D + E c2], [D + E c2, D]]   (M22 = m2 lc2^2 + l2 = D)
//   h = E s2,  G = [P c1 + Q c12, Q c12],  C dq = [-h dq2 (2 dq1 + dq2), h dq1^2]
//   ddq = M^-1 (v - C dq - G);  dq += ddq dt;  q += dq dt
// c2/s2 come from the angle-difference identities of the cached sincos of
// q1 and q1 + q2, so each step evaluates exactly two sincos (of the NEW q),
// which the next step's dynamics and this step's kinematics share.
struct ArmState {
    float q1, q2, dq1, dq2;
    float s1, c1, s12, c12;
};

__device__ __forceinline__ void dyn_step(ArmState& x, float v1, float v2, const KConst& c) {
    const float c2 = fmaf(x.c12, x.c1, x.s12 * x.s1);
    const float s2 = fmaf(x.s12, x.c1, -x.c12 * x.s1);
    const float M11 = fmaf(c.B, c2, c.A);
    const float M12 = fmaf(c.E, c2, c.D);
    const float h = c.E * s2;
    const float G2 = c.Q * x.c12;
    const float G1 = fmaf(c.P, x.c1, G2);
    const float r1 = fmaf(h * x.dq2, fmaf(2.f, x.dq1, x.dq2), v1 - G1);
    const float r2 = fmaf(-h * x.dq1, x.dq1, v2 - G2);
    const float det = fmaf(M11, c.D, -M12 * M12);
    const float rdet = __builtin_amdgcn_rcpf(det);
    const float ddq1 = fmaf(c.D, r1, -M12 * r2) * rdet;
    const float ddq2 = fmaf(M11, r2, -M12 * r1) * rdet;
    x.dq1 = fmaf(ddq1, c.dt, x.dq1);
    x.dq2 = fmaf(ddq2, c.dt, x.dq2);
    x.q1 = fmaf(x.dq1, c.dt, x.q1);
    x.q2 = fmaf(x.dq2, c.dt, x.q2);
    sincos_f32(x.q1, &x.s1, &x.c1);
    sincos_f32(x.q1 + x.q2, &x.s12, &x.c12);
}

// --------------------------------------------------- merge + update helpers

constexpr int kMaxWaves = 16;       // up to 1024-thread workgroups
constexpr int kGroup = 16;          // workgroups per first-level merge group
// A partial whose rescale factor s = exp((rho - rho_i) / lambda) is below 2^-64
// changes eta and N by less than 2^-64 * 512 relative to the leading term
// (which has s = 1 and eta >= 1): far below the fp64 resolution of the result.
constexpr double kMergeFloor = 5.421010862427522e-20;  // 2^-64

// Rows {rho, eta, N[2T]} handed between workgroups of one launch travel
// write-through: every store and every load of them is a `sc1` buffer access
// (MI355X guide G16, "Valid forms" row 1), so neither side needs an
// agent-scope fence (~1.7 us each) — only each storing wave's vmcnt drain, a
// workgroup barrier and one relaxed agent atomic per workgroup.
typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
constexpr int kSC1 = 16;  // buffer aux bit: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const double* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double ld_wt(__amdgpu_buffer_rsrc_t r, int idx) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, kSC1));
}
// Element index past every rows buffer: a raw buffer load beyond num_records
// returns 0 without a memory access, so a predicated-off load needs no branch
// (a branch around each load makes the compiler wait for it at the join).
constexpr int kOffRange = 1 << 27;   // x 8 B = 1 GiB > any rows buffer, no int overflow

// Tagged granules (MI355X guide, Guideline 16 R2: "the data IS the flag").  One
// fp64 value travels as {lo32, tag, hi32, tag} in ONE 16-B sc1 store; each 8-B
// half is a naturally aligned {value, tag} granule, so a reader that sees both
// tags equal to this launch's epoch holds the whole value — no drain, no flag,
// no counter.  Tags come from a device-resident epoch (never a kernel argument:
// graph replay freezes those), zeroed once at context creation.
typedef unsigned int u32x4 __attribute__((__vector_size__(4 * sizeof(unsigned int))));
__device__ __forceinline__ void st_gran(__amdgpu_buffer_rsrc_t r, int idx, double v, unsigned tag) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const u32x4 x = {(unsigned)b, tag, (unsigned)(b >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, idx * 16, 0, kSC1);
}
// Poll loads are plain sc1 loads; every spin loop opens with an empty asm
// memory clobber so the loads are re-issued each pass (without it LLVM hoists
// the read-only loads out of the loop — nothing else in it writes memory — and
// polls registers).
__device__ __forceinline__ u32x4 ld_gran(__amdgpu_buffer_rsrc_t r, int idx) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, idx * 16, 0, kSC1);
}
__device__ __forceinline__ bool gran_ok(u32x4 x, unsigned tag) { return x[1] == tag && x[3] == tag; }
__device__ __forceinline__ double gran_val(u32x4 x) {
    return __longlong_as_double((long long)(((unsigned long long)x[2] << 32) | x[0]));
}
// Bounded spins: ~1 s of polling, then the hand-off reports a timeout (host
// error word) instead of hanging the GPU; results of that launch are invalid.
constexpr unsigned kSpinMax = 1u << 20;
__device__ __forceinline__ void report_timeout(unsigned* tmo) {
    if (tmo) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double poll_gran(__amdgpu_buffer_rsrc_t r, int idx, unsigned tag, unsigned* tmo) {
    for (unsigned spins = 0;; ++spins) {
        asm volatile("" ::: "memory");
        const u32x4 x = ld_gran(r, idx);
        if (gran_ok(x, tag)) return gran_val(x);
        if (spins >= kSpinMax) {
            report_timeout(tmo);
            return gran_val(x);
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, int idx, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, idx * 8, 0, kSC1);
}

constexpr int kMergeRows = 32;   // rows per load round in a merge (<= 64: one row per lane)

struct MergeScratch {
    double red[kMaxWaves];
    double weps[2 * kMaxT];
    double unew[2 * kMaxT];
    int nrel;
};

// Workgroup minimum.  One use per kernel: the caller's next barrier protects
// sm.red before any reuse.
template <int NT>
__device__ __forceinline__ double block_min_f64(double v, MergeScratch& sm) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_min_f64(v);
    if (lane == 0) sm.red[wave] = v;
    __syncthreads();
    double r = sm.red[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) r = fmin(r, sm.red[w]);
    return r;
}

// Merge n rows {rho, eta, N[2T]} (row stride 2 + 2T, read write-through from
// `rows`) with a log-sum-exp rescale, rho = min rho_i, s_i = exp((rho - rho_i)
// / lambda), eta = sum s_i eta_i, N = sum s_i N_i, in ascending row order
// (deterministic).  Rows are consumed kMergeRows at a time, every load of a
// round issued together (one memory round trip per round) with an online
// rescale of the running sums when a round lowers rho; rows whose factor is
// below 2^-64 of the running best are skipped (below fp64 resolution).
// Wave-local: every wave loads the round's rho_i / eta_i into its lanes,
// reduces rho with DPP and evaluates s_i, eta itself; s_i reach the column
// FMAs as scalars (v_readlane) — no LDS traffic and no barrier per round.
// Thread tid owns column tid (col 0 = eta, 1 + j = N[j]) and tid + NT.
// The merged row goes to out_wt (write-through, next level) and/or out_row
// (plain, read after the launch); with `final`, w_eps = N / eta
// (control.py:112-118) goes to sm.weps and w_eps_out.
//
// GRAN: rows are tagged granules (16 B per value) published without any drain
// or counter; every wave re-reads its round's loads until every tag matches
// `tag` (kGranRows rows per round: 16 B per load in flight), and out_wt is
// written as granules too.  Otherwise rows are 8-B sc1 words behind an
// arrival counter (arrive_last).
constexpr int kGranRows = 16;

// Final merged row: {rho, eta, N} to out_row (plain, read after the launch) and
// w_eps = N / eta (control.py:112-118) to sm.weps and w_eps_out.  Thread tid
// holds column tid (col 0 = eta) and tid + NT.
template <int NT>
__device__ __forceinline__ void put_final(double rho, double acc0, double acc1, double eta, int nrel, bool has0,
                                          bool has1, MergeScratch& sm, double* out_row, double* w_eps_out) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        sm.nrel = nrel;
        if (out_row) {
            out_row[0] = rho;
            out_row[1] = acc0;
        }
    } else if (has0) {
        if (out_row) out_row[1 + tid] = acc0;
        const double w = acc0 / eta;
        sm.weps[tid - 1] = w;
        if (w_eps_out) w_eps_out[tid - 1] = w;
    }
    if (has1) {
        if (out_row) out_row[1 + tid + NT] = acc1;
        const double w = acc1 / eta;
        sm.weps[tid + NT - 1] = w;
        if (w_eps_out) w_eps_out[tid + NT - 1] = w;
    }
    __syncthreads();
}

template <int NT, bool final, bool GRAN>
__device__ __forceinline__ void merge_rows_block(__amdgpu_buffer_rsrc_t rows, int row0, int n, const KConst& c,
                                                 MergeScratch& sm, const __amdgpu_buffer_rsrc_t* out_wt, int out_idx,
                                                 double* out_row, double* w_eps_out, unsigned tag, unsigned* tmo) {
    constexpr int R = GRAN ? kGranRows : kMergeRows;
    static_assert(R <= 64, "one row per lane");
    const int tid = threadIdx.x, lane = tid & 63;
    const int stride = 2 + 2 * c.T;
    const int ncol = 2 * c.T + 1;
    const bool has0 = tid < ncol, has1 = tid + NT < ncol;
    double acc0 = 0.0, acc1 = 0.0, eta = 0.0, rho = INFINITY;
    int nrel = 0;
    for (int r0 = 0; r0 < n; r0 += R) {
        const int nr = min(R, n - r0);   // uniform
        const int rb = row0 + r0;
        const int lrow = lane < nr ? (rb + lane) * stride : kOffRange;
        double rho_r, eta_l, v[R];
        if constexpr (GRAN) {
            // phase 1: poll only the rho granules, one lane per row (a pass
            // moves 16 B per row, so a row that lands is seen within ~one
            // short round trip; the bulk of the row is fetched once, below)
            u32x4 gr;
            for (unsigned spins = 0;; ++spins) {
                asm volatile("" ::: "memory");
                gr = ld_gran(rows, lrow);
                if (__all(lane >= nr || gran_ok(gr, tag))) break;
                if (spins >= kSpinMax) {
                    if (lane == 0) report_timeout(tmo);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            rho_r = gran_val(gr);
        } else {
            rho_r = ld_wt(rows, lrow);
            eta_l = ld_wt(rows, lrow + 1);
#pragma unroll
            for (int i = 0; i < R; ++i) v[i] = ld_wt(rows, (i < nr && has0) ? (rb + i) * stride + 1 + tid : kOffRange);
        }
        const double rho_l = lane < nr ? rho_r : INFINITY;
        const double rnew = fmin(rho, wave_min_f64(rho_l));
        double s_l = 0.0;
        if (lane < nr) {
            const double s = exp((rnew - rho_l) * c.inv_lambda);
            s_l = s >= kMergeFloor ? s : 0.0;
        }
        const unsigned long long rel = __ballot(s_l != 0.0);   // rows that carry weight (uniform)
        nrel += __popcll(rel);
        if constexpr (GRAN) {
            // phase 2: eta and the columns of the weighted rows only (usually one
            // or two at run.py's lambda), re-read until every tag matches
            u32x4 ge, gv[R];
            for (unsigned spins = 0;; ++spins) {
                asm volatile("" ::: "memory");
                ge = ld_gran(rows, ((rel >> lane) & 1) ? lrow + 1 : kOffRange);
#pragma unroll
                for (int i = 0; i < R; ++i)
                    gv[i] = ld_gran(rows, (((rel >> i) & 1) && has0) ? (rb + i) * stride + 1 + tid : kOffRange);
                bool ok = !((rel >> lane) & 1) || gran_ok(ge, tag);
#pragma unroll
                for (int i = 0; i < R; ++i) ok = ok && (!(((rel >> i) & 1) && has0) || gran_ok(gv[i], tag));
                if (__all(ok)) break;
                if (spins >= kSpinMax) {
                    if (lane == 0) report_timeout(tmo);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            eta_l = gran_val(ge);
#pragma unroll
            for (int i = 0; i < R; ++i) v[i] = gran_val(gv[i]);
        }
        if (rnew < rho && rho != INFINITY) {  // uniform: rescale the running sums to the new minimum
            const double f = exp((rnew - rho) * c.inv_lambda);
            acc0 *= f;
            acc1 *= f;
            eta *= f;
        }
        rho = rnew;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if (i < nr) {
                const double s = readlane_f64(s_l, i);
                if (s != 0.0) {
                    acc0 = fma(s, v[i], acc0);
                    eta = fma(s, readlane_f64(eta_l, i), eta);
                }
            }
        }
        if (ncol > NT) {  // second column pass (T = 128 only: 2T + 1 = 257 columns)
            for (int i = 0; i < nr; ++i) {
                const double s = readlane_f64(s_l, i);
                if (s != 0.0 && has1) {
                    const int idx = (rb + i) * stride + 1 + tid + NT;
                    acc1 = fma(s, GRAN ? poll_gran(rows, idx, tag, tmo) : ld_wt(rows, idx), acc1);
                }
            }
        }
    }
    if constexpr (final) {
        put_final<NT>(rho, acc0, acc1, eta, nrel, has0, has1, sm, out_row, w_eps_out);
    } else {
        auto put = [&](int col, double v) {  // col 0 = rho, 1 = eta, 2 + j = N[j]
            if constexpr (GRAN) st_gran(*out_wt, out_idx * stride + col, v, tag);
            else st_wt(*out_wt, out_idx * stride + col, v);
        };
        if (tid == 0) {
            put(0, rho);
            put(1, acc0);
        } else if (has0) {
            put(1 + tid, acc0);
        }
        if (has1) put(1 + tid + NT, acc1);
    }
}

// The k-th (0-based) set bit of m; k < popcount(m).
__device__ __forceinline__ int select_bit(unsigned long long m, int k) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        const int cnt = __popcll(m & ((1ull << w) - 1));
        if (k >= cnt) {
            k -= cnt;
            m >>= w;
            pos += w;
        }
    }
    return pos;
}

constexpr int kDirectRows = 256;  // workgroup rows the direct merge scans (4 per lane)
constexpr int kDirectMax = 16;    // weighted rows it merges; more go through the group rows

// Single-level finish for the usual regime (few weighted rows, S spread >> lambda):
// read rho of EVERY workgroup row (n <= kDirectRows), and when at most
// kDirectMax rows carry weight relative to the global minimum, merge exactly
// those rows in ascending order straight from the workgroup slab — one hand-off
// on the critical path instead of two.  Returns false (uniformly) when more rows
// carry weight; the caller then merges through the group rows.  Wave-local
// like merge_rows_block; the result goes out as in a final merge.
template <int NT, bool GRAN>
__device__ __forceinline__ bool direct_merge(__amdgpu_buffer_rsrc_t rows, int n, const KConst& c, MergeScratch& sm,
                                             double* out_row, double* w_eps_out, unsigned tag, unsigned* tmo) {
    constexpr int P = kDirectRows / 64;
    const int tid = threadIdx.x, lane = tid & 63;
    const int stride = 2 + 2 * c.T;
    const int ncol = 2 * c.T + 1;
    const bool has0 = tid < ncol, has1 = tid + NT < ncol;
    // phase 1: rho of row lane + 64 j in slot j
    double rho_l[P];
    if constexpr (GRAN) {
        u32x4 gr[P];
        for (unsigned spins = 0;; ++spins) {
            asm volatile("" ::: "memory");
            bool ok = true;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int r = lane + 64 * j;
                gr[j] = ld_gran(rows, r < n ? r * stride : kOffRange);
                ok = ok && (r >= n || gran_ok(gr[j], tag));
            }
            if (__all(ok)) break;
            if (spins >= kSpinMax) {
                if (lane == 0) report_timeout(tmo);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int j = 0; j < P; ++j) rho_l[j] = lane + 64 * j < n ? gran_val(gr[j]) : INFINITY;
    } else {
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int r = lane + 64 * j;
            const double x = ld_wt(rows, r < n ? r * stride : kOffRange);
            rho_l[j] = r < n ? x : INFINITY;
        }
    }
    double m = rho_l[0];
#pragma unroll
    for (int j = 1; j < P; ++j) m = fmin(m, rho_l[j]);
    const double rho = wave_min_f64(m);
    double s_l[P];
    unsigned long long rel[P];
    int nrel = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const double s = exp((rho - rho_l[j]) * c.inv_lambda);
        s_l[j] = (lane + 64 * j < n && s >= kMergeFloor) ? s : 0.0;
        rel[j] = __ballot(s_l[j] != 0.0);
        nrel += __popcll(rel[j]);
    }
    if (nrel > kDirectMax) return false;
    // lane k < nrel: the k-th weighted row (ascending) and its factor
    int k = lane, row = 0;
    bool found = false;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int cnt = __popcll(rel[j]);
        if (!found && k < cnt) {
            row = 64 * j + select_bit(rel[j], k);
            found = true;
        } else if (!found) {
            k -= cnt;
        }
    }
    double sk = 0.0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const double sj = __shfl(s_l[j], row & 63);
        if ((row >> 6) == j) sk = sj;
    }
    const bool mine = lane < nrel;
    // phase 2: eta and the columns of the weighted rows
    double eta_k, v[kDirectMax];
    if constexpr (GRAN) {
        u32x4 ge, gv[kDirectMax];
        for (unsigned spins = 0;; ++spins) {
            asm volatile("" ::: "memory");
            ge = ld_gran(rows, mine ? row * stride + 1 : kOffRange);
#pragma unroll
            for (int i = 0; i < kDirectMax; ++i)
                gv[i] = ld_gran(rows, (i < nrel && has0) ? __builtin_amdgcn_readlane(row, i) * stride + 1 + tid
                                                         : kOffRange);
            bool ok = !mine || gran_ok(ge, tag);
#pragma unroll
            for (int i = 0; i < kDirectMax; ++i) ok = ok && (!(i < nrel && has0) || gran_ok(gv[i], tag));
            if (__all(ok)) break;
            if (spins >= kSpinMax) {
                if (lane == 0) report_timeout(tmo);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        eta_k = gran_val(ge);
#pragma unroll
        for (int i = 0; i < kDirectMax; ++i) v[i] = gran_val(gv[i]);
    } else {
        eta_k = ld_wt(rows, mine ? row * stride + 1 : kOffRange);
#pragma unroll
        for (int i = 0; i < kDirectMax; ++i)
            v[i] = ld_wt(rows, (i < nrel && has0) ? __builtin_amdgcn_readlane(row, i) * stride + 1 + tid : kOffRange);
    }
    double acc0 = 0.0, acc1 = 0.0, eta = 0.0;
#pragma unroll
    for (int i = 0; i < kDirectMax; ++i) {
        if (i < nrel) {
            const double s = readlane_f64(sk, i);
            acc0 = fma(s, v[i], acc0);
            eta = fma(s, readlane_f64(eta_k, i), eta);
        }
    }
    if (ncol > NT) {  // second column pass (T = 128 only)
        for (int i = 0; i < nrel; ++i) {
            const double s = readlane_f64(sk, i);
            if (has1) {
                const int idx = __builtin_amdgcn_readlane(row, i) * stride + 1 + tid + NT;
                acc1 = fma(s, GRAN ? poll_gran(rows, idx, tag, tmo) : ld_wt(rows, idx), acc1);
            }
        }
    }
    put_final<NT>(rho, acc0, acc1, eta, nrel, has0, has1, sm, out_row, w_eps_out);
    return true;
}

// Arrive on `counter` after this workgroup's write-through stores; true in
// every thread of the workgroup that arrived last (which re-arms the counter).
// sc1 loads alone stand in for the acquire only at one workgroup per CU (the
// measured form, MI355X guide "Valid forms"); with `acquire` (larger grids)
// the last arriver also runs an agent-scope acquire before the barrier.
template <int NT>
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned expected, unsigned* s_flag, bool acquire) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = prev == expected - 1;
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (last && acquire) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *s_flag = last ? 1u : 0u;
    }
    __syncthreads();
    return *s_flag != 0;
}

// Upper median of 10 (rank 5): a 29-comparator sorting network (verified on all
// 2^10 0/1 inputs), the element scipy.ndimage.median_filter(size=10) returns.
__device__ __forceinline__ double median10(double* v) {
#define CX(i, j) { const double lo = fmin(v[i], v[j]), hi = fmax(v[i], v[j]); v[i] = lo; v[j] = hi; }
    CX(4, 9) CX(3, 8) CX(2, 7) CX(1, 6) CX(0, 5) CX(1, 4) CX(6, 9) CX(0, 3) CX(5, 8) CX(0, 2)
    CX(3, 6) CX(7, 9) CX(0, 1) CX(2, 4) CX(5, 7) CX(8, 9) CX(1, 2) CX(4, 6) CX(7, 8) CX(3, 5)
    CX(2, 5) CX(6, 8) CX(1, 3) CX(4, 7) CX(2, 3) CX(6, 7) CX(3, 4) CX(5, 6) CX(4, 5)
#undef CX
    return v[5];
}

// Median filter (scipy.ndimage.median_filter(size=10, mode='reflect'),
// control.py:319-327, window [t-5, t+4], valid for T >= 5), u += w_eps
// (control.py:126), shift (control.py:148-149) and the fp32 per-step constants
// of the next launch.  u_cur: this thread's cur->u[t][d] (t = tid/2, d = tid%2),
// read at kernel entry.
template <int NT>
__device__ void nominal_update_block(const DevStep* cur, DevStep* nxt, const KConst& c, MergeScratch& sm,
                                     double u_cur) {
    const int tid = threadIdx.x;
    const int T = c.T;
    if (tid < 2 * T) {
        const int t = tid >> 1, d = tid & 1;
        double v[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            int m = t - 5 + i;              // one reflection suffices for T >= 5
            m = m < 0 ? -m - 1 : m;
            m = m >= T ? 2 * T - 1 - m : m;
            v[i] = sm.weps[2 * m + d];
        }
        sm.unew[tid] = u_cur + median10(v);
    }
    __syncthreads();
    if (tid < T) {
        const int src = tid + 1 < T ? tid + 1 : T - 1;
        const double u0 = sm.unew[2 * src], u1 = sm.unew[2 * src + 1];
        nxt->u[tid][0] = u0;
        nxt->u[tid][1] = u1;
        const double g0 = c.gamma * u0, g1 = c.gamma * u1;
        const double a0 = g0 * c.sig_inv[0] + g1 * c.sig_inv[2];
        const double a1 = g0 * c.sig_inv[1] + g1 * c.sig_inv[3];
        nxt->ua[tid] = make_float4((float)u0, (float)u1, (float)a0, (float)a1);
    }
    // win / key / x0 / ctr are written to both ping-pong blocks by
    // mppi_set_step_inputs, so only the nominal moves here.
}

// ------------------------------------------------------------ rollout kernel

// Noise row load for step t.  Each prefetch is followed by an empty asm
// statement with a memory clobber: a scheduling boundary that keeps the load
// where it is written (otherwise the scheduler sinks it next to its use and
// every step pays the full memory latency).
#ifdef MPPI_ABL_NONOISE  // diagnostic ablation: no noise traffic (wrong results)
__device__ __forceinline__ float2 noise_ld(const float2* p) {
    const unsigned a = (unsigned)(uintptr_t)p;
    return make_float2((float)(a & 255u) * 0.01f - 1.2f, (float)((a >> 8) & 255u) * 0.01f - 1.2f);
}
#else
__device__ __forceinline__ float2 noise_ld(const float2* p) { return *p; }
#endif
#define PIN_LOADS() asm volatile("" ::: "memory")

// The per-step constants are read through the constant address space: scalar
// (SMEM) loads that stay scalar across the scheduling boundaries above.  The
// block is written only by host copies or by the PREVIOUS launch (ping-pong).
typedef __attribute__((address_space(4))) const float cfloat;
__device__ __forceinline__ float4 const_ld4(cfloat* p) { return make_float4(p[0], p[1], p[2], p[3]); }

typedef float f32x2 __attribute__((ext_vector_type(2)));

// v_min3_f32 / v_min_f32 issued directly: the operands are bit-packed keys, and
// fminf() would make hipcc canonicalise every one of them (v_max x, x) first.
__device__ __forceinline__ float min3_raw(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float min_raw(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int LPS>
struct Search {
    // window slots per lane, even so they pair up for packed math
    static constexpr int SL = ((MPPI_SEARCH_LEN + LPS - 1) / LPS + 1) & ~1;
    static constexpr int SP = SL / 2;
    f32x2 krx[SP], kry[SP], kc[SP];
    int sub;
    float cx, cy;

    // Nearest waypoint of the shared window (control.py:208-215):
    //   argmin_j |p - r_j|^2 = argmin_j (|r'_j|^2 - 2 p'.r'_j) (window-centred),
    // two slots per v_pk_fma_f32; the slot index is packed into the 5 low
    // mantissa bits so one v_min3 per two slots carries the argmin; the LPS
    // lanes of a sample close it with DPP.
    __device__ __forceinline__ unsigned nearest(float px, float py) const {
        const float ax = -2.f * (px - cx), ay = -2.f * (py - cy);
        const f32x2 ax2 = {ax, ax}, ay2 = {ay, ay};
        float best = 3.0e38f;
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            const f32x2 key = __builtin_elementwise_fma(ax2, krx[i], __builtin_elementwise_fma(ay2, kry[i], kc[i]));
            const unsigned j = (unsigned)(sub * SL + 2 * i);
            const float k0 = __uint_as_float((__float_as_uint(key.x) & ~31u) | j);
            const float k1 = __uint_as_float((__float_as_uint(key.y) & ~31u) | (j + 1));
            best = min3_raw(best, k0, k1);
        }
        if (LPS >= 2) best = min_raw(best, dpp_f32<0xB1>(best));  // quad_perm xor 1
        if (LPS >= 4) best = min_raw(best, dpp_f32<0x4E>(best));  // quad_perm xor 2
        return __float_as_uint(best) & 31u;
    }
};

__device__ __forceinline__ float weighted_sq(float ex, float ey, float e1, float e2, const float* w) {
    return fmaf(w[0], ex * ex, fmaf(w[1], ey * ey, fmaf(w[2], e1 * e1, w[3] * e2 * e2)));
}

// Diagnostic builds only (-DMPPI_STAMPS, a separate .so): per-workgroup
// timeline in s_memrealtime ticks (100 MHz) + counters.  Never in the product.
#ifdef MPPI_STAMPS
#define STAMP(slot, val) do { if (dbg && threadIdx.x == 0) dbg[(size_t)blockIdx.x * 16 + (slot)] = (val); } while (0)
#define NOW() __builtin_amdgcn_s_memrealtime()
#else
#define STAMP(slot, val) do { (void)dbg; } while (0)
#define NOW() 0ull
#endif

constexpr int kPF = 4;  // noise rows in flight per lane
constexpr int kSparseMax = 16;  // weighted samples per workgroup handled by the gather path

// POLL: the partial rows travel as tagged granules (see st_gran) to consumer
// workgroups that poll for them — the highest-numbered workgroup of each group
// of kGroup merges its group, workgroup nblocks - 1 merges the groups — so no
// workgroup drains its stores or waits on a counter, and the merges overlap the
// stragglers.  Needs every workgroup resident at once (the host enables it
// when the grid is at most one workgroup per CU); correctness does not depend
// on placement or order, every value is tag-checked.  Otherwise (!POLL) the
// last workgroup to arrive on a counter merges (arrive_last).
template <int LPS, int NT, bool POLL>
__global__ __launch_bounds__(NT) void rollout_kernel(
    const KConst c, const DevStep* __restrict__ st, const float2* __restrict__ noise,
    double* __restrict__ S_out, double* __restrict__ slab, double* __restrict__ gslab,
    unsigned* __restrict__ counters, double* __restrict__ partial_out, double* __restrict__ w_eps_out,
    DevStep* __restrict__ nxt, unsigned flags, unsigned* __restrict__ epoch, unsigned* __restrict__ tmo,
    unsigned long long* __restrict__ dbg) {
    __shared__ float4 s_win[kSlots];
    __shared__ float s_redf[NT / 64];
    __shared__ int s_cnt[NT / 64];
    __shared__ int s_k[NT];
    __shared__ float s_e[NT];
    __shared__ unsigned s_flag;
    __shared__ MergeScratch sm;

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
    // this launch's granule tag (device epoch + 1), fetched now so its latency is hidden
    const unsigned tag_v = POLL ? __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    // nominal element for the fused update, fetched now so its latency is hidden
    const double u_cur = ((flags & MPPI_FLAG_FUSED_UPDATE) && tid < 2 * T) ? st->u[tid >> 1][tid & 1] : 0.0;
    if (tid < kSlots) s_win[tid] = st->win[tid];
    Search<LPS> sr;
    if (LPS == 1) {
        // lane-opaque zero: keeps the 30 window slots in VGPRs (as uniform
        // values they would go to SGPRs and spill)
        int z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        sr.sub = z;
    } else {
        sr.sub = tid & (LPS - 1);
    }
    static_assert(Search<LPS>::SL * LPS <= kSlots, "window slots");
#pragma unroll
    for (int i = 0; i < Search<LPS>::SP; ++i) {
        const float4 k0 = st->key[sr.sub * Search<LPS>::SL + 2 * i];
        const float4 k1 = st->key[sr.sub * Search<LPS>::SL + 2 * i + 1];
        sr.krx[i] = f32x2{k0.x, k1.x};
        sr.kry[i] = f32x2{k0.y, k1.y};
        sr.kc[i] = f32x2{k0.z, k1.z};
    }
    sr.cx = st->ctr.x;
    sr.cy = st->ctr.y;
    const float4 x0 = st->x0;
    ArmState x;
    x.q1 = x0.x;
    x.q2 = x0.y;
    x.dq1 = x0.z;
    x.dq2 = x0.w;
    sincos_f32(x.q1, &x.s1, &x.c1);
    sincos_f32(x.q1 + x.q2, &x.s12, &x.c12);
    const float2* np = noise + k;
    cfloat* cua = (cfloat*)(st->ua);
    float2 ring[kPF];   // noise rows eps[t][k] in flight
    float4 uring[kPF];  // per-step constants (u_t, a_t), uniform
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
        const int tj = j < T ? j : T - 1;
        ring[j] = noise_ld(np + (size_t)tj * K);
        uring[j] = const_ld4(cua + 4 * tj);
    }
    __syncthreads();

    // Horizon loop (control.py:95-109): v = u + eps -> _F -> end effector ->
    // nearest waypoint -> stage cost + control cost, S in fp64.
    double S = 0.0;
    float S4 = 0.f;  // fp32 partial over one 4-step block, folded into fp64 S
    float ex = 0.f, ey = 0.f, e1 = 0.f, e2 = 0.f;
    // `slot` (= t % kPF) is a compile-time constant at every call, so the rings
    // stay in registers (a runtime index sends them to scratch).
    auto step = [&](int t, auto slot_c) {
        constexpr int slot = decltype(slot_c)::value;
        const float2 e = ring[slot];
        const float4 ua = uring[slot];
        const int tl = t + kPF < T ? t + kPF : T - 1;
        ring[slot] = noise_ld(np + (size_t)tl * K);
        uring[slot] = const_ld4(cua + 4 * tl);
        PIN_LOADS();
        const float v1 = fmaf(exf, ua.x, e.x);  // u[t] + eps (exploit) or eps, control.py:99-101
        const float v2 = fmaf(exf, ua.y, e.y);
        dyn_step(x, v1, v2, c);
        const float px = fmaf(c.fk1, x.c1, c.fk2 * x.c12);  // control.py:178-179
        const float py = fmaf(c.fk1, x.s1, c.fk2 * x.s12);
        const float4 r = s_win[sr.nearest(px, py)];
        ex = px - r.x;
        ey = py - r.y;
        e1 = x.dq1 - r.z;
        e2 = x.dq2 - r.w;
        const float g = fmaf(ua.z, v1, ua.w * v2);  // (gamma u^T Sigma^-1) v, control.py:106
        S4 += weighted_sq(ex, ey, e1, e2, c.sw) + g;
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    static_assert(kPF == 4, "unrolled for a 4-deep ring");
    int t = 0;
    for (; t + kPF <= T; t += kPF) {
        step(t, I0{});
        step(t + 1, I1{});
        step(t + 2, I2{});
        step(t + 3, I3{});
        S += (double)S4;
        S4 = 0.f;
    }
    if (t < T) step(t, I0{});          // remainder: t % kPF == 0, 1, 2 in order
    if (t + 1 < T) step(t + 1, I1{});
    if (t + 2 < T) step(t + 2, I2{});
    S += (double)S4;
    S += (double)weighted_sq(ex, ey, e1, e2, c.tw);  // terminal cost, control.py:109

    STAMP(1, NOW());
    const bool owner = valid && sr.sub == 0;
    if (S_out && owner) S_out[k] = S;

    // ---- workgroup partial: rho_b, eta_b, N_b (control.py:112-118 over this block)
    const double rho_b = block_min_f64<NT>(owner ? S : INFINITY, sm);
    // weights below 2^-64 of the block's best are dropped (see kMergeFloor)
    const float wgt = owner ? __expf((float)((rho_b - S) * c.inv_lambda)) : 0.f;
    const bool nz = wgt >= 5.421010862e-20f;
    const unsigned long long bal = __ballot(nz);
    const float esum = wave_sum_f32(nz ? wgt : 0.f);
    if (lane == 0) {
        s_cnt[wave] = __popcll(bal);
        s_redf[wave] = esum;
    }
    __syncthreads();
    int off = 0, nl = 0;
    double eta_b = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        off += (w < wave) ? s_cnt[w] : 0;
        nl += s_cnt[w];
        eta_b += (double)s_redf[w];
    }
    if (nz) {
        const int pos = off + lanes_below(bal);
        s_k[pos] = k;
        s_e[pos] = wgt;
    }
    __syncthreads();
    const int stride = 2 + 2 * T;
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
    nl = __builtin_amdgcn_readfirstlane(nl);
    if (nl <= kSparseMax) {
        // few weighted samples (the usual case: S spread >> lambda): column
        // threads gather eps[t][k_l] for the listed samples, all loads of a
        // column issued together
        const float* nf = reinterpret_cast<const float*>(noise);
        for (int col = tid; col < 2 * T; col += NT) {
            const float* base = nf + (size_t)(col >> 1) * K * 2 + (col & 1);
            float e[kSparseMax];
#pragma unroll
            for (int l = 0; l < kSparseMax; ++l) e[l] = base[(size_t)(nl > 0 ? s_k[min(l, nl - 1)] : 0) * 2];
            double acc = 0.0;
#pragma unroll
            for (int l = 0; l < kSparseMax; ++l)
                if (l < nl) acc = fma((double)s_e[l], (double)e[l], acc);
            publish(blockIdx.x * stride + 2 + col, acc);
        }
    } else {
        // dense weights: each wave takes whole rows eps[t][k0 : k0 + NS] (coalesced),
        // lane l owns samples l, l + 64, ...; the loads of kRowBatch rows are in
        // flight together, then one DPP wave reduction per row and component
        constexpr int NS = NT / LPS;               // samples of this workgroup
        constexpr int PER = (NS + 63) / 64;
        constexpr int kRowBatch = 4;
        const int k0 = blockIdx.x * NS;
        if (tid < NS) s_e[tid] = 0.f;
        __syncthreads();
        if (nz) s_e[k - k0] = wgt;
        __syncthreads();
        double w[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int ks = lane + 64 * i;
            w[i] = (ks < NS && k0 + ks < K) ? (double)s_e[ks] : 0.0;
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
    if (tid == 0) {
        publish(blockIdx.x * stride, rho_b);
        publish(blockIdx.x * stride + 1, eta_b);
    }
    STAMP(2, NOW());
    STAMP(5, (unsigned long long)nl);
    const int g = blockIdx.x / kGroup;
    const int gsz = min(kGroup, nrows - g * kGroup);
    if constexpr (POLL) {
        // ---- level 1: the group's highest-numbered workgroup polls and merges its rows
        if ((int)blockIdx.x != g * kGroup + gsz - 1) return;
        STAMP(3, NOW());
        if (ngroups == 1) {
            merge_rows_block<NT, true, true>(slab_r, 0, gsz, c, sm, nullptr, 0, partial_out, w_eps_out, tag, tmo);
        } else if ((int)blockIdx.x == nrows - 1 && nrows <= kDirectRows &&
                   direct_merge<NT, true>(slab_r, nrows, c, sm, partial_out, w_eps_out, tag, tmo)) {
            // few weighted rows: finished straight from the workgroup rows
        } else {
            merge_rows_block<NT, false, true>(slab_r, g * kGroup, gsz, c, sm, &gslab_r, g, nullptr, nullptr, tag, tmo);
            STAMP(10, NOW());
            // ---- level 2: the last workgroup polls and merges the group rows
            if ((int)blockIdx.x != nrows - 1) return;
            STAMP(4, NOW());
            merge_rows_block<NT, true, true>(gslab_r, 0, ngroups, c, sm, nullptr, 0, partial_out, w_eps_out, tag,
                                             tmo);
        }
        // every workgroup read the epoch before publishing, and all have published
        if (threadIdx.x == 0) __hip_atomic_store(epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        // ---- level 1: the last workgroup of each group of kGroup merges the group
        if (!arrive_last<NT>(counters + g, (unsigned)gsz, &s_flag, c.acquire != 0)) return;
        STAMP(3, NOW());
        merge_rows_block<NT, false, false>(slab_r, g * kGroup, gsz, c, sm, &gslab_r, g, nullptr, nullptr, 0u, nullptr);
        STAMP(10, NOW());
        // ---- level 2: the last group merges the group rows and finishes the step
        if (!arrive_last<NT>(counters + ngroups, (unsigned)ngroups, &s_flag, c.acquire != 0)) return;
        STAMP(4, NOW());
        // the same decision as the poll form (identical results either way)
        if (!(ngroups > 1 && nrows <= kDirectRows &&
              direct_merge<NT, false>(slab_r, nrows, c, sm, partial_out, w_eps_out, 0u, nullptr)))
            merge_rows_block<NT, true, false>(gslab_r, 0, ngroups, c, sm, nullptr, 0, partial_out, w_eps_out, 0u,
                                              nullptr);
    }
    STAMP(11, NOW());
    STAMP(6, (unsigned long long)sm.nrel);
    if (flags & MPPI_FLAG_FUSED_UPDATE) nominal_update_block<NT>(st, nxt, c, sm, u_cur);
    STAMP(7, NOW());
}

constexpr int kMergeThreads = 256;

__global__ __launch_bounds__(kMergeThreads) void merge_kernel(const KConst c, const double* parts, int n,
                                                              double* w_eps_out, const DevStep* cur,
                                                              DevStep* nxt, unsigned flags) {
    __shared__ MergeScratch sm;
    const int tid = threadIdx.x;
    const double u_cur = ((flags & MPPI_FLAG_FUSED_UPDATE) && tid < 2 * c.T) ? cur->u[tid >> 1][tid & 1] : 0.0;
    const __amdgpu_buffer_rsrc_t r = rows_rsrc(parts, n * (2 + 2 * c.T) * 8);
    merge_rows_block<kMergeThreads, true, false>(r, 0, n, c, sm, nullptr, 0, nullptr, w_eps_out, 0u, nullptr);
    if (flags & MPPI_FLAG_FUSED_UPDATE) nominal_update_block<kMergeThreads>(cur, nxt, c, sm, u_cur);
}

// Trajectory re-roll (control.py:129-145): control(t) = base[(t-1) mod T] (+ eps).
__global__ __launch_bounds__(kThreads) void traj_kernel(const KConst c, const DevStep* __restrict__ st,
                                                        const float2* __restrict__ base,
                                                        const float2* __restrict__ noise, int Kn,
                                                        float4* __restrict__ out) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= Kn) return;
    const int T = c.T;
    const float exf = noise ? ((c.k_offset + k) < c.k_exploit ? 1.f : 0.f) : 1.f;
    const float4 x0 = st->x0;
    ArmState x;
    x.q1 = x0.x;
    x.q2 = x0.y;
    x.dq1 = x0.z;
    x.dq2 = x0.w;
    sincos_f32(x.q1, &x.s1, &x.c1);
    sincos_f32(x.q1 + x.q2, &x.s12, &x.c12);
    for (int t = 0; t < T; ++t) {
        const int ti = t == 0 ? T - 1 : t - 1;
        const float2 b = base[ti];
        float v1 = b.x, v2 = b.y;
        if (noise) {
            const float2 e = noise[(size_t)ti * c.K_local + k];
            v1 = fmaf(exf, b.x, e.x);
            v2 = fmaf(exf, b.y, e.y);
        }
        dyn_step(x, v1, v2, c);
        out[(size_t)k * T + t] = make_float4(x.q1, x.q2, x.dq1, x.dq2);
    }
}

// Philox4x32-10 (Salmon et al., SC'11) + Box-Muller; eps = L z, L = chol(Sigma).
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned lo0 = 0xD2511F53u * ctr.x, hi0 = __umulhi(0xD2511F53u, ctr.x);
        const unsigned lo1 = 0xCD9E8D57u * ctr.z, hi1 = __umulhi(0xCD9E8D57u, ctr.z);
        ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return ctr;
}

__global__ __launch_bounds__(kThreads) void philox_noise_kernel(int K_local, int T, long long k_offset,
                                                                unsigned long long seed,
                                                                unsigned long long step, float L00,
                                                                float L10, float L11, float2* out) {
    const long long idx = (long long)blockIdx.x * kThreads + threadIdx.x;
    const int tp = (T + 1) / 2;
    if (idx >= (long long)K_local * tp) return;
    const int k = (int)(idx % K_local);
    const int t0 = 2 * (int)(idx / K_local);
    const unsigned long long kg = (unsigned long long)(k_offset + k);
    const uint4 ctr = make_uint4((unsigned)kg, (unsigned)(kg >> 32), (unsigned)t0, (unsigned)step);
    const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32) ^ (unsigned)(step >> 32));
    const uint4 r = philox4x32_10(ctr, key);
    const float inv = 2.3283064365386963e-10f;  // 2^-32
    const float u0 = ((float)r.x + 1.0f) * inv, u1 = (float)r.y * inv;
    const float u2 = ((float)r.z + 1.0f) * inv, u3 = (float)r.w * inv;
    float s, co;
    const float ra = sqrtf(-2.0f * logf(fminf(u0, 1.0f)));
    sincospif(2.0f * u1, &s, &co);
    const float z0 = ra * co, z1 = ra * s;
    const float rb = sqrtf(-2.0f * logf(fminf(u2, 1.0f)));
    sincospif(2.0f * u3, &s, &co);
    const float z2 = rb * co, z3 = rb * s;
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
    DevStep* d_step = nullptr;  // [2] ping-pong
    int cur = 0;
    DevStep* h_step = nullptr;  // pinned staging
    hipEvent_t staged = nullptr;
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
    double sig_inv[4];
    unsigned long long* d_dbg = nullptr;  // diagnostic stamp buffer (MPPI_STAMPS builds)
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

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
    if (c->h_tmo && __atomic_load_n(c->h_tmo, __ATOMIC_ACQUIRE)) {
        *c->h_tmo = 0;
        return fail(MPPI_E_HIP, "in-launch hand-off timed out (workgroups not co-resident?); results invalid");
    }
    return MPPI_OK;
}

int auto_lps(int K_local) {
    // Measured on MI355X (tools/ubench_valu.hip, tools/stamps.py): a lone wave
    // issues a VALU op every ~6-8 cycles, 2 waves/SIMD ~4.4, 4 waves ~3.0.
    // Splitting the window search over LPS lanes multiplies the instructions
    // per sample by ~1.6 (LPS=2) / ~2.7 (LPS=4); at K = 65536 (one wave per
    // SIMD) one lane per sample won (37 vs 45 us span), so split only when the
    // grid would leave SIMDs empty.
    const long long waves1 = ((long long)K_local + 63) / 64;
    if (waves1 >= 1024) return 1;
    if (waves1 >= 256) return 2;
    return 4;
}
}  // namespace

extern "C" {

const char* mppi_last_error(void) { return g_err.c_str(); }

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
    if (lps != 1 && lps != 2 && lps != 4) {
        delete c;
        return fail(MPPI_E_ARG, "lanes_per_sample must be 0, 1, 2 or 4");
    }
    c->lps = lps;
    // 512-thread workgroups when the grid fills every CU with one of them (8 waves:
    // two per SIMD); 256 otherwise.  MPPI_BLOCK=256|512 overrides (diagnostics).
    const long long lanes = (long long)cfg->K_local * lps;
    c->nt = lanes >= 512LL * 256 ? 512 : 256;
    if (const char* ev = getenv("MPPI_BLOCK")) c->nt = atoi(ev) == 512 ? 512 : 256;
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
    k.gamma = cfg->param_lambda * (1.0 - cfg->param_alpha);  // control.py:45
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
        if (c->nt == 512) rc = lps == 1 ? occupancy<1, 512>(&per_cu) : lps == 2 ? occupancy<2, 512>(&per_cu) : occupancy<4, 512>(&per_cu);
        else rc = lps == 1 ? occupancy<1, 256>(&per_cu) : lps == 2 ? occupancy<2, 256>(&per_cu) : occupancy<4, 256>(&per_cu);
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
        (e = hipHostMalloc(&c->h_step, sizeof(DevStep), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_buf, 2 * kMaxT * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_base, kMaxT * sizeof(float2), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_tmo, 256, hipHostMallocMapped)) != hipSuccess ||
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
    *c->h_tmo = 0;
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
    if (c->h_step) (void)hipHostFree(c->h_step);
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->h_base) (void)hipHostFree(c->h_base);
    if (c->h_tmo) (void)hipHostFree(c->h_tmo);
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

int mppi_set_step_inputs(mppi_ctx* c, const double* x0, const double* window, int W, const double* u) {
    if (!c || !x0 || !window) return fail(MPPI_E_ARG, "null argument");
    if (W < 1 || W > MPPI_SEARCH_LEN) return fail(MPPI_E_ARG, "window rows must be in [1, 30]");
    HIP_TRY(hipEventSynchronize(c->staged));  // staging block free again
    DevStep* h = c->h_step;
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
            h->win[j] = make_float4((float)r[0], (float)r[1], (float)r[2], (float)r[3]);
            const double rx = r[0] - cx, ry = r[1] - cy;
            h->key[j] = make_float4((float)rx, (float)ry, (float)(rx * rx + ry * ry), 0.f);
        } else {
            h->win[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            h->key[j] = make_float4(0.f, 0.f, kPadKey, 0.f);
        }
    }
    h->x0 = make_float4((float)x0[0], (float)x0[1], (float)x0[2], (float)x0[3]);
    h->ctr = make_float4((float)cx, (float)cy, (float)W, 0.f);
    size_t bytes = offsetof(DevStep, ua);
    if (u) {
        const KConst& k = c->kc;
        for (int t = 0; t < c->cfg.T; ++t) {
            const double u0 = u[2 * t], u1 = u[2 * t + 1];
            const double g0 = k.gamma * u0, g1 = k.gamma * u1;  // ((gamma u^T) Sigma^-1), control.py:106
            const double a0 = g0 * k.sig_inv[0] + g1 * k.sig_inv[2];
            const double a1 = g0 * k.sig_inv[1] + g1 * k.sig_inv[3];
            h->ua[t] = make_float4((float)u0, (float)u1, (float)a0, (float)a1);
            h->u[t][0] = u0;
            h->u[t][1] = u1;
        }
        bytes = sizeof(DevStep);
    }
    // static part (window, keys, x0) into both ping-pong blocks, nominal into the current one
    HIP_TRY(hipMemcpyAsync(c->d_step + (c->cur ^ 1), h, offsetof(DevStep, ua), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_step + c->cur, h, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->staged, c->stream));
    return MPPI_OK;
}

int mppi_rollout(mppi_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags) {
    if (!c || !noise_dev) return fail(MPPI_E_ARG, "null argument");
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    const DevStep* cur = c->d_step + c->cur;
    DevStep* nxt = c->d_step + (c->cur ^ 1);
    const float2* nz = reinterpret_cast<const float2*>(noise_dev);
#define MPPI_LAUNCH2(L, NTH, P)                                                                                \
    hipLaunchKernelGGL((rollout_kernel<L, NTH, P>), dim3(c->nblocks), dim3(NTH), 0, c->stream, c->kc, cur, nz, \
                       S_dev, c->d_slab, c->d_gslab, c->d_counter, partial_dev, c->d_weps, nxt, flags, c->d_epoch, \
                       c->d_tmo, c->d_dbg)
#define MPPI_LAUNCH(L, NTH)               \
    do {                                  \
        if (c->poll) MPPI_LAUNCH2(L, NTH, true);  \
        else MPPI_LAUNCH2(L, NTH, false); \
    } while (0)
    if (c->nt == 512) {
        if (c->lps == 1) MPPI_LAUNCH(1, 512);
        else if (c->lps == 2) MPPI_LAUNCH(2, 512);
        else MPPI_LAUNCH(4, 512);
    } else {
        if (c->lps == 1) MPPI_LAUNCH(1, 256);
        else if (c->lps == 2) MPPI_LAUNCH(2, 256);
        else MPPI_LAUNCH(4, 256);
    }
#undef MPPI_LAUNCH
#undef MPPI_LAUNCH2
    const int rc = launch_check("rollout_kernel");
    if (rc == MPPI_OK && (flags & MPPI_FLAG_FUSED_UPDATE)) c->cur ^= 1;
    return rc;
}

int mppi_merge_partials(mppi_ctx* c, const double* partials_dev, int n, unsigned flags) {
    if (!c || !partials_dev || n < 1) return fail(MPPI_E_ARG, "bad argument");
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    const DevStep* cur = c->d_step + c->cur;
    DevStep* nxt = c->d_step + (c->cur ^ 1);
    hipLaunchKernelGGL(merge_kernel, dim3(1), dim3(kMergeThreads), 0, c->stream, c->kc, partials_dev, n,
                       c->d_weps, cur, nxt, flags);
    const int rc = launch_check("merge_kernel");
    if (rc == MPPI_OK && (flags & MPPI_FLAG_FUSED_UPDATE)) c->cur ^= 1;
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
    if (base_u) {
        HIP_TRY(hipEventSynchronize(c->staged));
        for (int t = 0; t < c->cfg.T; ++t) c->h_base[t] = make_float2((float)base_u[2 * t], (float)base_u[2 * t + 1]);
        HIP_TRY(hipMemcpyAsync(c->d_base, c->h_base, c->cfg.T * sizeof(float2), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->staged, c->stream));
        base = c->d_base;
    } else {
        // nominal u0,u1 of the current step block: ua[t].xy, read with stride 16 B
        HIP_TRY(hipMemcpy2DAsync(c->d_base, sizeof(float2), (const char*)cur + offsetof(DevStep, ua), sizeof(float4),
                                 sizeof(float2), c->cfg.T, hipMemcpyDeviceToDevice, c->stream));
        base = c->d_base;
    }
    const int blocks = (K + kThreads - 1) / kThreads;
    hipLaunchKernelGGL(traj_kernel, dim3(blocks), dim3(kThreads), 0, c->stream, c->kc, cur, base,
                       reinterpret_cast<const float2*>(noise_dev), K, reinterpret_cast<float4*>(out_dev));
    return launch_check("traj_kernel");
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
    const long long n = (long long)c->cfg.K_local * ((c->cfg.T + 1) / 2);
    const int blocks = (int)((n + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(philox_noise_kernel, dim3(blocks), dim3(kThreads), 0, c->stream, c->cfg.K_local,
                       c->cfg.T, (long long)c->cfg.k_offset, seed, step, (float)L00, (float)L10, (float)L11,
                       reinterpret_cast<float2*>(out_dev));
    return launch_check("philox_noise_kernel");
}

int mppi_debug_set_buffer(mppi_ctx* c, void* dbg_dev) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    c->d_dbg = (unsigned long long*)dbg_dev;
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
