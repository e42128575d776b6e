// mppi_chain.hip — MI355X (gfx950) MPPI engine for an n-link planar chain
// (BASELINE config 5: "7-DoF arm dynamics (extended sys_params.py), K=131072
// T=128, xydq_circle.txt reference").  The reference has no 7-DoF model; the
// model is build-defined (oracle/chain_oracle.py, equations there) and reduces
// to the reference's _F (control.py:234-263) at n = 2 with inertia := length.
//
//  * chain_rollout_kernel<N>: one lane per sample, the whole n-link step in
//    fp32 registers (fully unrolled for N): prefix sums -> cos/sin of the
//    absolute-angle differences from the cached sincos -> D = mu o cos(.) + I,
//    Coriolis/centrifugal and gravity terms -> Cholesky of D (v_rsq) -> two
//    triangular solves -> joint accelerations -> semi-implicit Euler -> new
//    sincos (shared with the next step and the end-effector kinematics) ->
//    the window search of the 2-link engine -> stage + control cost.  Noise is
//    [T][K][N] fp32 (like the 2-link engine's [T][K][2]): a sample's N values of
//    a step contiguous, so a weighted sample's noise is T cache lines.  Same epilogue,
//    in-launch merges and fused update as the 2-link engine (mppi_device.h),
//    with T*N columns per partial row (MAXCH = 4 column chunks).
//  * chain_traj_kernel<N, NOISE>, chain_philox_kernel: trajectory re-roll and
//    counter-based Gaussian noise with an n x n Cholesky factor.
//
// C ABI: include/mppi_rocm.h (mppi_chain_*).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "mppi_device.h"
#include "mppi_host.h"
#include "mppi_rocm.h"

namespace {

using namespace mppi;

constexpr int kCMax = MPPI_CHAIN_MAX_DOF;   // links
constexpr int kCDebugN = 7;                  // the link count with slot-recording debug instances (config 5)
constexpr int kCT = 256;                    // threads per workgroup, one lane per sample
constexpr int kCMaxCh = 4;                  // column chunks of a partial row: T N + 1 <= 4 x 256 ... (N <= 7)
constexpr int kCMaxVals = kMaxT * kCMax;    // T N values per row, at most
constexpr int kCPF = 2;                     // noise steps in flight per lane (N rows each)
// the same for a quad per sample (its steps are ~4x shorter); 2 and 4 measured: equal at K = 16384, 4 -2.1 % at
// K = 32768 (profiles/r13/chain_quad_ring_depth_ab.txt)
constexpr int kQPF = 4;
constexpr int kCPU = 2;                     // per-step constant rows in flight

// Device-resident per-step parameter block (ping-pong pair in the context).
struct alignas(16) ChainStep {
    float4 win[kSlots];                    // rx, ry, rdq1, rdq2 of window slot j
    float4 key[kSlots];                    // centred search keys (see Search)
    float4 ctr;                            // window centre (cx, cy), W
    float x0[2 * kCMax];                   // q[n], dq[n]
    double x0d[2 * kCMax];                 // the same in fp64 (fp64 rollout)
    double wind[kSlots][4];                // the window rows in fp64 (fp64 rollout); rows >= W unused
    float ua[kMaxT + kCPU][2 * kCMax];     // u_t[n], a_t[n] (a = (gamma u_t)^T Sigma^-1), fp32; rows >= T zero
    double u[kMaxT][kCMax];                // nominal control sequence, fp64
    double a[kMaxT][kCMax];                // a_t in fp64 (fp64 rollout)
    double u_first[kCMax];                 // fused update: u_new[0], the element the shift drops (optimal_traj)
    double eta;                            // fused update: the merge's eta (read back with u_first)
};

// Launch constants (kernel argument, by value).
constexpr int kCDyn = 72;
struct ChainConst {
    int K_local, T, k_offset, k_exploit, nblocks, acquire, n, cu_off;   // cu_off: per-CU tickets in counters[]
    int fair, pad0;   // fair: > 1 workgroup per CU (fair_priority)
    alignas(8) float dyn[kCDyn];   // packed dynamics / cost constants (layout: kOff* below)
    double lambda, inv_lambda, gamma;
    double sig_inv[kCMax * kCMax];
};

using CScratch = MergeScratch<kCMaxVals>;

// The dynamics / cost constants, packed (floats, pairs 8-byte aligned).  The
// chain's coupling is separable: mu_ab = l_a nu_b for a < b (chain_oracle.py
// coefficients), so D' and the bias need only the per-link l and nu.  Pairs
// hold links / rows (2p, 2p+1); the pad link of an odd chain has l = nu = fk =
// damping = 0 and D'_aa = 1.  The rollout kernel reads them from a device copy
// through the constant address space every step (scalar loads re-issued after
// each step's scheduling boundary) rather than holding them in SGPRs across the
// loop, where they spill and return as v_readlane (~28 per step at n = 7).
enum : int {
    kOffL = 0,                    // l_a (dynamics link lengths)
    kOffNu = kOffL + kCMax,       // nu_a = m_a lc_a + l_a sum_{b>a} m_b
    kOffDd = kOffNu + kCMax,      // D'_aa = mu_aa + I_a + J_a + J_{a+1}
    kOffJ = kOffDd + kCMax,       // [a]: the pair holding row a+1 of column a: -J_{a+1} at row a+1, 0 beside it
    kOffDamp = kOffJ + 2 * kCMax, // joint viscous damping b_a
    kOffFk = kOffDamp + kCMax,    // cost kinematics lengths
    kOffSw = kOffFk + kCMax,      // stage weights x 10000
    kOffTw = kOffSw + 4,          // terminal weights x 10000
    kOffDt = kOffTw + 4,
    kOffG = kOffDt + 1,
    kDynFloats = kOffG + 7,
};
static_assert(kDynFloats == kCDyn, "dyn layout");
constexpr int kDynF64Off = (kCDyn + 1) & ~1;   // floats before the fp64 copy of the constants (8-B aligned)

template <class F>   // F: const float (generic, kernel argument) or cfloat (constant address space)
struct Dyn {
    F* p;
    __device__ __forceinline__ f32x2 pair(int off, int i) const { return f32x2{p[off + 2 * i], p[off + 2 * i + 1]}; }
    __device__ __forceinline__ f32x2 l2(int i) const { return pair(kOffL, i); }
    __device__ __forceinline__ f32x2 nu2(int i) const { return pair(kOffNu, i); }
    __device__ __forceinline__ f32x2 damp2(int i) const { return pair(kOffDamp, i); }
    __device__ __forceinline__ f32x2 fk2(int i) const { return pair(kOffFk, i); }
    __device__ __forceinline__ f32x2 joff2(int a) const { return pair(kOffJ, a); }
    __device__ __forceinline__ float Dd(int a) const { return p[kOffDd + a]; }
    __device__ __forceinline__ float dt() const { return p[kOffDt]; }
    __device__ __forceinline__ float g() const { return p[kOffG]; }
};
using DynMem = Dyn<cfloat>;
using DynArg = Dyn<const float>;

__device__ __forceinline__ f32x2 splat(float x) { return f32x2{x, x}; }
__device__ __forceinline__ f32x2 pfma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
template <int P> __device__ __forceinline__ float get(const f32x2 (&v)[P], int i) { return v[i >> 1][i & 1]; }
template <int P> __device__ __forceinline__ void put(f32x2 (&v)[P], int i, float x) { v[i >> 1][i & 1] = x; }

// Chain state of one sample in row pairs: joint angles / rates and the cached
// cos / sin of the absolute angles theta_a = q_1 + ... + q_a.  Pad entries of an
// odd chain stay 0.
template <int N>
struct ChainState {
    static constexpr int P = (N + 1) / 2;
    f32x2 q[P], dq[P], c[P], s[P];

    __device__ __forceinline__ void load(const float* x0) {
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] = dq[p] = c[p] = s[p] = f32x2{0.f, 0.f};
#pragma unroll
        for (int a = 0; a < N; ++a) {
            put(q, a, x0[a]);
            put(dq, a, x0[N + a]);
        }
        angles();
    }
    __device__ __forceinline__ float qa(int a) const { return get(q, a); }
    __device__ __forceinline__ float dqa(int a) const { return get(dq, a); }

    __device__ __forceinline__ void angles() {
        float th = 0.f;
#pragma unroll
        for (int a = 0; a < N; ++a) {
            th += get(q, a);
            float sa, ca;
            sincos_f32(th, &sa, &ca);
            put(s, a, sa);
            put(c, a, ca);
        }
    }

    // One semi-implicit Euler step (oracle/chain_oracle.py chain_forward_dynamics):
    //   D' theta_ddot = tau - bias - g,  tau_a = v'_a - v'_{a+1},  v' = v - b dq,
    //   D'_ab = l_a nu_b cos(th_a - th_b) (a < b; constants I_a + J_a + J_{a+1} on
    //   the diagonal and -J_{a+1} at (a+1, a): the joint armature in absolute
    //   angles), bias_a = sum_b mu_ab sin(th_a - th_b) thdot_b^2,
    //   g_a = g nu_a cos th_a, q_ddot_a = theta_ddot_a - theta_ddot_{a-1},
    //   dq += q_ddot dt, q += dq dt.
    // Packed (v_pk_*) over row pairs; D' is factored in place by a right-looking
    // Cholesky on column-major row pairs; the bias is O(n) through the prefix /
    // suffix sums the separable mu allows:
    //   bias_a = s_a X_a - c_a Y_a,  X_a = l_a C+_a + nu_a C-_a,  Y_a = l_a S+_a + nu_a S-_a,
    //   C+_a = sum_{b>a} nu_b w_b c_b,  C-_a = sum_{b<a} l_b w_b c_b  (S: s_b).
    template <class KC>
    __device__ __forceinline__ void step(const float (&v)[N], const KC& k) {
        f32x2 lc[P], ls[P], vc[P], vs[P], w[P];
        {
            float acc = 0.f;
#pragma unroll
            for (int a = 0; a < N; ++a) {
                acc += get(dq, a);
                put(w, a, acc);
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const f32x2 l = k.l2(p), nu = k.nu2(p);
            w[p] = w[p] * w[p];   // thdot^2
            lc[p] = l * c[p];
            ls[p] = l * s[p];
            vc[p] = nu * c[p];
            vs[p] = nu * s[p];
        }
        // r = tau - g - bias
        f32x2 r[P];
        {
            f32x2 ve[P], vv[P], Cs[P], Ss[P], Cp[P], Sp[P];
#pragma unroll
            for (int a = 0; a < N; ++a) put(vv, a, v[a]);
#pragma unroll
            for (int p = 0; p < P; ++p) ve[p] = pfma(-k.damp2(p), dq[p], vv[p]);
            f32x2 wvc[P], wvs[P], wlc[P], wls[P];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                wvc[p] = w[p] * vc[p];
                wvs[p] = w[p] * vs[p];
                wlc[p] = w[p] * lc[p];
                wls[p] = w[p] * ls[p];
            }
            float cs = 0.f, ss = 0.f, cp = 0.f, sp = 0.f;
#pragma unroll
            for (int a = N - 1; a >= 0; --a) {
                put(Cs, a, cs);
                put(Ss, a, ss);
                cs += get(wvc, a);
                ss += get(wvs, a);
            }
#pragma unroll
            for (int a = 0; a < N; ++a) {
                put(Cp, a, cp);
                put(Sp, a, sp);
                cp += get(wlc, a);
                sp += get(wls, a);
                put(r, a, a + 1 < N ? get(ve, a) - get(ve, a + 1) : get(ve, a));   // tau
            }
            const f32x2 mg = splat(-k.g());
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const f32x2 l = k.l2(p), nu = k.nu2(p);
                const f32x2 X = pfma(l, Cs[p], nu * Cp[p]);
                const f32x2 Y = pfma(l, Ss[p], nu * Sp[p]);
                r[p] = pfma(c[p], Y, pfma(-s[p], X, pfma(mg, vc[p], r[p])));
            }
        }
        // D' lower triangle, column-major row pairs: col[a][p] = rows (2p, 2p+1) of
        // column a; rows < a are don't-cares (kept finite).
        f32x2 col[N][P];
#pragma unroll
        for (int a = 0; a < N; ++a) {
            const f32x2 ca = splat(get(lc, a)), sa = splat(get(ls, a));
#pragma unroll
            for (int p = a / 2; p < P; ++p) {
                if ((a & 1) && p == a / 2) {
                    col[a][p] = splat(k.Dd(a));   // row a - 1: a don't-care
                    continue;
                }
                const f32x2 t = p == (a + 1) / 2 && a + 1 < N ? pfma(sa, vs[p], k.joff2(a)) : sa * vs[p];
                col[a][p] = pfma(ca, vc[p], t);
            }
            if (!(a & 1)) col[a][a / 2].x = k.Dd(a);
        }
        // Cholesky, right-looking: column j scaled by 1 / L_jj, then the trailing
        // columns k > j updated on the rows >= k.
        float inv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            inv[j] = __builtin_amdgcn_rsqf(col[j][j / 2][j & 1]);
            const f32x2 ij = splat(inv[j]);
#pragma unroll
            for (int p = (j + 1) / 2; p < P; ++p) col[j][p] = col[j][p] * ij;
#pragma unroll
            for (int kk = j + 1; kk < N; ++kk) {
                const f32x2 m = splat(-col[j][kk / 2][kk & 1]);
#pragma unroll
                for (int p = kk / 2; p < P; ++p) col[kk][p] = pfma(m, col[j][p], col[kk][p]);
            }
        }
        // L y = r, column-oriented (row j's own pair: only its partner row)
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const float y = r[j / 2][j & 1] * inv[j];
            r[j / 2][j & 1] = y;
            if (!(j & 1) && j + 1 < N) r[j / 2].y = fmaf(-y, col[j][j / 2].y, r[j / 2].y);
#pragma unroll
            for (int p = j / 2 + 1; p < P; ++p) r[p] = pfma(splat(-y), col[j][p], r[p]);
        }
        // L^T x = y, row dots over column i's rows > i (x_i itself is still 0)
        // (full pairs packed; row i's partner and the pad row of an odd chain scalar)
        f32x2 xs[P];
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {
            float e = r[i / 2][i & 1];
            if (!(i & 1) && i + 1 < N) e = fmaf(-col[i][i / 2].y, xs[i / 2].y, e);
            constexpr int PF = N / 2;   // pairs [0, PF) hold two real rows
            const int p0 = i / 2 + 1;
            if (p0 < PF) {
                f32x2 acc = col[i][p0] * xs[p0];
#pragma unroll
                for (int p = p0 + 1; p < PF; ++p) acc = pfma(col[i][p], xs[p], acc);
                e -= acc.x + acc.y;
            }
            if ((N & 1) && i < N - 1 && N / 2 >= p0) e = fmaf(-col[i][N / 2].x, xs[N / 2].x, e);
            xs[i / 2][i & 1] = e * inv[i];
        }
        // q_ddot = diff(theta_ddot); integrate
        f32x2 qdd[P];
#pragma unroll
        for (int a = 0; a < N; ++a) put(qdd, a, a ? get(xs, a) - get(xs, a - 1) : get(xs, 0));
        const f32x2 dt = splat(k.dt());
#pragma unroll
        for (int p = 0; p < P; ++p) {
            dq[p] = pfma(qdd[p], dt, dq[p]);
            q[p] = pfma(dq[p], dt, q[p]);
        }
        angles();
    }

    template <class KC>
    __device__ __forceinline__ void effector(const KC& k, float* px, float* py) const {
        f32x2 x = k.fk2(0) * c[0], y = k.fk2(0) * s[0];
#pragma unroll
        for (int p = 1; p < P; ++p) {
            const f32x2 f = k.fk2(p);
            x = pfma(f, c[p], x);
            y = pfma(f, s[p], y);
        }
        *px = x.x + x.y;
        *py = y.x + y.y;
    }
};
// The chain in fp64 (mppi_chain_config.precision = 1): the same equations as
// ChainState, scalar doubles, sincos from the fp64 library.  Used where the
// weights are spread (lambda comparable to the spread of S): in fp32 the
// end effector sits ~1e-6 m from the fp64 one after 128 steps, so at a near-tie
// of two window slots (slots 6e-5 m apart) the fp32 rollout may take the
// neighbour, and that stage cost moves S by up to ~1e-3 relative — harmless
// while one sample carries the weight, visible in w_eps when tens do.
typedef __attribute__((address_space(4))) const double cdouble;
// 1 / sqrt in fp64 on either side (the device's rsqrt; the host's sqrt and divide)
__host__ __device__ __forceinline__ double rsqrt_hd(double x) {
#ifdef __HIP_DEVICE_COMPILE__
    return rsqrt(x);
#else
    return 1.0 / sqrt(x);
#endif
}

template <int N>
struct ChainStateD {
    double q[N], dq[N], c[N], s[N];

    __host__ __device__ __forceinline__ void load(const double* x0) {
#pragma unroll
        for (int a = 0; a < N; ++a) {
            q[a] = x0[a];
            dq[a] = x0[N + a];
        }
        angles();
    }
    __host__ __device__ __forceinline__ void angles() {
        double th = 0.0;
#pragma unroll
        for (int a = 0; a < N; ++a) {
            th += q[a];
            sincos(th, &s[a], &c[a]);
        }
    }
    // one semi-implicit Euler step (ChainState::step, oracle/chain_oracle.py chain_forward_dynamics);
    // host and device: k is the fp64 constant block (constant memory on the device)
    template <class KP>
    __host__ __device__ __forceinline__ void step(const double (&v)[N], KP k) {
        double w[N], lc[N], ls[N], vc[N], vs[N], r[N];
        double acc = 0.0;
#pragma unroll
        for (int a = 0; a < N; ++a) {
            acc += dq[a];
            w[a] = acc * acc;   // thdot^2
            lc[a] = k[kOffL + a] * c[a];
            ls[a] = k[kOffL + a] * s[a];
            vc[a] = k[kOffNu + a] * c[a];
            vs[a] = k[kOffNu + a] * s[a];
        }
        double ve[N];
#pragma unroll
        for (int a = 0; a < N; ++a) ve[a] = fma(-k[kOffDamp + a], dq[a], v[a]);
        double Cs[N], Ss[N];
        {
            double cs = 0.0, ss = 0.0;
#pragma unroll
            for (int a = N - 1; a >= 0; --a) {
                Cs[a] = cs;
                Ss[a] = ss;
                cs = fma(w[a], vc[a], cs);
                ss = fma(w[a], vs[a], ss);
            }
        }
        {
            double cp = 0.0, sp = 0.0;
            const double g = k[kOffG];
#pragma unroll
            for (int a = 0; a < N; ++a) {
                const double X = fma(k[kOffL + a], Cs[a], k[kOffNu + a] * cp);
                const double Y = fma(k[kOffL + a], Ss[a], k[kOffNu + a] * sp);
                const double tau = a + 1 < N ? ve[a] - ve[a + 1] : ve[a];
                r[a] = fma(c[a], Y, fma(-s[a], X, fma(-g, vc[a], tau)));
                cp = fma(w[a], lc[a], cp);
                sp = fma(w[a], ls[a], sp);
            }
        }
        // D' lower triangle (L[i][a], i >= a), Cholesky in place
        double L[N][N];
#pragma unroll
        for (int a = 0; a < N; ++a) {
            L[a][a] = k[kOffDd + a];
#pragma unroll
            for (int i = a + 1; i < N; ++i) {
                const double t = fma(ls[a], vs[i], lc[a] * vc[i]);
                L[i][a] = i == a + 1 ? t + k[kOffJ + 2 * a + ((a + 1) & 1)] : t;   // -J_{a+1} beside the diagonal
            }
        }
        double inv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            inv[j] = rsqrt_hd(L[j][j]);
#pragma unroll
            for (int i = j + 1; i < N; ++i) L[i][j] *= inv[j];
#pragma unroll
            for (int kk = j + 1; kk < N; ++kk)
#pragma unroll
                for (int i = kk; i < N; ++i) L[i][kk] = fma(-L[i][j], L[kk][j], L[i][kk]);
        }
#pragma unroll
        for (int j = 0; j < N; ++j) {   // L y = r
            r[j] *= inv[j];
#pragma unroll
            for (int i = j + 1; i < N; ++i) r[i] = fma(-L[i][j], r[j], r[i]);
        }
#pragma unroll
        for (int i = N - 1; i >= 0; --i) {   // L^T x = y
            double e = r[i];
#pragma unroll
            for (int kk = i + 1; kk < N; ++kk) e = fma(-L[kk][i], r[kk], e);
            r[i] = e * inv[i];
        }
        const double dt = k[kOffDt];
#pragma unroll
        for (int a = 0; a < N; ++a) {
            const double qdd = a ? r[a] - r[a - 1] : r[0];
            dq[a] = fma(qdd, dt, dq[a]);
            q[a] = fma(dq[a], dt, q[a]);
        }
        angles();
    }
    __device__ __forceinline__ void effector(cdouble* k, double* px, double* py) const {
        double x = 0.0, y = 0.0;
#pragma unroll
        for (int a = 0; a < N; ++a) {
            x = fma(k[kOffFk + a], c[a], x);
            y = fma(k[kOffFk + a], s[a], y);
        }
        *px = x;
        *py = y;
    }
};

// The fused update's median filter runs over windows of kMedRun consecutive steps per thread: thread
// (q, d) = (tid / N, tid % N) takes the windows of t = kMedRun q .. kMedRun q + 3 of column d.
constexpr int kMedRun = 4;
static_assert(kCMax * ((kMaxT + kMedRun - 1) / kMedRun) <= kCT && 2 * kMaxT <= kCT, "one pass of the workgroup");

// This thread's values of the current nominal (cur->u) for chain_update_block, read at kernel entry so their
// latency is hidden
template <int N>
__device__ __forceinline__ void chain_nominal_prefetch(const ChainStep* s, int T, bool on, double (&u4)[kMedRun]) {
    const int q = threadIdx.x / N, d = threadIdx.x - q * N;
#pragma unroll
    for (int j = 0; j < kMedRun; ++j) {
        const int t = kMedRun * q + j;
        u4[j] = (on && t < T) ? s->u[t][d] : 0.0;
    }
}

// Median filter (control.py:319-327) of the T x N weighted noise, u += w_eps
// (control.py:126), shift (control.py:148-149) and the next launch's fp32
// per-step constants.  u4: chain_nominal_prefetch's values.
//
// The four windows of a thread (t - 5 .. t + 4 for t = t0 .. t0 + 3) share the 7 values t0 - 2 .. t0 + 4:
// those are sorted once (16 comparators), and each window's median — scipy's median of 10, the upper one
// (rank 5, as median10) — is the 6th smallest of that sorted A and the window's 3 other values sorted as B:
// min(A5, max(A4, B0), max(A3, B1), max(A2, B2)) (the k-th smallest of two sorted lists is the least
// max(A_i, B_j) over i + j = k).  80 min / max for the four windows against 4 x 58 with median10, and one
// pass of the workgroup instead of four; the same element is selected, so the same bits.
template <int N>
__device__ __forceinline__ void chain_update_block(ChainStep* nxt, const ChainConst& c, CScratch& sm, const double (&u4)[kMedRun]) {
    const int tid = threadIdx.x, T = c.T;
    const int q = tid / N, d = tid - q * N, t0 = kMedRun * q;
    if (t0 < T) {
        double e[13];   // t0 - 5 .. t0 + 7, reflected at both ends (T >= 5: one reflection)
#pragma unroll
        for (int i = 0; i < 13; ++i) {
            int m = t0 - 5 + i;
            m = m < 0 ? -m - 1 : m;
            m = m >= T ? 2 * T - 1 - m : m;
            m = min(max(m, 0), T - 1);   // only windows past T (never written) read a clamped value
            e[i] = sm.weps[m * N + d];
        }
#define CX(v, i, j) { const double lo = min_raw_f64(v[i], v[j]), hi = max_raw_f64(v[i], v[j]); v[i] = lo; v[j] = hi; }
        double A[7] = {e[3], e[4], e[5], e[6], e[7], e[8], e[9]};
        CX(A, 0, 6) CX(A, 2, 3) CX(A, 4, 5) CX(A, 0, 2) CX(A, 1, 4) CX(A, 3, 6) CX(A, 0, 1) CX(A, 2, 5)
        CX(A, 3, 4) CX(A, 1, 2) CX(A, 4, 6) CX(A, 2, 3) CX(A, 4, 5) CX(A, 1, 2) CX(A, 3, 4) CX(A, 5, 6)
#pragma unroll
        for (int j = 0; j < kMedRun; ++j) {
            // window t0 + j: e[j .. j + 9]; besides A, e[j .. 2] and e[10 .. 9 + j]
            double B[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) B[k] = e[j + k < 3 ? j + k : j + k + 7];
            CX(B, 0, 1) CX(B, 1, 2) CX(B, 0, 1)
            const double med = min_raw_f64(min_raw_f64(A[5], max_raw_f64(A[4], B[0])),
                                           min_raw_f64(max_raw_f64(A[3], B[1]), max_raw_f64(A[2], B[2])));
            if (t0 + j < T) sm.unew[(t0 + j) * N + d] = u4[j] + med;
        }
#undef CX
    }
    __syncthreads();
    if (tid < N) nxt->u_first[tid] = sm.unew[tid];
    if (tid == 0) nxt->eta = sm.eta;
    // row t of the shifted nominal and its a_t = (gamma u_t)^T Sigma^-1: two threads a row, in different waves
    // (h wave-uniform), the first taking d < 4
    const int t = tid % kMaxT;
    if (t < T) {
        const int src = t + 1 < T ? t + 1 : T - 1;
        double u[N];
#pragma unroll
        for (int dd = 0; dd < N; ++dd) u[dd] = sm.unew[src * N + dd];
        auto put = [&](int dd) {   // dd a compile-time constant at every call (sig_inv stays in SGPRs)
            nxt->u[t][dd] = u[dd];
            nxt->ua[t][dd] = (float)u[dd];
            double a = 0.0;
#pragma unroll
            for (int e = 0; e < N; ++e) a += (c.gamma * u[e]) * c.sig_inv[e * N + dd];
            nxt->ua[t][kCMax + dd] = (float)a;
            nxt->a[t][dd] = a;
        };
        if (__builtin_amdgcn_readfirstlane(tid) < kMaxT) {
#pragma unroll
            for (int dd = 0; dd < (N < 4 ? N : 4); ++dd) put(dd);
        } else {
#pragma unroll
            for (int dd = 4; dd < N; ++dd) put(dd);
        }
    }
}

// The horizon loop in fp64 (control.py:95-109 with the chain model): returns S
// of sample k.  Window rows in LDS; the nearest slot by the reference's own
// distance ((x - rx)^2 + (y - ry)^2, first minimum, control.py:205-215).
struct alignas(16) WinRowD {
    double x, y, d1, d2;
};
template <int N>
__device__ __forceinline__ double chain_horizon_f64(const ChainConst& c, const ChainStep* st, cdouble* kd,
                                                    const float* noise, int k, float exf, WinRowD* s_wind,
                                                    int* slots) {
    const int tid = threadIdx.x, K = c.K_local, T = c.T;
    if (tid < kSlots) {
        const double* r = st->wind[tid];
        s_wind[tid] = WinRowD{r[0], r[1], r[2], r[3]};
    }
    __syncthreads();
    ChainStateD<N> x;
    x.load(st->x0d);
    cdouble* cu = (cdouble*)&st->u[0][0];
    cdouble* ca = (cdouble*)&st->a[0][0];
    const int W = (int)st->ctr.z;
    double S = 0.0, ex = 0.0, ey = 0.0, e1 = 0.0, e2 = 0.0;
    float nx[N];
#pragma unroll
    for (int d = 0; d < N; ++d) nx[d] = noise[(size_t)k * N + d];
    for (int t = 0; t < T; ++t) {
        double v[N], g = 0.0;
#pragma unroll
        for (int d = 0; d < N; ++d) {
            v[d] = exf != 0.f ? cu[t * kCMax + d] + (double)nx[d] : (double)nx[d];   // control.py:99-101
            g = fma(ca[t * kCMax + d], v[d], g);                                      // control.py:106
        }
        const int tn = t + 1 < T ? t + 1 : t;
#pragma unroll
        for (int d = 0; d < N; ++d) nx[d] = noise[((size_t)tn * K + k) * N + d];
        x.step(v, kd);
        double px, py;
        x.effector(kd, &px, &py);
        int best = 0;
        double dmin = INFINITY;
        for (int j = 0; j < W; ++j) {
            const WinRowD r = s_wind[j];
            const double dx = px - r.x, dy = py - r.y;
            const double d = fma(dx, dx, dy * dy);
            if (d < dmin) {
                dmin = d;
                best = j;
            }
        }
        if (slots) slots[(size_t)k * T + t] = best;   // debug instances only (mppi_chain_debug_slots)
        const WinRowD r = s_wind[best];
        ex = px - r.x;
        ey = py - r.y;
        e1 = x.dq[0] - r.d1;
        e2 = x.dq[1] - r.d2;
        S += fma(kd[kOffSw], ex * ex, fma(kd[kOffSw + 1], ey * ey, fma(kd[kOffSw + 2], e1 * e1, kd[kOffSw + 3] * (e2 * e2)))) + g;
    }
    // terminal cost, control.py:109
    return S + fma(kd[kOffTw], ex * ex, fma(kd[kOffTw + 1], ey * ey, fma(kd[kOffTw + 2], e1 * e1, kd[kOffTw + 3] * (e2 * e2))));
}

// ---------------------------------------------------------------- 4 lanes per sample
//
// When K is too small to give every SIMD a wave (config 5 sharded 8 ways: K =
// 16384 per GPU is 256 waves on 1024 SIMDs), the four lanes of a quad share one
// sample: lane p holds the link pair (2p, 2p+1) — exactly one f32x2 of
// ChainState's representation — and the quad exchanges values with DPP
// quad_perm (one instruction per broadcast or scan step).  Per lane and step:
// one pair's sincos, prefix / suffix sums as 4-lane scans, the rows (2p, 2p+1)
// of D' and of its right-looking L D L^T factorization (each pivot and each
// L[kk][j] broadcast from the lane that owns it, so every lane ends with all of
// L), the forward solve on the pairs with each y_j broadcast, the backward solve
// redundantly from those broadcast values, and 8 of the 30 window slots.
// ~0.52x the instructions per lane of one lane per sample, on 4x the lanes.

// v from lane Q of each quad
template <int Q>
__device__ __forceinline__ float qbc(float v) {
    return dpp_f32<Q * 0x55>(v);   // quad_perm [Q, Q, Q, Q]
}
// sum over the lanes p' < p of the quad (m1 = p >= 1 as 1.f / 0.f): the shift with a zero at lane 0 (its
// own x times 0), then two Hillis-Steele steps whose out-of-range reads land on that 0 — no mask after the
// first step, so every DPP move folds into its v_mul / v_add (v_mul_f32_dpp, v_add_f32_dpp)
__device__ __forceinline__ float q_excl_prefix(float x, float m1) {
#pragma clang fp contract(off)   // a contracted e + dpp(e) would re-read x through an unfolded move
    const float e = dpp_f32<0x90>(x) * m1;   // quad_perm [0, 0, 1, 2]: (0, x0, x1, x2)
    const float f = e + dpp_f32<0x90>(e);    // + e_{p-1}: (0, x0, x0 + x1, x1 + x2)
    return f + dpp_f32<0x40>(f);            // quad_perm [0, 0, 0, 1]: + f_{p-2}
}
// sum over the lanes p' > p of the quad (u1 = p <= 2), the mirror image: the zero sits at lane 3
__device__ __forceinline__ float q_excl_suffix(float x, float u1) {
#pragma clang fp contract(off)
    const float e = dpp_f32<0xF9>(x) * u1;   // quad_perm [1, 2, 3, 3]: (x1, x2, x3, 0)
    const float f = e + dpp_f32<0xF9>(e);    // + e_{p+1}
    return f + dpp_f32<0xFE>(f);            // quad_perm [2, 3, 3, 3]: + f_{p+2}
}
__device__ __forceinline__ float q_sum(float x) {
    x += dpp_f32<0xB1>(x);   // quad_perm xor 1
    return x + dpp_f32<0x4E>(x);
}
__device__ __forceinline__ double q_sum_f64(double x) {
    x += dpp_f64<0xB1>(x);
    return x + dpp_f64<0x4E>(x);
}
template <int J>
__device__ __forceinline__ float elem(f32x2 v) {
    return (J & 1) ? v.y : v.x;
}

// The quad stepped in absolute angles (theta_a = q_1 + ... + q_a, kept in
// revolutions, the unit of v_sin_f32 / v_cos_f32) and their rates: the solve
// gives theta_ddot directly; the joint rates the damping needs are one
// difference (theta_dot of link a0 - 1 from the lane below).  Scheduled for one
// wave per SIMD, where every latency is exposed:
// - D' = L D L^T (unit lower L) instead of Cholesky: 1 / d_j is the rcp of the
//   broadcast pivot, each L entry and each y_j one multiply with its broadcast
//   folded in, and the back solve has no scaling (no square roots, no column
//   scalings, 7 fewer multiplies per step);
// - the state's end effector, window search and LDS row read sit inside the
//   factorization (after column kSearchAt), whose pivot chain leaves issue
//   slots idle; the state's stage cost is taken one step later, when its row
//   has long arrived.  State 0 carries no cost (control.py:95-109), so step 0
//   has no search, and the last state's search follows the loop;
// - noise rows through a buffer resource (the row offset in soffset, the
//   lane's in its VGPR: no 64-bit address arithmetic per step), prefetched two
//   steps ahead; the per-step constants from a 2-deep register ring.
// The stage cost's four terms go to two lanes, two apiece (lane 0 has both joint
// rates of the cost in its own pair), so it needs no broadcast.
template <int N>
__device__ __forceinline__ double chain_horizon_q4(const ChainConst& c, const ChainStep* st, const float* dyn,
                                                   const float* noise, int k, float exf, float4* s_ua4,
                                                   float4* s_win, int* slots, unsigned long long* dbg) {
    static_assert(N <= 8, "four link pairs");
    // the column after which the search is placed: after 2 / 3 / 4 / 5 / 6 measured 77.0 / 76.6 / 77.6 / 75.3 /
    // 77.3 us at K = 16384 (one process, profiles/r13/chain_quad_search_at_ab.txt)
    constexpr int kSearchAt = N > 5 ? 5 : N - 1;
    const int tid = threadIdx.x, sub = tid & 3, K = c.K_local, T = c.T;
    if (tid < kSlots) s_win[tid] = st->win[tid];
    for (int i = tid; i < (T + kQPF) * 4; i += kCT) {
        const int t = min(i >> 2, T - 1), p = i & 3;
        const float* r = st->ua[t];
        s_ua4[i] = make_float4(r[2 * p], r[2 * p + 1], r[kCMax + 2 * p], r[kCMax + 2 * p + 1]);
    }
    Search<4, true> sr;
    sr.load(st->key, st->ctr, sub);
    const int a0 = 2 * sub, a1 = 2 * sub + 1;   // this lane's links
    const float m1 = sub >= 1 ? 1.f : 0.f, u1 = sub <= 2 ? 1.f : 0.f;
    // the stage cost's four terms split over two lanes, two apiece: lane 0 the joint-rate terms (its own
    // theta_dot pair gives q_dot_1, q_dot_2), lane 1 the position terms; lanes 2, 3 weigh theirs by 0
    const bool l0 = sub == 0;
    const f32x2 pad = {a0 < N ? 1.f : 0.f, a1 < N ? 1.f : 0.f};
    const f32x2 l2 = {dyn[kOffL + a0], dyn[kOffL + a1]}, nu2 = {dyn[kOffNu + a0], dyn[kOffNu + a1]};
    const f32x2 damp2 = {dyn[kOffDamp + a0], dyn[kOffDamp + a1]}, fk2 = {dyn[kOffFk + a0], dyn[kOffFk + a1]};
    const float dt = dyn[kOffDt], g = dyn[kOffG];
    constexpr float kRev = 0.15915494309189535f;   // 1 / (2 pi)
    const float dtr = dt * kRev;
    const f32x2 sw2 = l0 ? f32x2{dyn[kOffSw + 2], dyn[kOffSw + 3]}
                         : (sub == 1 ? f32x2{dyn[kOffSw], dyn[kOffSw + 1]} : f32x2{0.f, 0.f});
    const f32x2 tw2 = l0 ? f32x2{dyn[kOffTw + 2], dyn[kOffTw + 3]}
                         : (sub == 1 ? f32x2{dyn[kOffTw], dyn[kOffTw + 1]} : f32x2{0.f, 0.f});
    const float2* const s_win2 = reinterpret_cast<const float2*>(s_win) + (l0 ? 1 : 0);   // (rdq1, rdq2) / (rx, ry)
    // column a of D' on rows (a0, a1): l_a nu_i cos(th_a - th_i) from the broadcast (l c, l s) of link a, plus
    // corr[a]: Dd_a - l_a nu_a on the diagonal (the product gives l_a nu_a there) and -J_{a+1} below it
    f32x2 corr[N];
    {
        const float dc0 = dyn[kOffDd + a0] - l2.x * nu2.x, dc1 = dyn[kOffDd + a1] - l2.y * nu2.y;
        const float j0 = a0 >= 1 ? dyn[kOffJ + 2 * (a0 - 1) + (a0 & 1)] : 0.f;   // -J_{a0} at (a0, a0 - 1)
        const float j1 = dyn[kOffJ + 2 * (a1 - 1) + (a1 & 1)];                    // -J_{a1} at (a1, a1 - 1)
#pragma unroll
        for (int a = 0; a < N; ++a)
            corr[a] = f32x2{a0 == a ? dc0 : (a0 == a + 1 ? j0 : 0.f), a1 == a ? dc1 : (a1 == a + 1 ? j1 : 0.f)};
    }
    // absolute angles (revolutions) and rates of this lane's pair from x0 = (q, q_dot)
    f32x2 TH, THD, C, Sn;
    {
        const f32x2 Q = {a0 < N ? st->x0[a0] : 0.f, a1 < N ? st->x0[a1] : 0.f};
        const f32x2 DQ = {a0 < N ? st->x0[N + a0] : 0.f, a1 < N ? st->x0[N + a1] : 0.f};
        const float tq = Q.x + Q.y, e = q_excl_prefix(tq, m1);
        const float td = DQ.x + DQ.y, ed = q_excl_prefix(td, m1);
        TH = f32x2{e + Q.x, e + tq} * splat(kRev);
        THD = f32x2{ed + DQ.x, ed + td};
    }
    auto angles = [&]() {
        C = f32x2{__builtin_amdgcn_cosf(TH.x), __builtin_amdgcn_cosf(TH.y)};
        Sn = f32x2{__builtin_amdgcn_sinf(TH.x), __builtin_amdgcn_sinf(TH.y)};
    };
    angles();
    // noise of links (a0, a1) at step t: floats (t K + k) N + d; pad links read link N - 1 (masked below);
    // the host keeps T N K 4 below 2^31 for this kernel (mppi_chain_ctx_create)
    const unsigned o0 = (unsigned)(k * N + min(a0, N - 1)) * 4u, o1 = (unsigned)(k * N + min(a1, N - 1)) * 4u;
    const __amdgpu_buffer_rsrc_t nrs = rows_rsrc(noise, T * N * K * 4);
    const int rowb = N * K * 4;
    auto nrow = [&](int t) {
        const int so = min(t, T - 1) * rowb;
        return f32x2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(nrs, (int)o0, so, 0)),
                     __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(nrs, (int)o1, so, 0))};
    };
    f32x2 ring[kQPF];
#pragma unroll
    for (int j = 0; j < kQPF; ++j) ring[j] = nrow(j);
    __syncthreads();
    float4 uar[kQPF];
#pragma unroll
    for (int j = 0; j < kQPF; ++j) uar[j] = s_ua4[j * 4 + sub];

    double S = 0.0;
    f32x2 S2 = {0.f, 0.f};   // this lane's two stage-cost terms
    f32x2 G2 = {0.f, 0.f};   // this lane's (gamma u^T Sigma^-1) v terms
    // the pending stage cost (the previous step's state): this lane's two values and their window-row entries,
    // all zero until the first search, so the cost taken in steps 0 and 1 is exactly 0; (nAB, nrw) this step's
    f32x2 pAB = {0.f, 0.f}, prw = {0.f, 0.f}, nAB = {0.f, 0.f}, nrw = {0.f, 0.f};
    auto search_state = [&](int t, float anchor) {   // the current state (t): end effector, nearest slot, row
        const f32x2 fx = fk2 * C, fy = fk2 * Sn;
        float px = q_sum(fx.x + fx.y), py = q_sum(fy.x + fy.y);
        asm volatile("" : "+v"(px), "+v"(py) : "v"(anchor));   // no earlier than the anchor (and opaque: the
                                                                 // SLP vectoriser would pair the two sums)
        // lane 0: q_dot_1 = theta_dot_1, q_dot_2 = theta_dot_2 - theta_dot_1; the others: the position
        nAB = l0 ? f32x2{THD.x, THD.y - THD.x} : f32x2{px, py};
        const unsigned j = sr.nearest(px, py);
        if (slots && sub == 0) slots[(size_t)k * T + t - 1] = (int)j;   // debug instances only
        const float2 r2 = s_win2[2 * j];
        nrw = f32x2{r2.x, r2.y};
    };
    auto step = [&](int t, auto slot_c, auto srch_c) {
        constexpr int slot = decltype(slot_c)::value;
        constexpr bool srch = decltype(srch_c)::value;
        // the slot's values are taken here (volatile asm keeps its place against the previous step's
        // PIN_LOADS): left free, the scheduler hoists their uses into the previous step, where waiting for
        // them means waiting for every load in flight (as rollout_kernel's dstep)
        f32x2 nz = ring[slot];
        f32x4 ua = {uar[slot].x, uar[slot].y, uar[slot].z, uar[slot].w};
        asm volatile("" : "+v"(nz), "+v"(ua));
        const f32x2 v = __builtin_elementwise_fma(splat(exf), f32x2{ua.x, ua.y}, nz) * pad;  // control.py:99-101
        G2 = __builtin_elementwise_fma(f32x2{ua.z, ua.w}, v, G2);                          // control.py:106
        ring[slot] = nrow(t + kQPF);
        uar[slot] = s_ua4[(t + kQPF) * 4 + sub];
        PIN_LOADS();
        // ---- dynamics in absolute angles: bias, D' rows (a0, a1), L D L^T with the forward solve
        const f32x2 w = THD * THD;   // thdot^2
        const f32x2 lc = l2 * C, ls = l2 * Sn, vc = nu2 * C, vs = nu2 * Sn;
        const f32x2 wvc = w * vc, wvs = w * vs, wlc = w * lc, wls = w * ls;
        const float sC = q_excl_suffix(wvc.x + wvc.y, u1), sS = q_excl_suffix(wvs.x + wvs.y, u1);
        const float pC = q_excl_prefix(wlc.x + wlc.y, m1), pS = q_excl_prefix(wls.x + wls.y, m1);
        const f32x2 Cs = {wvc.y + sC, sC}, Ss = {wvs.y + sS, sS};
        const f32x2 Cp = {pC, wlc.x + pC}, Sp = {pS, wls.x + pS};
        const f32x2 X = __builtin_elementwise_fma(l2, Cs, nu2 * Cp);
        const f32x2 Y = __builtin_elementwise_fma(l2, Ss, nu2 * Sp);
        const float thd_prev = dpp_f32<0x90>(THD.y) * m1;                // theta_dot of link a0 - 1 (0 at the base)
        const f32x2 qd = THD - f32x2{thd_prev, THD.x};                   // joint rates q_dot of (a0, a1)
        const f32x2 ve = __builtin_elementwise_fma(-damp2, qd, v);
        const float ve_next = dpp_f32<0xF9>(ve.x) * u1;                 // link a1 + 1 (0 past the quad)
        f32x2 r = {ve.x - ve.y, ve.y - ve_next};                         // tau
        r = __builtin_elementwise_fma(C, Y, __builtin_elementwise_fma(-Sn, X, __builtin_elementwise_fma(splat(-g), vc, r)));
        f32x2 col[N];
        unroll_seq([&](auto a_c) {
            constexpr int a = decltype(a_c)::value;
            const float la = qbc<a / 2>(elem<a>(lc)), sa = qbc<a / 2>(elem<a>(ls));
            col[a] = __builtin_elementwise_fma(splat(la), vc, __builtin_elementwise_fma(splat(sa), vs, corr[a]));
        }, std::make_integer_sequence<int, N>{});
        // right-looking on the raw columns, every factor kept negated: -1 / d_j is the rcp of the negated
        // broadcast pivot (a source modifier of the DPP form), -L[kk][j] and -y_j are the broadcast entries
        // times it, so no product needs a negation that would take it out of the VOP2 encoding the broadcast
        // folds into; every lane keeps every -L[kk][j] and -y_j (y = D^-1 L^-1 r: the back solve needs no
        // scaling)
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
                    // the last row's products, left free, are paired by the SLP vectoriser into a v_pk_mul_f32,
                    // which has no DPP form: their broadcasts come back as separate moves (7 per step)
                    if constexpr (kk == N - 1) asm volatile("" : "+v"(Ln[kk][j]));
                    col[kk] = __builtin_elementwise_fma(splat(Ln[kk][j]), col[j], col[kk]);
                }
            }, std::make_integer_sequence<int, N>{});
            if constexpr (srch && j == kSearchAt) search_state(t, nrd);
        }, std::make_integer_sequence<int, N>{});
        float x[N];   // L^T x = y: theta_ddot, redundantly in every lane; the oldest x first
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
        THD = __builtin_elementwise_fma(f32x2{xa, xb}, splat(dt), THD);  // semi-implicit Euler (chain_oracle.py)
        TH = __builtin_elementwise_fma(THD, splat(dtr), TH);
        angles();
        {   // the pending (previous state's) stage cost, control.py:174-185; the row is taken only now (the
            // asm needs TH, this step's last dynamics result)
            f32x2 rw = prw;
            asm volatile("" : "+v"(rw) : "v"(TH));
            const f32x2 e = pAB - rw;
            S2 = __builtin_elementwise_fma(sw2, e * e, S2);
        }
        if constexpr (srch) {
            pAB = nAB;
            prw = nrw;
        }
        if constexpr (slot == kQPF - 1) {
            S += (double)((S2.x + S2.y) + (G2.x + G2.y));
            S2 = f32x2{0.f, 0.f};
            G2 = f32x2{0.f, 0.f};
        }
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using Y = std::true_type;
    STAMP(12, NOW());   // stamp builds: the prologue's end, then the first steps and the horizon's middle
    step(0, I0{}, std::false_type{});
    int t = 1;
    if constexpr (kQPF == 2) {
        for (; t + 2 <= T; t += 2) {
            step(t, I1{}, Y{});
            step(t + 1, I0{}, Y{});
        }
        if (t < T) step(t, I1{}, Y{});
    } else {
        static_assert(kQPF == 4, "a 2- or 4-deep ring");
        for (; t + 4 <= T; t += 4) {   // slots 1, 2, 3, 0
            step(t, I1{}, Y{});
            step(t + 1, I2{}, Y{});
            step(t + 2, I3{}, Y{});
            step(t + 3, I0{}, Y{});
#ifdef MPPI_STAMPS
            if (t == 1) STAMP(13, NOW());
            if (t + 4 == T / 2 + 1) STAMP(14, NOW());
#endif
        }
        if (t < T) step(t, I1{}, Y{});   // remainder: slots 1, 2, 3 in order
        if (t + 1 < T) step(t + 1, I2{}, Y{});
        if (t + 2 < T) step(t + 2, I3{}, Y{});
    }
    {   // state T - 1's pending cost, then the last state's search: its stage and terminal cost
        // (control.py:106-109) on the same state
        const f32x2 e = pAB - prw;
        S2 = __builtin_elementwise_fma(sw2, e * e, S2);
    }
    search_state(T, TH.x);
    const f32x2 e = nAB - nrw, ee = e * e;
    S2 = __builtin_elementwise_fma(sw2, ee, S2);
    S += (double)((S2.x + S2.y) + (G2.x + G2.y));
    const f32x2 te = tw2 * ee;
    S += (double)(te.x + te.y);
    return q_sum_f64(S);
}

// POLL / counter hand-off and the merges as in rollout_kernel (mppi_rocm.hip).
// SLOTS (debug instances, mppi_chain_debug_slots): dbg receives the window slot
// each sample picked at each step, int32 [k][t].
template <int N, bool POLL, bool F64, int LPS, bool SLOTS = false>
__global__ __launch_bounds__(kCT) __attribute__((amdgpu_waves_per_eu(2, 2))) void chain_rollout_kernel(
    const ChainConst c, const ChainStep* __restrict__ st, const float* __restrict__ dyn,
    const float* __restrict__ noise, double* __restrict__ S_out, double* __restrict__ slab, double* __restrict__ gslab,
    unsigned* __restrict__ counters, double* __restrict__ partial_out, double* __restrict__ w_eps_out,
    ChainStep* __restrict__ nxt, unsigned flags, const XDesc xd, unsigned* __restrict__ epoch, unsigned* __restrict__ tmo,
    unsigned long long* __restrict__ runmin, unsigned long long* __restrict__ dbg) {
    static_assert(N <= kCMax && N >= 2, "links");
    __shared__ float4 s_win[kSlots];
    __shared__ KeyPair s_keys[kKeyPairs];
    __shared__ WinRowD s_wind[F64 ? kSlots : 1];
    __shared__ float4 s_ua4[LPS == 4 ? (kMaxT + kQPF) * 4 : 1];
    __shared__ double s_redd[kCT / 64];
    __shared__ int s_cnt[kCT / 64];
    __shared__ int s_k[kCT];
    __shared__ double s_e[kCT];
    __shared__ unsigned s_flag, s_parity;
    __shared__ double s_run;
    __shared__ CScratch sm;

    static_assert(LPS == 1 || (LPS == 4 && !F64), "lanes per sample: 1, or 4 for the fp32 rollout");
    constexpr int NS = kCT / LPS;   // samples per workgroup
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k_raw = (blockIdx.x * kCT + tid) / LPS;
    if (c.fair) draw_cu_ticket(counters + c.cu_off, &s_parity);
    const bool valid = k_raw < c.K_local;
    const bool owner = valid && (tid & (LPS - 1)) == 0;   // the lane that stands for its sample
    const int k = valid ? k_raw : c.K_local - 1;
    const float exf = (c.k_offset + k) < c.k_exploit ? 1.f : 0.f;  // control.py:98-101
    const int K = c.K_local, T = c.T;
    int* const slots = SLOTS ? reinterpret_cast<int*>(dbg) : nullptr;

    STAMP(0, NOW());
#ifdef MPPI_STAMPS
    STAMP(8, (unsigned long long)__builtin_amdgcn_s_getreg(0xF804));   // HW_ID
    STAMP(9, (unsigned long long)__builtin_amdgcn_s_getreg(0xF814));   // XCC_ID
#endif
    // poll tags are never 0 (fresh memory)
    unsigned tag_v = POLL ? __hip_atomic_load(epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u : 0u;
    if (POLL && tag_v == 0u) tag_v = 1u;
    double u_cur[kMedRun];
    chain_nominal_prefetch<N>(st, T, flags & MPPI_FLAG_FUSED_UPDATE, u_cur);
    double S = 0.0;
    if constexpr (F64) {
        S = chain_horizon_f64<N>(c, st, (cdouble*)(dyn + kDynF64Off), noise, k, exf, s_wind, slots);
    } else if constexpr (LPS == 4) {
        S = chain_horizon_q4<N>(c, st, dyn, noise, k, exf, s_ua4, s_win, slots, dbg);
    } else {
    if (tid < kSlots) s_win[tid] = st->win[tid];
    // window keys in LDS (broadcast reads): the 90 key registers would cost the
    // chain kernel its second wave per SIMD; precise keys: the config-5 start
    // pose sits on a waypoint
    SearchLDS<true>::fill(s_keys, st->key, tid);
    SearchLDS<true> sr{s_keys, st->ctr.x, st->ctr.y};
    ChainState<N> x;
    x.load(st->x0);
    // noise (t, d) of sample k: noise[(t K + k) N + d] (a sample's N values of a step contiguous); prefetches
    // past the last step read step T - 1 again (never used)
    // (uniform step base + a 32-bit lane byte offset: the saddr form of global_load)
    const unsigned kb = (unsigned)k * (unsigned)N * 4u;
    auto nrow = [&](int t, int d) {
        const char* row = (const char*)(noise + (size_t)min(t, T - 1) * K * N + d);
        return *(const float*)(row + kb);
    };
    cfloat* cua = (cfloat*)(&st->ua[0][0]);
    float ring[kCPF][N];
    float uring[kCPU][2 * N];
#pragma unroll
    for (int j = 0; j < kCPF; ++j)
#pragma unroll
        for (int d = 0; d < N; ++d) ring[j][d] = nrow(j, d);
#pragma unroll
    for (int j = 0; j < kCPU; ++j)
#pragma unroll
        for (int d = 0; d < 2 * N; ++d) uring[j][d] = cua[j * 2 * kCMax + (d < N ? d : kCMax + d - N)];
    __syncthreads();

    const DynMem kd{(cfloat*)dyn};
    // Horizon loop (control.py:95-109 with the chain model), S in fp64.
    float S4 = 0.f;
    float ex = 0.f, ey = 0.f, e1 = 0.f, e2 = 0.f;
    auto step = [&](int t, auto i_c) {
        constexpr int i = decltype(i_c)::value;
        float v[N];
        float g = 0.f;
#pragma unroll
        for (int d = 0; d < N; ++d) {
            v[d] = fmaf(exf, uring[i % kCPU][d], ring[i % kCPF][d]);   // u_t + eps or eps
            g = fmaf(uring[i % kCPU][N + d], v[d], g);                 // (gamma u_t^T Sigma^-1) v, control.py:106
        }
#pragma unroll
        for (int d = 0; d < N; ++d) ring[i % kCPF][d] = nrow(t + kCPF, d);
#pragma unroll
        for (int d = 0; d < 2 * N; ++d)
            uring[i % kCPU][d] = cua[(t + kCPU) * 2 * kCMax + (d < N ? d : kCMax + d - N)];
        PIN_LOADS();
        x.step(v, kd);
        float px, py;
        x.effector(kd, &px, &py);
        const unsigned j = sr.nearest(px, py);
        if constexpr (SLOTS) slots[(size_t)k * T + t] = (int)j;
        const float4 r = s_win[j];
        ex = px - r.x;
        ey = py - r.y;
        e1 = x.dqa(0) - r.z;
        e2 = x.dqa(1) - r.w;
        const float sw[4] = {kd.p[kOffSw], kd.p[kOffSw + 1], kd.p[kOffSw + 2], kd.p[kOffSw + 3]};   // control.py:185
        S4 += weighted_sq(ex, ey, e1, e2, sw) + g;
        if constexpr ((i & 3) == 3) {
            S += (double)S4;
            S4 = 0.f;
        }
    };
    int t = 0;
    const unsigned parity = c.fair ? __builtin_amdgcn_readfirstlane(s_parity) : 2u;
    for (; t + 4 <= T; t += 4) {
        if (parity < 2u) fair_priority(parity);
        unroll_seq([&](auto i_c) { step(t + decltype(i_c)::value, i_c); }, std::make_integer_sequence<int, 4>{});
    }
    unroll_seq([&](auto i_c) {
        if (t + decltype(i_c)::value < T) step(t + decltype(i_c)::value, i_c);
    }, std::make_integer_sequence<int, 3>{});
    S += (double)S4;
    S += (double)weighted_sq(ex, ey, e1, e2, c.dyn + kOffTw);  // terminal cost, control.py:109
    }

    STAMP(1, NOW());
    if (S_out && owner) S_out[k] = S;

    // ---- workgroup partial: rho_b, eta_b, N_b (control.py:112-118 over this block)
    // With a quad per sample (one workgroup per CU, every workgroup finishing at once) the running minimum
    // (below) is read before the block minimum, so its round trip runs under it, and the workgroup's own
    // atomic goes out after the last barrier, unwaited; with one lane per sample (two workgroups per CU,
    // finishing spread out) the atomic's fresher return skips more gathers (measured: +1.7 % with the early
    // read at config 5, -1.7 % at its shard)
    constexpr bool kEarlyRun = LPS == 4;
    unsigned long long run0 = ~0ull;
    if (kEarlyRun && tid == 0) run0 = __hip_atomic_load(runmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double rho_b = block_min_f64<kCT>(owner ? S : INFINITY, sm);
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
    // The running minimum of the workgroups' rho_b (one 64-bit atomic min per
    // workgroup on an order-preserving key; reset by the final merger).  The final
    // rho is at most any minimum over published rho_b, so a workgroup whose rho_b
    // is 2^-64 or more below it in weight can carry no weight in any merge: it
    // publishes rho_b = +inf and skips the gather of its weighted samples' noise —
    // each of those is T n scattered 4-B reads, one cache line apiece (1.14x the
    // algorithmic bytes at config 5).
    if (tid == 0) {
        const unsigned long long key = ord_key(rho_b);
        unsigned long long run;
        if constexpr (kEarlyRun) {
            run = min(run0, key);
        } else {
            const unsigned long long old = __hip_atomic_fetch_min(runmin, key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            run = old < key ? old : key;
        }
        s_run = ord_val(run);
    }
    __syncthreads();
    const bool skip = exp((s_run - rho_b) * c.inv_lambda) < kMergeFloor;   // uniform
    int off = 0, nl = 0;
    double eta_b = 0.0;
#pragma unroll
    for (int w = 0; w < kCT / 64; ++w) {
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
    // past the barriers (a barrier's fence would wait for the atomic to complete): fire and forget; the
    // gather's loads, issued after it, return after it anyway
    if (kEarlyRun && tid == 0) __hip_atomic_fetch_min(runmin, ord_key(rho_b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nval = T * N;
    const RowGeo geo(nval);
    const int stride = geo.stride;
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
    // rho_b and eta_b leave first (see rollout_kernel in mppi_rocm.hip)
    nl = __builtin_amdgcn_readfirstlane(nl);
    if (tid == 0) {
        publish(blockIdx.x * stride, skip ? INFINITY : rho_b);
        publish(blockIdx.x * stride + 1, eta_b);
    }
    if (skip) {
        // no merge reads this row past rho
    } else if (nl <= kSparseMax) {
        // column (t, d) = t N + d of the noise: sample k's value at noise[(t K + k) N + d]
        for (int col = tid; col < nval; col += kCT) {
            const int tt = col / N;
            const float* base = noise + (size_t)tt * K * N + (col - tt * N);
            publish(blockIdx.x * stride + 2 + col, gather_col(base, N, s_k, s_e, nl));
        }
    } else {
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
        for (int cb = wave * kRowBatch; cb < nval; cb += (kCT / 64) * kRowBatch) {
            float e[kRowBatch][PER];
#pragma unroll
            for (int r = 0; r < kRowBatch; ++r) {
                const int cr = min(cb + r, nval - 1);
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int tt = cr / N;
                    e[r][i] = noise[((size_t)tt * K + min(k0 + lane + 64 * i, K - 1)) * N + (cr - tt * N)];
                }
            }
#pragma unroll
            for (int r = 0; r < kRowBatch; ++r) {
                double a = 0.0;
#pragma unroll
                for (int i = 0; i < PER; ++i) a = fma(w[i], (double)e[r][i], a);
                a = wave_sum_f64(a);
                if (lane == 0 && cb + r < nval) publish(blockIdx.x * stride + 2 + cb + r, a);
            }
        }
    }
    STAMP(2, NOW());
    STAMP(5, (unsigned long long)nl);
    const int g = blockIdx.x / kGroup;
    const int gsz = min(kGroup, nrows - g * kGroup);
    if constexpr (POLL) {
        if ((int)blockIdx.x != g * kGroup) return;
        STAMP(3, NOW());
        if (ngroups == 1) {
            merge_rows_block<kCT, kCMaxCh, true, true>(slab_r, 0, gsz, geo, c.inv_lambda, sm, nullptr, 0, partial_out,
                                                       w_eps_out, tag, tmo);
        } else if (blockIdx.x == 0 && nrows <= kDirectRows &&
                   direct_merge<kCT, kCMaxCh, true>(slab_r, nrows, geo, c.inv_lambda, sm, partial_out, w_eps_out, tag,
                                                    tmo)) {
        } else {
            merge_rows_block<kCT, kCMaxCh, false, true>(slab_r, g * kGroup, gsz, geo, c.inv_lambda, sm, &gslab_r, g,
                                                        nullptr, nullptr, tag, tmo);
            STAMP(10, NOW());
            if (blockIdx.x != 0) return;
            STAMP(4, NOW());
            merge_rows_block<kCT, kCMaxCh, true, true>(gslab_r, 0, ngroups, geo, c.inv_lambda, sm, nullptr, 0,
                                                       partial_out, w_eps_out, tag, tmo);
        }
        if (threadIdx.x == 0) {
            __hip_atomic_store(epoch, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(runmin, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // every row is in
        }
    } else {
        if (!arrive_last(counters + g, (unsigned)gsz, &s_flag, c.acquire != 0)) return;
        STAMP(3, NOW());
        merge_rows_block<kCT, kCMaxCh, false, false>(slab_r, g * kGroup, gsz, geo, c.inv_lambda, sm, &gslab_r, g,
                                                     nullptr, nullptr, 0u, nullptr);
        STAMP(10, NOW());
        if (!arrive_last(counters + ngroups, (unsigned)ngroups, &s_flag, c.acquire != 0)) return;
        STAMP(4, NOW());
        if (!(ngroups > 1 && nrows <= kDirectRows &&
              direct_merge<kCT, kCMaxCh, false>(slab_r, nrows, geo, c.inv_lambda, sm, partial_out, w_eps_out, 0u,
                                                nullptr)))
            merge_rows_block<kCT, kCMaxCh, true, false>(gslab_r, 0, ngroups, geo, c.inv_lambda, sm, nullptr, 0,
                                                        partial_out, w_eps_out, 0u, nullptr);
        if (threadIdx.x == 0) __hip_atomic_store(runmin, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    STAMP(11, NOW());
    STAMP(6, (unsigned long long)sm.nrel);
    // with the exchange, the update is computed while the ranks' statuses travel: it lands in the ping-pong
    // block the host makes current only after a good verdict (on failure the host keeps its block)
    const unsigned xtag = (flags & MPPI_FLAG_EXCHANGE)
                              ? exchange_send_merge<kCT, kCMaxCh>(xd, geo, c.inv_lambda, sm, w_eps_out, tmo) : 0u;
    if (tid == 0 && w_eps_out) w_eps_out[nval] = sm.eta;   // the weights' spread (mppi_chain_last_eta)
    if (flags & MPPI_FLAG_FUSED_UPDATE) chain_update_block<N>(nxt, c, sm, u_cur);
    if (flags & MPPI_FLAG_EXCHANGE) exchange_verdict<kCT>(xd, geo, xtag, tmo);
    STAMP(7, NOW());
}

// Merge of the all-gathered per-device rows (multi-GPU), plus the fused update.
template <int N>
__global__ __launch_bounds__(kCT) void chain_merge_kernel(const ChainConst c, const ChainStep* cur, const double* parts,
                                                          int n, double* w_eps_out, ChainStep* nxt, unsigned flags) {
    __shared__ CScratch sm;
    const int tid = threadIdx.x, T = c.T;
    double u_cur[kMedRun];
    chain_nominal_prefetch<N>(cur, T, flags & MPPI_FLAG_FUSED_UPDATE, u_cur);
    const RowGeo geo(T * N);
    const __amdgpu_buffer_rsrc_t r = rows_rsrc(parts, n * geo.stride * 8);
    merge_rows_block<kCT, kCMaxCh, true, false>(r, 0, n, geo, c.inv_lambda, sm, nullptr, 0, nullptr, w_eps_out, 0u,
                                                nullptr);
    if (tid == 0 && w_eps_out) w_eps_out[T * N] = sm.eta;
    if (flags & MPPI_FLAG_FUSED_UPDATE) chain_update_block<N>(nxt, c, sm, u_cur);
}

// Trajectory re-roll (control.py:129-145 with the chain): control(t) =
// base[(t-1) mod T] (+ eps); out[k][t][2N] = (q, dq) after step t.  As in
// traj_kernel, the states of kChainTB steps go through an LDS tile and each
// flush writes every sample's kChainTB * 2N floats as one contiguous run.
constexpr int kChainTB = 2;
template <int N, bool NOISE>
__global__ __launch_bounds__(kCT) void chain_traj_kernel(const ChainConst c, const ChainStep* __restrict__ st,
                                                         const float* __restrict__ base,
                                                         const float* __restrict__ noise, int Kn,
                                                         float* __restrict__ out) {
    constexpr int W = 2 * N;   // floats per state
    __shared__ float tile[kChainTB][W][kCT];
    const int tid = threadIdx.x;
    const int k0 = blockIdx.x * kCT;
    const int k = min(k0 + tid, Kn - 1);   // lanes past Kn recompute the last sample, never stored
    const int nk = min(kCT, Kn - k0);
    const int T = c.T;
    const float exf = NOISE ? ((c.k_offset + k) < c.k_exploit ? 1.f : 0.f) : 1.f;
    ChainState<N> x;
    x.load(st->x0);
    // a tile's noise is loaded one tile ahead (see traj_kernel)
    auto load_tile = [&](int t0, float (&e)[kChainTB][N]) {
#pragma unroll
        for (int j = 0; j < kChainTB; ++j) {
            const int t = min(t0 + j, T - 1);
            const int ti = t == 0 ? T - 1 : t - 1;
#pragma unroll
            for (int d = 0; d < N; ++d) e[j][d] = NOISE ? noise[((size_t)ti * c.K_local + k) * N + d] : 0.f;
        }
    };
    float cur[kChainTB][N];
    load_tile(0, cur);
    for (int t0 = 0; t0 < T; t0 += kChainTB) {
        const int nt = min(kChainTB, T - t0);
        float nxt[kChainTB][N];
        load_tile(t0 + kChainTB, nxt);
#pragma unroll
        for (int j = 0; j < kChainTB; ++j) {
            if (j >= nt) break;
            const int t = t0 + j;
            const int ti = t == 0 ? T - 1 : t - 1;
            float v[N];
#pragma unroll
            for (int d = 0; d < N; ++d) {
                v[d] = base[ti * N + d];
                if (NOISE) v[d] = fmaf(exf, v[d], cur[j][d]);
            }
            x.step(v, DynArg{c.dyn});
#pragma unroll
            for (int a = 0; a < N; ++a) {
                tile[j][a][tid] = x.qa(a);
                tile[j][N + a][tid] = x.dqa(a);
            }
        }
        __syncthreads();
        const int run = nt * W;   // floats of one sample in this flush
        for (int i = tid; i < nk * run; i += kCT) {
            const int s = i / run, r = i - s * run;
            out[((size_t)(k0 + s) * T + t0) * W + r] = tile[r / W][r % W][s];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kChainTB; ++j)
#pragma unroll
            for (int d = 0; d < N; ++d) cur[j][d] = nxt[j][d];
    }
}

// eps[t][k][d] = (L z)_d, z ~ N(0, I) from Philox4x32-10 counters (global k, t,
// call) + Box-Muller: a shard generates exactly its slice of the unsharded draw.
// The factor travels by value (kernel argument, scalar loads) and the link count
// is a template argument, so the matvec unrolls and z stays in registers (a
// runtime-n loop indexed z dynamically and sent it to scratch: 504 us at config 5).
struct CholArg {
    float L[kCMax * kCMax];   // lower triangle, row-major, x kBoxMullerScale (box_muller's constant)
};
template <int N>
__global__ __launch_bounds__(kCT) void chain_philox_kernel(int K_local, int T, long long k_offset,
                                                           unsigned long long seed, unsigned long long step,
                                                           const CholArg Lc, float* __restrict__ out) {
    // grid (ceil(K_local / kCT), T): no 64-bit divide per thread
    const int k = (int)blockIdx.x * kCT + (int)threadIdx.x;
    if (k >= K_local) return;
    const int t = (int)blockIdx.y;
    const unsigned long long kg = (unsigned long long)(k_offset + k);
    const uint2 key = make_uint2((unsigned)seed, (unsigned)(seed >> 32) ^ (unsigned)(step >> 32));
    float z[kCMax];
#pragma unroll
    for (int call = 0; call < kCMax / 4; ++call) {
        const uint4 ctr = make_uint4((unsigned)kg, (unsigned)(kg >> 32), (unsigned)(t * 4 + call), (unsigned)step);
        const uint4 r = philox4x32_10(ctr, key);
        const float2 a = box_muller(r.x, r.y), b = box_muller(r.z, r.w);
        z[4 * call] = a.x;
        z[4 * call + 1] = a.y;
        z[4 * call + 2] = b.x;
        z[4 * call + 3] = b.y;
    }
    float* row = out + ((size_t)t * K_local + k) * N;
#pragma unroll
    for (int d = 0; d < N; ++d) {
        float e = 0.f;
#pragma unroll
        for (int j = 0; j <= d; ++j) e = fmaf(Lc.L[d * kCMax + j], z[j], e);
        row[d] = e;
    }
}

}  // namespace

// ================================================================ host side

struct mppi_chain_ctx {
    mppi_chain_config cfg;
    int device = 0, n = 0;
    hipStream_t stream = nullptr;
    int nblocks = 0;
    bool poll = false;
    ChainConst kc;
    ChainStep* d_step = nullptr;   // [2] ping-pong
    int cur = 0;
    ChainStep* h_step = nullptr;   // pinned staging
    hipEvent_t staged = nullptr;
    double* d_slab = nullptr;
    double* d_gslab = nullptr;
    unsigned* d_counter = nullptr;
    unsigned* d_epoch = nullptr;
    unsigned long long* d_runmin = nullptr;   // running minimum of the workgroups' rho_b (ord_key), ~0 between launches
    double* d_weps = nullptr;
    double* h_buf = nullptr;
    float* d_base = nullptr;
    float* h_base = nullptr;
    CholArg chol{};                // Cholesky factor of Sigma x kBoxMullerScale (kCMax x kCMax, fp32) for the Philox noise
    float* d_dyn = nullptr;        // packed per-step constants (DynMem), then the same in fp64 at kDynF64Off
    double h_dynd[kCDyn] = {};     // the fp64 constants on the host (the optimal trajectory)
    bool upd_valid = false;        // the current step block holds a fused update's output
    bool pub_valid = false;        // ... and h_pub is its shifted nominal as mppi_chain_wait_outputs returned it
    double* h_out = nullptr;       // MPPI_FLAG_HOST_OUT: the update's read-back, queued right behind the launch
    hipEvent_t out_ev = nullptr;   // ... recorded after that copy
    bool out_posted = false;
    bool x_flipped = false;        // the last launch flipped the ping-pong and exchanged (undone on MPPI_E_EXCHANGE)
    double last_eta = NAN;         // the weights' spread of the last update / weighted noise read back
    double h_pub[kCMaxVals] = {};
    bool f64 = false;              // cfg.precision == 1
    int lps = 1;                   // lanes per sample: 1, or 4 (fp32 rollout at small K)
    unsigned* h_tmo = nullptr;
    unsigned* d_tmo = nullptr;
    unsigned long long* d_dbg = nullptr;
    // node-level exchange (mppi_chain_exchange_*), as in mppi_ctx
    XDesc xd{};
    void* d_inbox = nullptr;
    double* d_xrow = nullptr;
    unsigned* d_xepoch = nullptr;
    int xworld_alloc = 0;
    void* xopened[kMaxWorld] = {};
};

namespace {

using mppi_host::exchange_timeout_ticks;
using mppi_host::fail;

template <int N, bool P, bool F64, int LPS>
void launch_rollout(mppi_chain_ctx* c, const ChainStep* cur, const float* noise, double* S, double* part, ChainStep* nxt,
                    unsigned flags, int* slots = nullptr) {
    if (slots) {   // the debug instance: identical arithmetic, plus the slot stores
        if constexpr (N == kCDebugN)
            hipLaunchKernelGGL((chain_rollout_kernel<N, P, F64, LPS, true>), dim3(c->nblocks), dim3(kCT), 0, c->stream, c->kc,
                               cur, c->d_dyn, noise, S, c->d_slab, c->d_gslab, c->d_counter, part, c->d_weps, nxt, flags,
                               c->xd, c->d_epoch, c->d_tmo, c->d_runmin, reinterpret_cast<unsigned long long*>(slots));
        return;
    }
    hipLaunchKernelGGL((chain_rollout_kernel<N, P, F64, LPS>), dim3(c->nblocks), dim3(kCT), 0, c->stream, c->kc, cur, c->d_dyn,
                       noise, S, c->d_slab, c->d_gslab, c->d_counter, part, c->d_weps, nxt, flags, c->xd, c->d_epoch, c->d_tmo,
                       c->d_runmin, c->d_dbg);
}

// the link counts with an instantiated kernel
#define MPPI_CHAIN_DISPATCH(n, F) \
    switch (n) {                  \
        case 2: F(2); break;      \
        case 3: F(3); break;      \
        case 4: F(4); break;      \
        case 5: F(5); break;      \
        case 6: F(6); break;      \
        case 7: F(7); break;      \
        default: break;           \
    }

// Lanes per sample of the fp32 rollout: 4 while one lane per sample would leave
// SIMDs without a wave (K <= 32768: at most 512 waves of 64 samples on 1024 SIMDs);
// measured in DESIGN §3b.  The fp64 rollout keeps one lane per sample.
int chain_auto_lps(int K_local, bool f64) {
    if (f64) return 1;
    return K_local <= 32768 ? 4 : 1;
}

int check_tmo(mppi_chain_ctx* c) {
    // tmo[0]: a local hand-off gave up (kTmoLocal); tmo[1]: the exchange's verdict bits (mppi_device.h)
    const unsigned v = c->h_tmo ? __atomic_load_n(c->h_tmo, __ATOMIC_ACQUIRE) | __atomic_load_n(c->h_tmo + 1, __ATOMIC_ACQUIRE)
                                : 0u;
    if (!v) return MPPI_OK;
    c->h_tmo[0] = c->h_tmo[1] = 0;
    if (v == kTmoExchange) {   // as the 2-link engine's check_timeout: the nominal before the launch
        if (c->x_flipped) c->cur ^= 1;
        c->x_flipped = false;
        c->upd_valid = false;
        c->pub_valid = false;
        c->out_posted = false;
        return fail(MPPI_E_EXCHANGE, "multi-GPU exchange: a rank's row did not arrive within the bound on every "
                                     "rank of this step; no rank applied the update (run the step again)");
    }
    // an aborted merge left the running minimum set: clear it for the next launch
    if (v & kTmoLocal) (void)hipMemsetAsync(c->d_runmin, 0xFF, sizeof(unsigned long long), c->stream);
    if (v & kTmoSplit)
        return fail(MPPI_E_HIP, "multi-GPU exchange: this rank had every row but not every rank's verdict within "
                                "the bound; other ranks may have applied the step, so it cannot be re-run");
    return fail(MPPI_E_HIP, "in-launch hand-off timed out (workgroups not co-resident?); results invalid");
}

}  // namespace

extern "C" {

void mppi_chain_config_init(mppi_chain_config* cfg) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->param_gamma = NAN;   // lambda (1 - alpha), control.py:45
    cfg->chain.g = 9.81;      // sys_params.py:13
}

int mppi_chain_ctx_create(const mppi_chain_config* cfg, int device, void* stream, mppi_chain_ctx** out) {
    if (!cfg || !out) return fail(MPPI_E_ARG, "null argument");
    *out = nullptr;
    const int n = cfg->chain.n;
    if (n < 2 || n > 7) return fail(MPPI_E_ARG, "chain.n must be in [2, 7]");
    if (cfg->T < 1 || cfg->T > MPPI_MAX_T) return fail(MPPI_E_ARG, "T must be in [1, 128]");
    if (cfg->T * n + 1 > kCMaxCh * kCT) return fail(MPPI_E_ARG, "T * n too large");
    if (cfg->precision != 0 && cfg->precision != 1) return fail(MPPI_E_ARG, "precision must be 0 (fp32) or 1 (fp64)");
    if (cfg->K_local < 1 || cfg->K_total < cfg->K_local || cfg->k_offset < 0 ||
        cfg->k_offset + (long long)cfg->K_local > cfg->K_total)
        return fail(MPPI_E_ARG, "bad sample geometry (K_local, K_total, k_offset)");
    if ((long long)cfg->K_local * cfg->T * n >= (1LL << 31)) return fail(MPPI_E_ARG, "too many samples");
    // Sigma: symmetric positive definite (Cholesky), inverse for the control cost
    double Lc[kCMax][kCMax] = {}, Si[kCMax * kCMax] = {};
    {
        const double* S = cfg->sigma;
        for (int j = 0; j < n; ++j) {
            double d = S[j * n + j];
            for (int q = 0; q < j; ++q) d -= Lc[j][q] * Lc[j][q];
            if (!(d > 0.0) || !isfinite(d)) return fail(MPPI_E_SINGULAR, "Sigma is not positive definite");
            Lc[j][j] = sqrt(d);
            for (int i = j + 1; i < n; ++i) {
                double e = 0.5 * (S[i * n + j] + S[j * n + i]);
                for (int q = 0; q < j; ++q) e -= Lc[i][q] * Lc[j][q];
                Lc[i][j] = e / Lc[j][j];
            }
        }
        for (int col = 0; col < n; ++col) {   // Sigma^-1 = L^-T L^-1, column by column
            double y[kCMax] = {};
            for (int i = 0; i < n; ++i) {
                double e = i == col ? 1.0 : 0.0;
                for (int q = 0; q < i; ++q) e -= Lc[i][q] * y[q];
                y[i] = e / Lc[i][i];
            }
            for (int i = n - 1; i >= 0; --i) {
                double e = y[i];
                for (int q = i + 1; q < n; ++q) e -= Lc[q][i] * y[q];
                y[i] = e / Lc[i][i];
            }
            for (int i = 0; i < n; ++i) Si[i * n + col] = y[i];
        }
    }
    mppi_chain_ctx* c = new mppi_chain_ctx();
    c->cfg = *cfg;
    c->device = device;
    c->n = n;
    c->stream = (hipStream_t)stream;
    c->f64 = cfg->precision == 1;
    c->lps = cfg->lanes_per_sample > 0 ? cfg->lanes_per_sample : chain_auto_lps(cfg->K_local, c->f64);
    if (c->lps != 1 && c->lps != 4) {
        delete c;
        return fail(MPPI_E_ARG, "lanes_per_sample must be 0 (auto), 1 or 4");
    }
    if (c->lps == 4 && c->f64) {
        delete c;
        return fail(MPPI_E_ARG, "lanes_per_sample 4 is for the fp32 rollout");
    }
    if (c->lps == 4 && (long long)cfg->K_local * cfg->T * n * 4 >= (1LL << 31)) {   // its noise buffer offsets
        if (cfg->lanes_per_sample > 0) {
            delete c;
            return fail(MPPI_E_ARG, "lanes_per_sample 4 needs K_local * T * n * 4 below 2^31 bytes of noise");
        }
        c->lps = 1;
    }
    c->nblocks = (int)(((long long)cfg->K_local * c->lps + kCT - 1) / kCT);
    ChainConst& k = c->kc;
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
    k.n = n;
    const mppi_chain_params& P = cfg->chain;
    float* dyn = k.dyn;
    for (int a = 0; a < kCMax; ++a) dyn[kOffDd + a] = 1.f;   // pad rows
    for (int a = 0; a < n; ++a) {
        double tail = 0.0;
        for (int q = a + 1; q < n; ++q) tail += P.m[q];
        const double mu_aa = P.m[a] * P.lc[a] * P.lc[a] + P.l[a] * P.l[a] * tail;
        const double Jn = a + 1 < n ? P.J[a + 1] : 0.0;
        dyn[kOffL + a] = (float)P.l[a];
        dyn[kOffNu + a] = (float)(P.m[a] * P.lc[a] + P.l[a] * tail);
        dyn[kOffDd + a] = (float)(mu_aa + P.I[a] + P.J[a] + Jn);
        dyn[kOffJ + 2 * a + ((a + 1) & 1)] = (float)(-Jn);   // row a+1 within its pair
        dyn[kOffDamp + a] = (float)P.b[a];
        dyn[kOffFk + a] = (float)P.fk[a];
    }
    for (int i = 0; i < 4; ++i) {
        dyn[kOffSw + i] = (float)(cfg->stage_cost_weight[i] * 10000.0);     // control.py:185
        dyn[kOffTw + i] = (float)(cfg->terminal_cost_weight[i] * 10000.0);  // control.py:198
    }
    dyn[kOffDt] = (float)cfg->delta_t;
    dyn[kOffG] = (float)P.g;
    // the fp64 rollout's constants: the same layout, unrounded
    double dynd[kCDyn] = {};
    for (int a = 0; a < kCMax; ++a) dynd[kOffDd + a] = 1.0;
    for (int a = 0; a < n; ++a) {
        double tail = 0.0;
        for (int q = a + 1; q < n; ++q) tail += P.m[q];
        const double Jn = a + 1 < n ? P.J[a + 1] : 0.0;
        dynd[kOffL + a] = P.l[a];
        dynd[kOffNu + a] = P.m[a] * P.lc[a] + P.l[a] * tail;
        dynd[kOffDd + a] = P.m[a] * P.lc[a] * P.lc[a] + P.l[a] * P.l[a] * tail + P.I[a] + P.J[a] + Jn;
        dynd[kOffJ + 2 * a + ((a + 1) & 1)] = -Jn;
        dynd[kOffDamp + a] = P.b[a];
        dynd[kOffFk + a] = P.fk[a];
    }
    for (int i = 0; i < 4; ++i) {
        dynd[kOffSw + i] = cfg->stage_cost_weight[i] * 10000.0;
        dynd[kOffTw + i] = cfg->terminal_cost_weight[i] * 10000.0;
    }
    dynd[kOffDt] = cfg->delta_t;
    dynd[kOffG] = P.g;
    memcpy(c->h_dynd, dynd, sizeof(dynd));
    k.lambda = cfg->param_lambda;
    k.inv_lambda = 1.0 / cfg->param_lambda;
    // control.py:45 fixes gamma at construction; the caller passes it as given (NaN: lambda (1 - alpha))
    k.gamma = isnan(cfg->param_gamma) ? cfg->param_lambda * (1.0 - cfg->param_alpha) : cfg->param_gamma;
    for (int i = 0; i < n * n; ++i) k.sig_inv[i] = Si[i];

    auto cleanup_fail = [&](int rc) {
        mppi_chain_ctx_destroy(c);
        return rc;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess)
        return cleanup_fail(fail(MPPI_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e)));
    int ncu = 0, per_cu = 0;
    if ((e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device)) != hipSuccess)
        return cleanup_fail(fail(MPPI_E_HIP, std::string("device attributes: ") + hipGetErrorString(e)));
#define MPPI_OCC(N)                                                                                          \
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(                                                      \
        &per_cu,                                                                                             \
        c->f64 ? (const void*)chain_rollout_kernel<N, true, true, 1>                                          \
               : (c->lps == 4 ? (const void*)chain_rollout_kernel<N, true, false, 4>                          \
                              : (const void*)chain_rollout_kernel<N, true, false, 1>),                        \
        kCT, 0)
    MPPI_CHAIN_DISPATCH(n, MPPI_OCC)
#undef MPPI_OCC
    c->poll = per_cu >= 1 && c->nblocks <= ncu;
    if (const char* ev = getenv("MPPI_HANDOFF")) {
        if (!strcmp(ev, "counter")) c->poll = false;
    }
    k.acquire = (!c->poll && c->nblocks > ncu) ? 1 : 0;
    const size_t val = c->poll ? 16 : sizeof(double);
    const int stride = 2 + cfg->T * n;
    const size_t slab = (size_t)c->nblocks * stride * val;
    const int ngroups = (c->nblocks + kGroup - 1) / kGroup;
    const size_t gslab = (size_t)ngroups * stride * val;
    const size_t cu_off = (((size_t)(ngroups + 2) * sizeof(unsigned) + 255) & ~(size_t)255) / sizeof(unsigned);
    const size_t ctr_bytes = (cu_off + kCuSlots) * sizeof(unsigned);
    c->kc.cu_off = (int)cu_off;
    c->kc.fair = c->nblocks > ncu ? 1 : 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) c->chol.L[i * kCMax + j] = (float)(Lc[i][j] * kBoxMullerScale);   // box_muller's constant
    if ((e = hipMalloc(&c->d_step, 2 * sizeof(ChainStep))) != hipSuccess ||
        (e = hipMalloc(&c->d_slab, slab)) != hipSuccess || (e = hipMalloc(&c->d_gslab, gslab)) != hipSuccess ||
        (e = hipMalloc(&c->d_counter, ctr_bytes)) != hipSuccess ||
        (e = hipMalloc(&c->d_runmin, 256)) != hipSuccess || (e = hipMemset(c->d_runmin, 0xFF, 256)) != hipSuccess ||
        (e = hipMalloc(&c->d_weps, (kCMaxVals + 1) * sizeof(double))) != hipSuccess ||
        (e = hipMalloc(&c->d_base, kCMaxVals * sizeof(float))) != hipSuccess ||
        (e = hipMalloc(&c->d_dyn, kDynF64Off * sizeof(float) + sizeof(dynd))) != hipSuccess ||
        (e = hipMemcpy(c->d_dyn + kDynF64Off, dynd, sizeof(dynd), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_step, sizeof(ChainStep), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_buf, (kCMaxVals + kCMax) * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_base, kCMaxVals * sizeof(float), hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_tmo, 256, hipHostMallocMapped)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->d_tmo, c->h_tmo, 0)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->staged, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->out_ev, hipEventDisableTiming)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_out, (kCMaxVals + kCMax + 1) * sizeof(double), hipHostMallocDefault)) != hipSuccess ||
        (e = hipMemset(c->d_counter, 0, ctr_bytes)) != hipSuccess || (e = hipMemset(c->d_slab, 0, slab)) != hipSuccess ||
        (e = hipMemset(c->d_gslab, 0, gslab)) != hipSuccess ||
        (e = hipMemset(c->d_step, 0, 2 * sizeof(ChainStep))) != hipSuccess ||
        (e = hipMemset(c->d_weps, 0, (kCMaxVals + 1) * sizeof(double))) != hipSuccess ||
        (e = hipMemcpy(c->d_dyn, k.dyn, sizeof(k.dyn), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipDeviceSynchronize()) != hipSuccess)
        return cleanup_fail(fail(MPPI_E_HIP, std::string("allocation: ") + hipGetErrorString(e)));
    memset(c->h_step, 0, sizeof(ChainStep));
    c->h_tmo[0] = c->h_tmo[1] = 0;
    c->d_epoch = c->d_counter + ngroups + 1;
    *out = c;
    return MPPI_OK;
}

void mppi_chain_ctx_destroy(mppi_chain_ctx* c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipDeviceSynchronize();
    (void)hipFree(c->d_step);
    (void)hipFree(c->d_slab);
    (void)hipFree(c->d_gslab);
    (void)hipFree(c->d_counter);
    (void)hipFree(c->d_runmin);
    (void)hipFree(c->d_weps);
    (void)hipFree(c->d_base);
    (void)hipFree(c->d_dyn);
    for (void* p : c->xopened)
        if (p) (void)hipIpcCloseMemHandle(p);
    (void)hipFree(c->d_inbox);
    (void)hipFree(c->d_xrow);
    (void)hipFree(c->d_xepoch);
    if (c->h_step) (void)hipHostFree(c->h_step);
    if (c->h_buf) (void)hipHostFree(c->h_buf);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->out_ev) (void)hipEventDestroy(c->out_ev);
    if (c->h_base) (void)hipHostFree(c->h_base);
    if (c->h_tmo) (void)hipHostFree(c->h_tmo);
    if (c->staged) (void)hipEventDestroy(c->staged);
    delete c;
}

int mppi_chain_set_stream(mppi_chain_ctx* c, void* stream) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    c->stream = (hipStream_t)stream;
    return MPPI_OK;
}

int mppi_chain_ctx_info(const mppi_chain_ctx* c, int* blocks, int* threads, int* poll, int* lanes_per_sample) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    if (lanes_per_sample) *lanes_per_sample = c->lps;
    if (blocks) *blocks = c->nblocks;
    if (threads) *threads = kCT;
    if (poll) *poll = c->poll ? 1 : 0;
    return MPPI_OK;
}

int mppi_chain_set_step_inputs(mppi_chain_ctx* c, const double* x0, const double* window, int W, const double* u) {
    if (!c || !x0 || !window) return fail(MPPI_E_ARG, "null argument");
    if (W < 1 || W > MPPI_SEARCH_LEN) return fail(MPPI_E_ARG, "window rows must be in [1, 30]");
    const int n = c->n, T = c->cfg.T;
    if (hipEventSynchronize(c->staged) != hipSuccess) return fail(MPPI_E_HIP, "staging event");
    ChainStep* h = c->h_step;
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
            h->key[j] = make_float4((float)(-2.0 * rx), (float)(-2.0 * ry), (float)(rx * rx + ry * ry), 0.f);
        } else {
            h->win[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            h->key[j] = make_float4(0.f, 0.f, kPadKey, 0.f);
        }
    }
    h->ctr = make_float4((float)cx, (float)cy, (float)W, 0.f);
    for (int a = 0; a < 2 * kCMax; ++a) h->x0[a] = a < 2 * n ? (float)x0[a] : 0.f;
    // fp64 rollout: x0 as [q(n), dq(n)] and the window rows unrounded
    for (int a = 0; a < 2 * kCMax; ++a) h->x0d[a] = a < 2 * n ? x0[a] : 0.0;
    for (int j = 0; j < kSlots; ++j)
        for (int i = 0; i < 4; ++i) h->wind[j][i] = j < W ? window[4 * j + i] : 0.0;
    size_t bytes = offsetof(ChainStep, ua);
    // the caller's u is the nominal the last fused launch wrote and wait_outputs returned: the device block
    // already holds it with the same (u, a) bits the staging below would compute, so only x0 and the window go
    bool same = u && c->pub_valid;
    for (int t = 0; same && t < T; ++t)
        for (int d = 0; d < n; ++d) same = same && u[t * n + d] == c->h_pub[t * kCMax + d];
    if (same) u = nullptr;
    if (u) {
        const ChainConst& k = c->kc;
        for (int t = 0; t < T; ++t) {
            for (int d = 0; d < kCMax; ++d) {
                h->ua[t][d] = d < n ? (float)u[t * n + d] : 0.f;
                h->u[t][d] = d < n ? u[t * n + d] : 0.0;
                double a = 0.0;
                if (d < n)
                    for (int e2 = 0; e2 < n; ++e2) a += (k.gamma * u[t * n + e2]) * k.sig_inv[e2 * n + d];
                h->ua[t][kCMax + d] = (float)a;
                h->a[t][d] = a;
            }
        }
        bytes = sizeof(ChainStep);
        c->upd_valid = false;   // the block now holds the staged nominal, not a fused update's output
        c->pub_valid = false;
    }
    if (hipMemcpyAsync(c->d_step + (c->cur ^ 1), h, offsetof(ChainStep, ua), hipMemcpyHostToDevice, c->stream) !=
            hipSuccess ||
        hipMemcpyAsync(c->d_step + c->cur, h, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipEventRecord(c->staged, c->stream) != hipSuccess)
        return fail(MPPI_E_HIP, "step input upload");
    return MPPI_OK;
}

}  // extern "C"

namespace {
// slots: the debug instances (kCDebugN links) record every sample's window slot per step
int chain_rollout(mppi_chain_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags,
                  int* slots) {
    if (!c || !noise_dev) return fail(MPPI_E_ARG, "null argument");
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    if (flags & MPPI_FLAG_EXCHANGE) {
        if (c->xd.world < 1) return fail(MPPI_E_ARG, "MPPI_FLAG_EXCHANGE before mppi_chain_exchange_attach");
        if (partial_dev) return fail(MPPI_E_ARG, "MPPI_FLAG_EXCHANGE merges on device: no partial_out");
        partial_dev = c->d_xrow;
    }
    const ChainStep* cur = c->d_step + c->cur;
    ChainStep* nxt = c->d_step + (c->cur ^ 1);
#define MPPI_L(N)                                                                       \
    if (c->f64) {                                                                       \
        if (c->poll) launch_rollout<N, true, true, 1>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots); \
        else launch_rollout<N, false, true, 1>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots); \
    } else if (c->lps == 4) {                                                           \
        if (c->poll) launch_rollout<N, true, false, 4>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots); \
        else launch_rollout<N, false, false, 4>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots); \
    } else if (c->poll) launch_rollout<N, true, false, 1>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots); \
    else launch_rollout<N, false, false, 1>(c, cur, noise_dev, S_dev, partial_dev, nxt, flags, slots)
    MPPI_CHAIN_DISPATCH(c->n, MPPI_L)
#undef MPPI_L
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("chain_rollout_kernel: ") + hipGetErrorString(e));
    if (flags & MPPI_FLAG_FUSED_UPDATE) c->cur ^= 1;
    c->x_flipped = (flags & MPPI_FLAG_FUSED_UPDATE) && (flags & MPPI_FLAG_EXCHANGE);   // undone on MPPI_E_EXCHANGE
    c->upd_valid = (flags & MPPI_FLAG_FUSED_UPDATE) != 0;
    if (flags & MPPI_FLAG_FUSED_UPDATE) c->pub_valid = false;
    c->out_posted = false;
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && (flags & MPPI_FLAG_HOST_OUT)) {
        // the update's read-back right behind the launch, so what the caller queues next (the next
        // step's noise) does not delay mppi_chain_wait_outputs
        const char* blk = (const char*)(c->d_step + c->cur);
        if (hipMemcpyAsync(c->h_out, blk + offsetof(ChainStep, u), (size_t)c->cfg.T * kCMax * sizeof(double),
                           hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipMemcpyAsync(c->h_out + kCMaxVals, blk + offsetof(ChainStep, u_first), (kCMax + 1) * sizeof(double),
                           hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipEventRecord(c->out_ev, c->stream) != hipSuccess)
            return fail(MPPI_E_HIP, "update read-back");
        c->out_posted = true;
    }
    return MPPI_OK;
}
}  // namespace

extern "C" {

int mppi_chain_rollout(mppi_chain_ctx* c, const float* noise_dev, double* S_dev, double* partial_dev, unsigned flags) {
    return chain_rollout(c, noise_dev, S_dev, partial_dev, flags, nullptr);
}

int mppi_chain_debug_slots(mppi_chain_ctx* c, const float* noise_dev, double* S_dev, int* slots_dev) {
    if (!c || !noise_dev || !slots_dev) return fail(MPPI_E_ARG, "null argument");
    if (c->n != kCDebugN) return fail(MPPI_E_ARG, "slot recording is built for the 7-link chain only");
    return chain_rollout(c, noise_dev, S_dev, nullptr, 0u, slots_dev);
}


int mppi_chain_exchange_handle(mppi_chain_ctx* c, int world, void* handle_out) {
    if (!c || !handle_out || world < 1 || world > kMaxWorld) return fail(MPPI_E_ARG, "bad argument");
    if (c->d_inbox && c->xworld_alloc != world) return fail(MPPI_E_ARG, "inbox already sized for another world");
    const int stride = 2 + c->cfg.T * c->n;
    if (!c->d_inbox) {
        const size_t bytes = (size_t)2 * world * (stride + 1) * 16;   // rows and statuses, two parities
        hipError_t e;
        if ((e = hipSetDevice(c->device)) != hipSuccess ||
            (e = hipExtMallocWithFlags(&c->d_inbox, bytes, hipDeviceMallocUncached)) != hipSuccess ||
            (e = hipMemset(c->d_inbox, 0, bytes)) != hipSuccess ||
            (e = hipMalloc(&c->d_xrow, stride * sizeof(double))) != hipSuccess ||
            (e = hipMalloc(&c->d_xepoch, 256)) != hipSuccess || (e = hipMemset(c->d_xepoch, 0, 256)) != hipSuccess ||
            (e = hipDeviceSynchronize()) != hipSuccess)
            return fail(MPPI_E_HIP, std::string("exchange inbox: ") + hipGetErrorString(e));
        c->xworld_alloc = world;
        c->xd.bytes = (int)bytes;
    }
    const hipError_t e = hipIpcGetMemHandle(static_cast<hipIpcMemHandle_t*>(handle_out), c->d_inbox);
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("hipIpcGetMemHandle: ") + hipGetErrorString(e));
    return MPPI_OK;
}

int mppi_chain_exchange_attach(mppi_chain_ctx* c, int rank, int world, const void* handles) {
    if (!c || !handles || world < 1 || rank < 0 || rank >= world) return fail(MPPI_E_ARG, "bad argument");
    if (!c->d_inbox || c->xworld_alloc != world) return fail(MPPI_E_ARG, "call mppi_chain_exchange_handle(world) first");
    if (c->xd.world) return fail(MPPI_E_ARG, "already attached");
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    const hipIpcMemHandle_t* h = static_cast<const hipIpcMemHandle_t*>(handles);
    for (int p = 0; p < world; ++p) {
        if (p == rank) {
            c->xd.peer[p] = c->d_inbox;
            continue;
        }
        void* ptr = nullptr;
        if ((e = hipIpcOpenMemHandle(&ptr, h[p], hipIpcMemLazyEnablePeerAccess)) != hipSuccess)
            return fail(MPPI_E_HIP, std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e));
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

int mppi_chain_merge_partials(mppi_chain_ctx* c, const double* partials_dev, int nparts, unsigned flags) {
    if (!c || !partials_dev || nparts < 1) return fail(MPPI_E_ARG, "bad argument");
    if ((flags & MPPI_FLAG_FUSED_UPDATE) && c->cfg.T < 5)
        return fail(MPPI_E_ARG, "device median filter needs T >= 5 (use the host update)");
    const ChainStep* cur = c->d_step + c->cur;
    ChainStep* nxt = c->d_step + (c->cur ^ 1);
#define MPPI_M(N)                                                                                              \
    hipLaunchKernelGGL(chain_merge_kernel<N>, dim3(1), dim3(kCT), 0, c->stream, c->kc, cur, partials_dev, nparts, \
                       c->d_weps, nxt, flags)
    MPPI_CHAIN_DISPATCH(c->n, MPPI_M)
#undef MPPI_M
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("chain_merge_kernel: ") + hipGetErrorString(e));
    if (flags & MPPI_FLAG_FUSED_UPDATE) c->cur ^= 1;
    c->x_flipped = (flags & MPPI_FLAG_FUSED_UPDATE) && (flags & MPPI_FLAG_EXCHANGE);   // undone on MPPI_E_EXCHANGE
    c->upd_valid = (flags & MPPI_FLAG_FUSED_UPDATE) != 0;
    if (flags & MPPI_FLAG_FUSED_UPDATE) c->pub_valid = false;
    return MPPI_OK;
}

int mppi_chain_get_weighted_noise(mppi_chain_ctx* c, double* w_eps_host) {
    if (!c || !w_eps_host) return fail(MPPI_E_ARG, "null argument");
    const size_t bytes = (size_t)c->cfg.T * c->n * sizeof(double);
    if (hipMemcpyAsync(c->h_buf, c->d_weps, bytes + sizeof(double), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return fail(MPPI_E_HIP, "weighted noise read-back");
    memcpy(w_eps_host, c->h_buf, bytes);
    c->last_eta = c->h_buf[(size_t)c->cfg.T * c->n];
    return check_tmo(c);
}

int mppi_chain_get_nominal(mppi_chain_ctx* c, double* u_host) {
    if (!c || !u_host) return fail(MPPI_E_ARG, "null argument");
    const int n = c->n, T = c->cfg.T;
    if (hipMemcpyAsync(c->h_buf, (const char*)(c->d_step + c->cur) + offsetof(ChainStep, u),
                       (size_t)T * kCMax * sizeof(double), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return fail(MPPI_E_HIP, "nominal read-back");
    for (int t = 0; t < T; ++t)
        for (int d = 0; d < n; ++d) u_host[t * n + d] = c->h_buf[t * kCMax + d];
    return check_tmo(c);
}

int mppi_chain_last_eta(const mppi_chain_ctx* c, double* eta) {
    if (!c || !eta) return fail(MPPI_E_ARG, "null argument");
    *eta = c->last_eta;
    return MPPI_OK;
}

}  // extern "C"

namespace {
// control.py:129-134 for the chain in fp64 on the host: x_{t+1} = F(x_t, u_new[t - 1]) (u_new[-1] at t = 0),
// the same ChainStateD step as the fp64 rollout.  One sequential trajectory: the host's fp64 is ~5x the
// device's single lane here (~1.7 us per step of dependent VALU on one wave).
template <int N>
__attribute__((always_inline)) inline void chain_traj_body(const double* kd, const double* x0, const double* u_new,
                                                           int T, double* out) {
    ChainStateD<N> x;
    x.load(x0);
    for (int t = 0; t < T; ++t) {
        const double* ut = u_new + (size_t)N * (t == 0 ? T - 1 : t - 1);
        double v[N];
        for (int d = 0; d < N; ++d) v[d] = ut[d];
        x.step(v, kd);
        for (int a = 0; a < N; ++a) {
            out[(size_t)t * 2 * N + a] = x.q[a];
            out[(size_t)t * 2 * N + N + a] = x.dq[a];
        }
    }
}
// The step's fma() calls as the hardware instruction where the CPU has it (the baseline x86-64 target calls
// libm's fma ~600 times per step set); fma is correctly rounded either way, and the host side of this file is
// compiled with -ffp-contract=off (build.py), so no other multiply-add is fused in either instance: the same
// bits (MPPI_HOST_FMA=0 forces the baseline instance; tests/test_gpu_chain.py compares the two).
template <int N>
__attribute__((target("fma"))) void chain_traj_host_fma(const double* kd, const double* x0, const double* u_new,
                                                        int T, double* out) {
    chain_traj_body<N>(kd, x0, u_new, T, out);
}
template <int N>
void chain_traj_host(const double* kd, const double* x0, const double* u_new, int T, double* out) {
    static const bool hw_fma = __builtin_cpu_supports("fma");
    const char* force = getenv("MPPI_HOST_FMA");
    if (hw_fma && !(force && force[0] == '0')) chain_traj_host_fma<N>(kd, x0, u_new, T, out);
    else chain_traj_body<N>(kd, x0, u_new, T, out);
}
}  // namespace

extern "C" {

int mppi_chain_wait_outputs(mppi_chain_ctx* c, const double* x0, double* u_out, double* traj_out) {
    if (!c || !u_out || (traj_out && !x0)) return fail(MPPI_E_ARG, "bad argument");
    if (!c->upd_valid) return fail(MPPI_E_ARG, "no fused update to read (mppi_chain_rollout with MPPI_FLAG_FUSED_UPDATE)");
    const int n = c->n, T = c->cfg.T;
    const double* h = c->h_out;
    if (c->out_posted) {   // MPPI_FLAG_HOST_OUT: the copy is already queued behind the launch
        if (hipEventSynchronize(c->out_ev) != hipSuccess) return fail(MPPI_E_HIP, "update read-back");
    } else {
        const char* blk = (const char*)(c->d_step + c->cur);
        if (hipMemcpyAsync(c->h_out, blk + offsetof(ChainStep, u), (size_t)T * kCMax * sizeof(double),
                           hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipMemcpyAsync(c->h_out + kCMaxVals, blk + offsetof(ChainStep, u_first), (kCMax + 1) * sizeof(double),
                           hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            return fail(MPPI_E_HIP, "update read-back");
    }
    if (int rc = check_tmo(c)) return rc;
    c->last_eta = h[kCMaxVals + kCMax];
    for (int t = 0; t < T; ++t)
        for (int d = 0; d < n; ++d) u_out[t * n + d] = h[t * kCMax + d];
    memcpy(c->h_pub, h, (size_t)T * kCMax * sizeof(double));
    c->pub_valid = true;
    if (traj_out) {
        // the update before the shift: u_new[0] from the block, u_new[t] = shifted[t - 1] for t >= 1
        double un[kMaxT * kCMax];
        for (int d = 0; d < n; ++d) un[d] = h[kCMaxVals + d];
        for (int t = 1; t < T; ++t)
            for (int d = 0; d < n; ++d) un[t * n + d] = h[(t - 1) * kCMax + d];
        return mppi_chain_optimal_traj_host(c, x0, un, traj_out);
    }
    return MPPI_OK;
}

int mppi_chain_optimal_traj_host(mppi_chain_ctx* c, const double* x0, const double* u_new, double* traj_out) {
    if (!c || !x0 || !u_new || !traj_out) return fail(MPPI_E_ARG, "null argument");
#define MPPI_TH(N) chain_traj_host<N>(c->h_dynd, x0, u_new, c->cfg.T, traj_out)
    MPPI_CHAIN_DISPATCH(c->n, MPPI_TH);
#undef MPPI_TH
    return MPPI_OK;
}

int mppi_chain_rollout_traj(mppi_chain_ctx* c, const double* base_u, const float* noise_dev, int K, float* out_dev) {
    if (!c || !out_dev || K < 1 || K > c->cfg.K_local) return fail(MPPI_E_ARG, "bad argument");
    const int n = c->n, T = c->cfg.T;
    const ChainStep* cur = c->d_step + c->cur;
    if (base_u) {
        if (hipEventSynchronize(c->staged) != hipSuccess) return fail(MPPI_E_HIP, "staging event");
        for (int i = 0; i < T * n; ++i) c->h_base[i] = (float)base_u[i];
        if (hipMemcpyAsync(c->d_base, c->h_base, (size_t)T * n * sizeof(float), hipMemcpyHostToDevice, c->stream) !=
                hipSuccess ||
            hipEventRecord(c->staged, c->stream) != hipSuccess)
            return fail(MPPI_E_HIP, "base upload");
    } else {
        // the nominal u of the current step block: ua[t][0:n], row stride 2 kCMax floats
        if (hipMemcpy2DAsync(c->d_base, n * sizeof(float), (const char*)cur + offsetof(ChainStep, ua),
                             2 * kCMax * sizeof(float), n * sizeof(float), T, hipMemcpyDeviceToDevice,
                             c->stream) != hipSuccess)
            return fail(MPPI_E_HIP, "base copy");
    }
    const int blocks = (K + kCT - 1) / kCT;
#define MPPI_T(N)                                                                                                \
    do {                                                                                                         \
        if (noise_dev)                                                                                           \
            hipLaunchKernelGGL((chain_traj_kernel<N, true>), dim3(blocks), dim3(kCT), 0, c->stream, c->kc, cur,  \
                               c->d_base, noise_dev, K, out_dev);                                                \
        else                                                                                                     \
            hipLaunchKernelGGL((chain_traj_kernel<N, false>), dim3(blocks), dim3(kCT), 0, c->stream, c->kc, cur, \
                               c->d_base, noise_dev, K, out_dev);                                                \
    } while (0)
    MPPI_CHAIN_DISPATCH(n, MPPI_T)
#undef MPPI_T
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("chain_traj_kernel: ") + hipGetErrorString(e));
    return MPPI_OK;
}

int mppi_chain_noise_philox(mppi_chain_ctx* c, unsigned long long seed, unsigned long long step, float* out_dev) {
    if (!c || !out_dev) return fail(MPPI_E_ARG, "null argument");
    const dim3 grid((unsigned)((c->cfg.K_local + kCT - 1) / kCT), (unsigned)c->cfg.T);
#define MPPI_PH(N)                                                                                            \
    hipLaunchKernelGGL(chain_philox_kernel<N>, grid, dim3(kCT), 0, c->stream, c->cfg.K_local, c->cfg.T,         \
                       (long long)c->cfg.k_offset, seed, step, c->chol, out_dev)
    MPPI_CHAIN_DISPATCH(c->n, MPPI_PH);
#undef MPPI_PH
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MPPI_E_HIP, std::string("chain_philox_kernel: ") + hipGetErrorString(e));
    return MPPI_OK;
}

int mppi_chain_sync(mppi_chain_ctx* c) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    if (hipStreamSynchronize(c->stream) != hipSuccess) return fail(MPPI_E_HIP, "stream synchronize");
    return check_tmo(c);
}

int mppi_chain_debug_set_buffer(mppi_chain_ctx* c, void* dbg_dev) {
    if (!c) return fail(MPPI_E_ARG, "null context");
    c->d_dbg = (unsigned long long*)dbg_dev;
    return MPPI_OK;
}

}  // extern "C"
