// mppi_device.h — device building blocks shared by the MPPI kernels for gfx950
// (mppi_rocm.hip: the reference's 2-link arm; mppi_chain.hip: the n-link chain
// of BASELINE config 5): DPP wave reductions, the window search, write-through
// row buffers and tagged granules, the in-launch log-sum-exp merges of the
// workgroup partial rows, the median-of-10 network, Philox.
//
// A partial row is {rho, eta, N[nval]} (control.py:112-118 over some set of
// samples in log-sum-exp form: rho = min S, eta = sum e^{-(S - rho)/lambda},
// N = sum e^{-(S - rho)/lambda} eps), nval = T * du values.  The merges read
// rows handed over by other workgroups of the same launch (MI355X guide,
// Guideline 16): 8-B sc1 words behind an arrival counter, or 16-B tagged
// granules polled without any counter.
#pragma once

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "mppi_rocm.h"  // MPPI_SEARCH_LEN, MPPI_MAX_T

namespace mppi {

// Diagnostic builds only (-DMPPI_STAMPS, a separate .so): per-workgroup
// timeline in s_memrealtime ticks (100 MHz) + counters.  Never in the product.
#ifdef MPPI_STAMPS
#define STAMP(slot, val) do { if (dbg && threadIdx.x == 0) dbg[(size_t)blockIdx.x * 16 + (slot)] = (val); } while (0)
#define NOW() __builtin_amdgcn_s_memrealtime()
#else
#define STAMP(slot, val) do { (void)dbg; } while (0)
#define NOW() 0ull
#endif

constexpr int kMaxT = MPPI_MAX_T;

constexpr int kSlots = 32;             // window slots (>= MPPI_SEARCH_LEN), index fits 5 bits
constexpr float kPadKey = 1.0e30f;
constexpr int kMaxWaves = 16;          // up to 1024-thread workgroups
constexpr int kGroup = 16;             // workgroups per first-level merge group
// A partial whose rescale factor s = exp((rho - rho_i) / lambda) is below 2^-64
// changes eta and N by less than 2^-64 * 512 relative to the leading term
// (which has s = 1 and eta >= 1): far below the fp64 resolution of the result.
constexpr double kMergeFloor = 5.421010862427522e-20;  // 2^-64
constexpr int kDirectRows = 256;       // workgroup rows the direct merge scans (4 per lane)
constexpr int kDirectMax = 16;         // weighted rows it merges; more go through the group rows
constexpr int kSparseMax = 16;         // weighted samples per workgroup handled by the epilogue gather

// ------------------------------------------------------------------ helpers

// Hardware v_sin_f32 / v_cos_f32 (argument pre-scaled by 1/(2 pi)): 30 % faster
// rollouts than OCML's sincosf at K=65536 T=64, parity unchanged (S rel-err
// budget 5e-5 in tests/test_gpu_parity.py).
__device__ __forceinline__ void sincos_f32(float x, float* s, float* c) { __sincosf(x, s, c); }

// Every control used here (quad_perm, row_mirror, row_half_mirror, row_ror) reads
// a valid lane, so bound_ctrl changes no value; set, it lets the compiler fold the
// move into a VOP1 / VOP2 consumer (v_mul_f32_dpp, v_add_f32_dpp, v_rsq_f32_dpp:
// GCNDPPCombine takes a move with an undefined old value only under bound_ctrl).
constexpr bool kDppBC = true;
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, kDppBC));
}

__device__ __forceinline__ int lanes_below(unsigned long long mask) {
    return __builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, kDppBC);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, kDppBC);
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

// v_min_f64 / v_max_f64 issued directly: fmin()/fmax() make hipcc canonicalise
// both operands first (a v_max_f64 x, x each).  Same results for every input
// but signalling NaNs (IEEE minNum / maxNum, like fmin / fmax).
__device__ __forceinline__ double min_raw_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double max_raw_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
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
struct OpMin {
    __device__ double operator()(double a, double b) const { return min_raw_f64(a, b); }
};
struct OpAdd {
    template <class T>
    __device__ T operator()(T a, T b) const { return a + b; }
};
__device__ __forceinline__ double wave_min_f64(double v) { return wave_reduce(v, OpMin{}); }
__device__ __forceinline__ double wave_sum_f64(double v) { return wave_reduce(v, OpAdd{}); }
__device__ __forceinline__ float wave_sum_f32(float v) { return wave_reduce(v, OpAdd{}); }

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

template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// Scheduling boundary after each prefetch: an empty asm statement with a
// memory clobber keeps the load where it is written (otherwise the scheduler
// sinks it next to its use and every step pays the full memory latency).
#define PIN_LOADS() asm volatile("" ::: "memory")

// The per-step constants are read through the constant address space: scalar
// (SMEM) loads that stay scalar across the scheduling boundaries above.  Their
// block is written only by host copies or by the PREVIOUS launch (ping-pong).
typedef __attribute__((address_space(4))) const float cfloat;
__device__ __forceinline__ float4 const_ld4(cfloat* p) { return make_float4(p[0], p[1], p[2], p[3]); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// ------------------------------------------------------------ window search

// Minimum of N packed keys as a tree of v_min3 (depth ceil(log3 N))
template <int N>
__device__ __forceinline__ float min_tree(const float (&k)[N]) {
    if constexpr (N == 1) {
        return k[0];
    } else {
        constexpr int M = (N + 2) / 3;
        float r[M];
#pragma unroll
        for (int g = 0; g < M; ++g) {
            const int a = 3 * g;
            if (a + 2 < N) r[g] = min3_raw(k[a], k[a + 1], k[a + 2]);
            else if (a + 1 < N) r[g] = min_raw(k[a], k[a + 1]);
            else r[g] = k[a];
        }
        return min_tree<M>(r);
    }
}

// Nearest waypoint of the shared window (control.py:200-232): the window is
// uploaded as centred keys (-2 rx', -2 ry', rx'^2 + ry'^2; pads 1e30 — the
// factor -2 is exact, so it costs nothing to fold it into the table), and
//   argmin_j |p - r_j|^2 = argmin_j (|r'_j|^2 - 2 p'.r'_j),
// two slots per v_pk_fma_f32; the slot index is packed into the 5 low mantissa
// bits so one v_min3 per two slots carries the argmin (first occurrence: equal
// keys resolve to the lower slot); the LPS lanes of a sample split the window
// and close the min with DPP.
//
// Precision: packing quantises a key to 2^-18 of its magnitude, ~|r'|^2 (the
// window's half-extent squared, ~5e-4 m^2 on xydq_circle.txt), so two
// waypoints whose squared distances differ by less than ~1e-9 m^2 may resolve
// to the lower slot.  PRECISE adds |p'|^2 to every key before packing (one
// v_pk_add per two slots): the key is then the squared distance itself, the
// quantisation acts on it, and what remains is the fp32 rounding of the key
// (~1e-10 m^2).  The 2-link engine keeps the cheaper form (its parity on the
// reference's fixtures is unaffected, +10 % instructions otherwise); the chain
// engine, whose config-5 start pose sits ON a waypoint, uses PRECISE.
template <int LPS, bool PRECISE = false>
struct Search {
    static constexpr int SL = ((MPPI_SEARCH_LEN + LPS - 1) / LPS + 1) & ~1;  // slots per lane, even
    static constexpr int SP = SL / 2;
    f32x2 krx[SP], kry[SP], kc[SP];
    int sub;
    float cx, cy;

    // key: the centred keys (kSlots float4), ctr: the window centre
    __device__ __forceinline__ void load(const float4* key, float4 ctr, int lane_sub) {
        static_assert(SL * LPS <= kSlots, "window slots");
        if (LPS == 1) {
            // lane-opaque zero: keeps the 30 window slots in VGPRs (as uniform
            // values they would go to SGPRs and spill)
            int z;
            asm volatile("v_mov_b32 %0, 0" : "=v"(z));
            sub = z;
        } else {
            sub = lane_sub;
        }
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            const float4 k0 = key[sub * SL + 2 * i];
            const float4 k1 = key[sub * SL + 2 * i + 1];
            krx[i] = f32x2{k0.x, k1.x};
            kry[i] = f32x2{k0.y, k1.y};
            kc[i] = f32x2{k0.z, k1.z};
        }
        cx = ctr.x;
        cy = ctr.y;
    }

    __device__ __forceinline__ unsigned nearest(float px, float py) const { return nearest_d(px - cx, py - cy); }

    // dx, dy: the position relative to the window centre
    __device__ __forceinline__ unsigned nearest_d(float dx, float dy) const {
        const f32x2 ax2 = {dx, dx}, ay2 = {dy, dy};
        const float pp = fmaf(dx, dx, dy * dy);
        const f32x2 pp2 = {pp, pp};
        float kk[2 * SP];
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            f32x2 key = __builtin_elementwise_fma(ax2, krx[i], __builtin_elementwise_fma(ay2, kry[i], kc[i]));
            if constexpr (PRECISE) key = key + pp2;   // |p - r_j|^2
            // through the opaque sub even at LPS = 1: measured 2.5% faster than a
            // constant index (v_and + v_or3 packing schedules better there; tools/ab.py)
            const unsigned j = (unsigned)(sub * SL + 2 * i);
            const float k0 = __uint_as_float((__float_as_uint(key.x) & ~31u) | j);
            const float k1 = __uint_as_float((__float_as_uint(key.y) & ~31u) | (j + 1));
            kk[2 * i] = k0;
            kk[2 * i + 1] = k1;
        }
        // the same v_min3 count as a running minimum, but 4 levels deep instead of
        // 15 (the keys carry distinct indices, so the order of the minima is free)
        float best = min_tree<2 * SP>(kk);
        if (LPS >= 2) best = min_raw(best, dpp_f32<0xB1>(best));  // quad_perm xor 1
        if (LPS >= 4) best = min_raw(best, dpp_f32<0x4E>(best));  // quad_perm xor 2
        if (LPS >= 8) best = min_raw(best, dpp_f32<0x141>(best));  // row_half_mirror: the other quad of 8
        if (LPS >= 16) best = min_raw(best, dpp_f32<0x128>(best));  // row_ror:8: the other half of the row
        return __float_as_uint(best) & 31u;
    }
};

// The same search with the window keys in LDS instead of registers: the keys
// are uniform across the workgroup, so every read is a broadcast ds_read_b128
// (two per two slots: {rx'0, rx'1, ry'0, ry'1}, {c'0, c'1, -, -}).  Costs one
// LDS read per slot and per step, frees the 3 x 30 key registers — for kernels
// whose per-lane state is large (the n-link chain) that buys occupancy.
struct alignas(16) KeyPair {
    float4 xy;   // -2 rx'(2i), -2 rx'(2i+1), -2 ry'(2i), -2 ry'(2i+1)
    float4 c;    // c'(2i), c'(2i+1), 0, 0
};
constexpr int kKeyPairs = kSlots / 2;

template <bool PRECISE = false>
struct SearchLDS {
    const KeyPair* kp;   // LDS, kKeyPairs entries
    float cx, cy;

    // cooperative fill by the first kKeyPairs threads; a barrier must follow
    __device__ __forceinline__ static void fill(KeyPair* dst, const float4* key, int tid) {
        if (tid < kKeyPairs) {
            const float4 k0 = key[2 * tid], k1 = key[2 * tid + 1];
            dst[tid].xy = make_float4(k0.x, k1.x, k0.y, k1.y);
            dst[tid].c = make_float4(k0.z, k1.z, 0.f, 0.f);
        }
    }

    __device__ __forceinline__ unsigned nearest(float px, float py) const {
        const float dx = px - cx, dy = py - cy;
        const f32x2 ax2 = {dx, dx}, ay2 = {dy, dy};
        const float pp = fmaf(dx, dx, dy * dy);
        const f32x2 pp2 = {pp, pp};
        float best = 3.0e38f;
        constexpr int SP = (MPPI_SEARCH_LEN + 1) / 2;
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            const float4 xy = kp[i].xy, cc = kp[i].c;
            f32x2 key = __builtin_elementwise_fma(ax2, f32x2{xy.x, xy.y},
                                                  __builtin_elementwise_fma(ay2, f32x2{xy.z, xy.w}, f32x2{cc.x, cc.y}));
            if constexpr (PRECISE) key = key + pp2;   // |p - r_j|^2
            const unsigned j = (unsigned)(2 * i);
            const float k0 = __uint_as_float((__float_as_uint(key.x) & ~31u) | j);
            const float k1 = __uint_as_float((__float_as_uint(key.y) & ~31u) | (j + 1));
            best = min3_raw(best, k0, k1);
        }
        return __float_as_uint(best) & 31u;
    }
};

// Epilogue gather of one noise column for the workgroup's listed samples:
// sum_l w_l eps[k_l] in ascending l (fp64 fma), the NL loads of the column
// issued together.  NL is a compile-time bucket >= nl, so a workgroup with one
// weighted sample issues one load per column, not kSparseMax.
template <int NL>
__device__ __forceinline__ double gather_col_n(const float* base, int kstride, const int* s_k, const double* s_e,
                                               int nl) {
    float e[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) e[l] = base[(size_t)(nl > 0 ? s_k[min(l, nl - 1)] : 0) * kstride];
    double acc = 0.0;
#pragma unroll
    for (int l = 0; l < NL; ++l)
        if (l < nl) acc = fma(s_e[l], (double)e[l], acc);
    return acc;
}
// nl: wave-uniform, <= kSparseMax
__device__ __forceinline__ double gather_col(const float* base, int kstride, const int* s_k, const double* s_e,
                                             int nl) {
    static_assert(kSparseMax == 16, "buckets");
    if (nl <= 1) return gather_col_n<1>(base, kstride, s_k, s_e, nl);
    if (nl <= 2) return gather_col_n<2>(base, kstride, s_k, s_e, nl);
    if (nl <= 4) return gather_col_n<4>(base, kstride, s_k, s_e, nl);
    if (nl <= 8) return gather_col_n<8>(base, kstride, s_k, s_e, nl);
    return gather_col_n<16>(base, kstride, s_k, s_e, nl);
}

// stage / terminal cost terms (control.py:185-198, weights x 10000 folded in)
__device__ __forceinline__ float weighted_sq(float ex, float ey, float e1, float e2, const float* w) {
    return fmaf(w[0], ex * ex, fmaf(w[1], ey * ey, fmaf(w[2], e1 * e1, w[3] * e2 * e2)));
}

// ------------------------------------------------ rows handed between workgroups

// Rows {rho, eta, N} handed between workgroups of one launch travel
// write-through: every store and every load of them is a `sc1` buffer access
// (MI355X guide G16, "Valid forms" row 1), so neither side needs an agent-scope
// fence (~1.7 us each).
typedef unsigned int u32x2 __attribute__((__vector_size__(2 * sizeof(unsigned int))));
typedef unsigned int u32x4 __attribute__((__vector_size__(4 * sizeof(unsigned int))));
constexpr int kSC1 = 16;  // buffer aux bit: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void* p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ double ld_wt(__amdgpu_buffer_rsrc_t r, int idx) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, kSC1));
}
__device__ __forceinline__ void st_wt(__amdgpu_buffer_rsrc_t r, int idx, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, idx * 8, 0, kSC1);
}
// Element index past every rows buffer: a raw buffer load beyond num_records
// returns 0 without a memory access, so a predicated-off load needs no branch
// (a branch around each load makes the compiler wait for it at the join).
constexpr int kOffRange = 1 << 26;  // x 16 B = 1 GiB > any rows buffer, no int overflow

// Tagged granules (MI355X guide, Guideline 16 R2: "the data IS the flag").  One
// fp64 value travels as {lo32, tag, hi32, tag} in ONE 16-B sc1 store; each 8-B
// half is a naturally aligned {value, tag} granule, so a reader that sees both
// tags equal to this launch's epoch holds the whole value — no drain, no flag,
// no counter.  Tags come from a device-resident epoch (never a kernel argument:
// graph replay freezes those), zeroed once at context creation.
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
// The host-mapped timeout words: tmo[0] = kTmoLocal (a hand-off of this launch gave up), tmo[1] = the
// exchange's verdict bits (kTmoExchange, kTmoSplit below).  Separate words, plain stores (no read-modify-write
// over the host link), so the exchange's verdict never overwrites a local cause; the host ORs them.
__device__ __forceinline__ void report_timeout(unsigned* tmo) {
    if (tmo) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
#define MPPI_SPIN_OR_GIVE_UP(spins, tmo, lane) MPPI_SPIN_OR_GIVE_UP_L(spins, 0ull, tmo, lane, (void)0)
// with a deadline of its own (s_memrealtime ticks, 100 MHz; 0: the spin bound alone) and a statement run
// when it gives up (the exchange's polls)
#define MPPI_SPIN_OR_GIVE_UP_L(spins, deadline, tmo, lane, on_give_up)                                   \
    if (spins >= kSpinMax || ((deadline) && __builtin_amdgcn_s_memrealtime() > (deadline))) {            \
        if ((lane) == 0) report_timeout(tmo);                                                            \
        on_give_up;                                                                                      \
        break;                                                                                           \
    }                                                                                                    \
    __builtin_amdgcn_s_sleep(1)

// Order-preserving 64-bit key of a double (unsigned order == numeric order; NaN
// above +inf) for integer atomic min / max, and its inverse.
__device__ __forceinline__ unsigned long long ord_key(double x) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | (1ull << 63));
}
__device__ __forceinline__ double ord_val(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & ~(1ull << 63)) : ~k));
}

// ------------------------------------------------------------ merge scratch

template <int MAXV>
struct MergeScratch {
    double red[kMaxWaves];
    double weps[MAXV];
    double unew[MAXV];
    double rho[kDirectRows];  // direct merge: the rows' rho, polled by wave 0
    double part[2 * kDirectRows];  // direct merge: per row-group column sums (one group per ncol threads)
    double eta;                    // the final merge's eta = sum_k e^{-(S_k - rho)/lambda} (>= 1; 1: one-hot)
    double rho_fin;                // the final merge's rho
    int nrel;
};

// Workgroup minimum.  One use per kernel: the caller's next barrier protects
// sm.red before any reuse.
template <int NT, class SM>
__device__ __forceinline__ double block_min_f64(double v, SM& sm) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wave_min_f64(v);
    if (lane == 0) sm.red[wave] = v;
    __syncthreads();
    double r = sm.red[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) r = min_raw_f64(r, sm.red[w]);
    return r;
}

// Geometry of a partial row {rho, eta, N[nval]}: stride values, merged columns
// (col 0 = eta, 1 + j = N[j]).  Thread tid owns columns tid + ch * NT, ch < MAXCH.
struct RowGeo {
    int stride, ncol;
    __device__ explicit RowGeo(int nval) : stride(2 + nval), ncol(1 + nval) {}
};

// Final merged row: {rho, eta, N} to out_row (plain, read after the launch) and
// w_eps = N / eta (control.py:112-118) to sm.weps and w_eps_out.
template <int NT, int MAXCH, class SM>
__device__ __forceinline__ void put_final(double rho, const double (&acc)[MAXCH], double eta, int nrel,
                                          const RowGeo& geo, SM& sm, double* out_row, double* w_eps_out) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int ch = 0; ch < MAXCH; ++ch) {
        const int col = tid + ch * NT;
        if (col >= geo.ncol) continue;
        if (col == 0) {
            sm.nrel = nrel;
            sm.eta = eta;
            sm.rho_fin = rho;
            if (out_row) {
                out_row[0] = rho;
                out_row[1] = acc[ch];
            }
        } else {
            if (out_row) out_row[1 + col] = acc[ch];
            const double w = acc[ch] / eta;
            sm.weps[col - 1] = w;
            if (w_eps_out) w_eps_out[col - 1] = w;
        }
    }
    __syncthreads();
}

// Merge n rows (read write-through from `rows`, rows row0 .. row0 + n - 1) with
// a log-sum-exp rescale: rho = min rho_i, s_i = exp((rho - rho_i) / lambda),
// eta = sum s_i eta_i, N = sum s_i N_i, in ascending row order (deterministic);
// rows whose factor is below 2^-64 of the running best are skipped.  Rows go in
// rounds with an online rescale of the running sums when a round lowers rho.
// Wave-local: every wave reads the round's rho_i into its lanes, reduces them
// with DPP and evaluates the s_i itself; the s_i reach the column FMAs as
// scalars (v_readlane) — no LDS traffic and no barrier per round.
//
// !GRAN: 8-B sc1 words behind an arrival counter.  With one column chunk
//   (MAXCH = 1) every load of a round — rho, eta and all entries of 32 rows —
//   is issued together (one memory round trip per round); with more chunks the
//   rounds are structured exactly as GRAN's (below) with plain sc1 loads, so
//   both hand-off forms rescale and accumulate identically (same bits).
// GRAN: 16-B tagged granules polled until every tag matches `tag`: rho first,
//   one lane per row (16 rows per round), then eta and the entries of only the
//   rows that carry weight, 16 / MAXCH rows per load batch.
// The merged row goes to out_wt (same format, next level) or, with `final`,
// to put_final.
template <int NT, int MAXCH, bool final, bool GRAN, class SM>
__device__ __forceinline__ void merge_rows_block(__amdgpu_buffer_rsrc_t rows, int row0, int n, const RowGeo& geo,
                                                 double inv_lambda, SM& sm, const __amdgpu_buffer_rsrc_t* out_wt,
                                                 int out_idx, double* out_row, double* w_eps_out, unsigned tag,
                                                 unsigned* tmo, unsigned long long deadline = 0ull,
                                                 bool* failed = nullptr) {
    // deadline / failed: the polls' deadline (s_memrealtime; 0: the spin bound alone), and (when given) whether
    // any poll of the workgroup gave up (uniform).
    constexpr bool EAGER = !GRAN && MAXCH == 1;  // one round trip per round of 32 rows
    constexpr int LB = EAGER ? 32 : 16;         // loads per batch per thread
    constexpr int RB = LB / MAXCH;              // rows per load batch
    constexpr int R1 = EAGER ? 32 : 16;         // rows per round
    static_assert(RB >= 1 && R1 <= 64, "one row per lane");
    const int tid = threadIdx.x, lane = tid & 63;
    const int stride = geo.stride, ncol = geo.ncol;
    double acc[MAXCH], eta = 0.0, rho = INFINITY;
#pragma unroll
    for (int ch = 0; ch < MAXCH; ++ch) acc[ch] = 0.0;
    int nrel = 0;
    bool gave_up = false;
    for (int r0 = 0; r0 < n; r0 += R1) {
        const int nr = min(R1, n - r0);   // uniform
        const int rb = row0 + r0;
        const int lrow = lane < nr ? (rb + lane) * stride : kOffRange;
        double rho_r, eta_l = 0.0, v[EAGER ? LB : 1];
        if constexpr (GRAN) {
            u32x4 gr;
            for (unsigned spins = 0;; ++spins) {
                asm volatile("" ::: "memory");
                gr = ld_gran(rows, lrow);
                if (__all(lane >= nr || gran_ok(gr, tag))) break;
                MPPI_SPIN_OR_GIVE_UP_L(spins, deadline, tmo, lane, gave_up = true);
            }
            rho_r = gran_val(gr);
        } else if constexpr (!EAGER) {
            rho_r = ld_wt(rows, lrow);
        } else {
            rho_r = ld_wt(rows, lrow);
            eta_l = ld_wt(rows, lrow + 1);
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int i = j / MAXCH, col = tid + (j % MAXCH) * NT;
                v[j] = ld_wt(rows, (i < nr && col < ncol) ? (rb + i) * stride + 1 + col : kOffRange);
            }
        }
        const double rho_l = lane < nr ? rho_r : INFINITY;
        const double rnew = min_raw_f64(rho, wave_min_f64(rho_l));
        double s_l = 0.0;
        if (lane < nr) {
            const double s = exp((rnew - rho_l) * inv_lambda);
            s_l = s >= kMergeFloor ? s : 0.0;
        }
        const unsigned long long rel = __ballot(s_l != 0.0);   // rows that carry weight (uniform)
        const int nrr = __popcll(rel);
        nrel += nrr;
        if (rnew < rho && rho != INFINITY) {  // uniform: rescale the running sums to the new minimum
            const double f = exp((rnew - rho) * inv_lambda);
#pragma unroll
            for (int ch = 0; ch < MAXCH; ++ch) acc[ch] *= f;
            eta *= f;
        }
        rho = rnew;
        if constexpr (EAGER) {
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int i = j / MAXCH, ch = j % MAXCH;
                if (i < nr) {
                    const double s = readlane_f64(s_l, i);
                    if (s != 0.0) {
                        acc[ch] = fma(s, v[j], acc[ch]);
                        if (ch == 0) eta = fma(s, readlane_f64(eta_l, i), eta);
                    }
                }
            }
        } else {
            // lane k < nrr: the round's k-th weighted row (ascending)
            const int krow = lane < nrr ? select_bit(rel, lane) : 0;
            for (int b0 = 0; b0 < nrr; b0 += RB) {
                const bool eta_on = b0 == 0 && lane < nrr;
                const int eidx = eta_on ? (rb + krow) * stride + 1 : kOffRange;
                double x[LB];
                if constexpr (GRAN) {
                    u32x4 ge, gv[LB];
                    for (unsigned spins = 0;; ++spins) {
                        asm volatile("" ::: "memory");
                        ge = ld_gran(rows, eidx);
                        bool ok = !eta_on || gran_ok(ge, tag);
#pragma unroll
                        for (int j = 0; j < LB; ++j) {
                            const int i = b0 + j / MAXCH, col = tid + (j % MAXCH) * NT;
                            const bool on = i < nrr && col < ncol;
                            gv[j] = ld_gran(rows, on ? (rb + __builtin_amdgcn_readlane(krow, i)) * stride + 1 + col
                                                     : kOffRange);
                            ok = ok && (!on || gran_ok(gv[j], tag));
                        }
                        if (__all(ok)) break;
                        MPPI_SPIN_OR_GIVE_UP_L(spins, deadline, tmo, lane, gave_up = true);
                    }
                    if (eta_on) eta_l = gran_val(ge);
#pragma unroll
                    for (int j = 0; j < LB; ++j) x[j] = gran_val(gv[j]);
                } else {
                    if (b0 == 0) eta_l = ld_wt(rows, eidx);
#pragma unroll
                    for (int j = 0; j < LB; ++j) {
                        const int i = b0 + j / MAXCH, col = tid + (j % MAXCH) * NT;
                        x[j] = ld_wt(rows, (i < nrr && col < ncol)
                                               ? (rb + __builtin_amdgcn_readlane(krow, i)) * stride + 1 + col
                                               : kOffRange);
                    }
                }
#pragma unroll
                for (int j = 0; j < LB; ++j) {
                    const int i = b0 + j / MAXCH, ch = j % MAXCH;
                    if (i < nrr) {
                        const double s = readlane_f64(s_l, __builtin_amdgcn_readlane(krow, i));
                        acc[ch] = fma(s, x[j], acc[ch]);
                        if (ch == 0) eta = fma(s, readlane_f64(eta_l, i), eta);
                    }
                }
            }
        }
    }
    if (failed) *failed = __syncthreads_or(gave_up);
    if constexpr (final) {
        put_final<NT, MAXCH>(rho, acc, eta, nrel, geo, sm, out_row, w_eps_out);
    } else {
        auto put = [&](int col, double x) {  // col 0 = rho, 1 = eta, 2 + j = N[j]
            if constexpr (GRAN) st_gran(*out_wt, out_idx * stride + col, x, tag);
            else st_wt(*out_wt, out_idx * stride + col, x);
        };
#pragma unroll
        for (int ch = 0; ch < MAXCH; ++ch) {
            const int col = tid + ch * NT;
            if (col >= ncol) continue;
            if (col == 0) put(0, rho);
            put(1 + col, acc[ch]);
        }
    }
}

// Single-level finish for the usual regime (few weighted rows, S spread >> lambda):
// read rho of EVERY workgroup row (n <= kDirectRows), and when at most
// kDirectMax rows carry weight relative to the global minimum, merge exactly
// those rows in ascending order straight from the workgroup slab — one hand-off
// on the critical path instead of two.  Returns false (uniformly) when more rows
// carry weight; the caller then merges through the group rows.  Wave-local
// like merge_rows_block; the result goes out as in a final merge.
template <int NT, int MAXCH, bool GRAN, class SM>
__device__ __forceinline__ bool direct_merge(__amdgpu_buffer_rsrc_t rows, int n, const RowGeo& geo,
                                             double inv_lambda, SM& sm, double* out_row, double* w_eps_out,
                                             unsigned tag, unsigned* tmo, unsigned long long* dbg = nullptr) {
    constexpr int P = kDirectRows / 64;
    constexpr int LB = 16;                      // loads per batch per thread
    constexpr int RB = LB / MAXCH;              // rows per load batch
    const int tid = threadIdx.x, lane = tid & 63;
    const int stride = geo.stride, ncol = geo.ncol;
    // phase 1: rho of row lane + 64 j in slot j
    double rho_l[P];
    if constexpr (GRAN) {
        // ONE wave polls (a hop's latency sits in the polling CU's memory queue:
        // MI355X guide, polling-cost / handoff-1to1) and hands the values over in LDS
        if (tid < 64) {
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
                MPPI_SPIN_OR_GIVE_UP(spins, tmo, lane);
            }
#pragma unroll
            for (int j = 0; j < P; ++j) sm.rho[lane + 64 * j] = lane + 64 * j < n ? gran_val(gr[j]) : INFINITY;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < P; ++j) rho_l[j] = sm.rho[lane + 64 * j];
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
    for (int j = 1; j < P; ++j) m = min_raw_f64(m, rho_l[j]);
    const double rho = wave_min_f64(m);
    double s_l[P];
    unsigned long long rel[P];
    int nrel = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const double s = exp((rho - rho_l[j]) * inv_lambda);
        s_l[j] = (lane + 64 * j < n && s >= kMergeFloor) ? s : 0.0;
        rel[j] = __ballot(s_l[j] != 0.0);
        nrel += __popcll(rel[j]);
    }
    // Phase 2 spreads the weighted rows over row groups when the merged columns
    // fill less than the workgroup (one column chunk: G = NT / ncol groups of
    // ncol threads, group g taking every G-th row), so one batch of loads covers
    // kDirectMax * G rows; up to two batches (and 64 rows, one lane each) stay
    // direct.  With one group (config 3's 129 columns) the measured optimum is
    // one batch of 16 rows (the group mergers' overlap wins beyond it).
    const int G = MAXCH == 1 ? max(1, NT / ncol) : 1;
    if (nrel > (G > 1 ? min(64, 2 * kDirectMax * G) : kDirectMax)) return false;
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
    STAMP(13, NOW());
    // phase 2: eta and the (row, column chunk) entries of the weighted rows
    double acc[MAXCH], eta = 0.0, eta_k = 0.0;
#pragma unroll
    for (int ch = 0; ch < MAXCH; ++ch) acc[ch] = 0.0;
    if (G == 1) {
        // one group: the rows of a batch are wave-uniform (v_readlane); eta as a
        // scalar in the same row order as column 0
        for (int b0 = 0; b0 < nrel; b0 += RB) {
            double v[LB];
            if constexpr (GRAN) {
                const bool eta_on = b0 == 0 && mine;
                u32x4 ge, gv[LB];
                for (unsigned spins = 0;; ++spins) {
                    asm volatile("" ::: "memory");
                    ge = ld_gran(rows, eta_on ? row * stride + 1 : kOffRange);
                    bool ok = !eta_on || gran_ok(ge, tag);
#pragma unroll
                    for (int j = 0; j < LB; ++j) {
                        const int i = b0 + j / MAXCH, col = tid + (j % MAXCH) * NT;
                        const bool on = i < nrel && col < ncol;
                        gv[j] = ld_gran(rows, on ? __builtin_amdgcn_readlane(row, i) * stride + 1 + col : kOffRange);
                        ok = ok && (!on || gran_ok(gv[j], tag));
                    }
                    if (__all(ok)) break;
                    MPPI_SPIN_OR_GIVE_UP(spins, tmo, lane);
                }
                if (eta_on) eta_k = gran_val(ge);
#pragma unroll
                for (int j = 0; j < LB; ++j) v[j] = gran_val(gv[j]);
            } else {
                if (b0 == 0) eta_k = ld_wt(rows, mine ? row * stride + 1 : kOffRange);
#pragma unroll
                for (int j = 0; j < LB; ++j) {
                    const int i = b0 + j / MAXCH, col = tid + (j % MAXCH) * NT;
                    v[j] = ld_wt(rows, (i < nrel && col < ncol) ? __builtin_amdgcn_readlane(row, i) * stride + 1 + col
                                                                 : kOffRange);
                }
            }
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int i = b0 + j / MAXCH, ch = j % MAXCH;
                if (i < nrel) {
                    const double s = readlane_f64(sk, i);
                    acc[ch] = fma(s, v[j], acc[ch]);
                    if (ch == 0) eta = fma(s, readlane_f64(eta_k, i), eta);
                }
            }
        }
    } else {
        // G groups of ncol threads (one column chunk), group g taking weighted rows
        // g, g + G, ...: the row of a load varies by lane and comes through
        // ds_bpermute, read for every lane before any per-lane test (a cross-lane
        // read returns nothing from a lane the EXEC mask has off)
        const int grp = tid / ncol, gcol = tid - grp * ncol;
        const bool active = grp < G;
        for (int b0 = 0; b0 < nrel; b0 += RB * G) {
            double v[LB], sf[LB];
            int roff[LB];
            bool on[LB];
#pragma unroll
            for (int j = 0; j < LB; ++j) {
                const int i = b0 + grp + G * j;
                on[j] = active && i < nrel;
                const int r = __builtin_amdgcn_ds_bpermute(min(i, 63) << 2, row);
                sf[j] = __shfl(sk, min(i, 63));
                roff[j] = on[j] ? r * stride + 1 + gcol : kOffRange;
            }
            if constexpr (GRAN) {
                u32x4 gv[LB];
                for (unsigned spins = 0;; ++spins) {
                    asm volatile("" ::: "memory");
                    bool ok = true;
#pragma unroll
                    for (int j = 0; j < LB; ++j) {
                        gv[j] = ld_gran(rows, roff[j]);
                        ok = ok && (!on[j] || gran_ok(gv[j], tag));
                    }
                    if (__all(ok)) break;
                    MPPI_SPIN_OR_GIVE_UP(spins, tmo, lane);
                }
#pragma unroll
                for (int j = 0; j < LB; ++j) v[j] = gran_val(gv[j]);
            } else {
#pragma unroll
                for (int j = 0; j < LB; ++j) v[j] = ld_wt(rows, roff[j]);
            }
#pragma unroll
            for (int j = 0; j < LB; ++j)
                if (on[j]) acc[0] = fma(sf[j], v[j], acc[0]);
        }
        // fold the groups' column sums in group order; eta is column 0
        if (active) sm.part[tid] = acc[0];
        __syncthreads();
        if (grp == 0) {
            double a = sm.part[gcol];
            for (int g = 1; g < G; ++g) a += sm.part[g * ncol + gcol];
            acc[0] = a;
            if (tid == 0) sm.red[0] = a;
        }
        __syncthreads();
        eta = sm.red[0];
    }
    STAMP(14, NOW());
    put_final<NT, MAXCH>(rho, acc, eta, nrel, geo, sm, out_row, w_eps_out);
    return true;
}

// Arrive on `counter` after this workgroup's write-through stores; true in
// every thread of the workgroup that arrived last (which re-arms the counter).
// sc1 loads alone stand in for the acquire only at one workgroup per CU (the
// measured form, MI355X guide "Valid forms"); with `acquire` (larger grids)
// the last arriver also runs an agent-scope acquire before the barrier.
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
#define CX(i, j) { const double lo = min_raw_f64(v[i], v[j]), hi = max_raw_f64(v[i], v[j]); v[i] = lo; v[j] = hi; }
    CX(4, 9) CX(3, 8) CX(2, 7) CX(1, 6) CX(0, 5) CX(1, 4) CX(6, 9) CX(0, 3) CX(5, 8) CX(0, 2)
    CX(3, 6) CX(7, 9) CX(0, 1) CX(2, 4) CX(5, 7) CX(8, 9) CX(1, 2) CX(4, 6) CX(7, 8) CX(3, 5)
    CX(2, 5) CX(6, 8) CX(1, 3) CX(4, 7) CX(2, 3) CX(6, 7) CX(3, 4) CX(5, 6) CX(4, 5)
#undef CX
    return v[5];
}

// scipy.ndimage.median_filter(size=10, mode='reflect') of column d of the
// T x du array sm.weps at row t (control.py:319-327, window [t-5, t+4]; one
// reflection suffices for T >= 5).
template <class SM>
__device__ __forceinline__ double median_at(const SM& sm, int t, int d, int T, int du) {
    double v[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        int m = t - 5 + i;
        m = m < 0 ? -m - 1 : m;
        m = m >= T ? 2 * T - 1 - m : m;
        v[i] = sm.weps[m * du + d];
    }
    return median10(v);
}

// ------------------------------------------------------------------ Philox

// Philox4x32-10 (Salmon et al., SC'11).  Each round's two 32 x 32 -> 64-bit
// products are one v_mad_u64_u32 apiece (the 64-bit product of zero-extended
// words, which the compiler emits as one), not a v_mul_lo_u32 + v_mul_hi_u32
// pair: half the quarter-rate multiplies.  The round's two three-way XORs
// (hi ^ word ^ key) are one v_bitop3_b32 each (truth table 0x96), the key word
// from an SGPR (it must be wave-uniform: the "s" constraint takes lane 0's
// value).  With the hardware Box-Muller below: 13.4 -> 8.35 us for config 3's
// draw (profiles/r11/philox_ab.txt).
__device__ __forceinline__ unsigned long long mul_wide(unsigned a, unsigned m) {
    return (unsigned long long)a * m;
}
__device__ __forceinline__ unsigned xor3(unsigned a, unsigned b, unsigned k) {
    unsigned r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
__device__ __forceinline__ uint4 philox4x32_10(uint4 ctr, uint2 key) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const unsigned long long p0 = mul_wide(ctr.x, 0xD2511F53u);
        const unsigned long long p1 = mul_wide(ctr.z, 0xCD9E8D57u);
        ctr = make_uint4(xor3((unsigned)(p1 >> 32), ctr.y, key.x), (unsigned)p1,
                         xor3((unsigned)(p0 >> 32), ctr.w, key.y), (unsigned)p0);
        key.x += 0x9E3779B9u;
        key.y += 0xBB67AE85u;
    }
    return ctr;
}

// Two standard normals from two 32-bit uniforms (Box-Muller) on the hardware
// transcendentals: v_log_f32 (log2), v_sqrt_f32, and v_sin_f32 / v_cos_f32, whose
// input is in revolutions — exactly u1, so no 2 pi scaling and no range
// reduction.  Returned WITHOUT the constant sqrt(2 ln 2) (kBoxMullerScale): the
// callers fold it into their Cholesky factor, so the value is
//   sqrt(-log2 u0) (cos 2 pi u1, sin 2 pi u1) = z / sqrt(2 ln 2).
// u0 = (a + 1) 2^-32 in [2^-32, 1] (a normal float: no denormal path) is one fma:
// scaling by 2^-32 is exact, so fma(a, 2^-32, 2^-32) rounds the same real as
// (float(a) + 1) * 2^-32, and it never exceeds 1 (float(a) <= 2^32, and 2^32 + 1
// rounds to 2^32), so no clamp.  The negation of log2 u0 <= 0 is a source modifier.
constexpr double kBoxMullerScale = 1.1774100225154747;   // sqrt(2 ln 2)
__device__ __forceinline__ float2 box_muller(unsigned a, unsigned b) {
    const float inv = 2.3283064365386963e-10f;  // 2^-32
    const float u0 = fmaf((float)a, inv, inv), u1 = (float)b * inv;
    const float r = __builtin_amdgcn_sqrtf(-__builtin_amdgcn_logf(u0));
    return make_float2(r * __builtin_amdgcn_cosf(u1), r * __builtin_amdgcn_sinf(u1));
}

}  // namespace mppi

namespace mppi {

// ------------------------------------------------------ node-level exchange
// Multi-GPU (one process per GPU, one node) without a collective call per step:
// the launch's final workgroup writes this rank's merged row {rho, eta, N} as
// tagged granules into slot [parity][rank] of EVERY rank's inbox (IPC-mapped
// device memory; remote ranks over xGMI, system-scope stores), then polls its
// own inbox until the world rows of this step carry the tag and merges them in
// rank order with the same granule merge as inside a launch.  The pattern is
// RCCL's LL protocol (flagged stores into a peer's buffer); the inbox is
// uncached device memory, so a poll never reads a stale L2 line.  Tags come
// from a per-rank exchange epoch advanced once per exchange launch: every rank
// runs the same launches, so the epochs agree.  Two parity halves: a rank can
// write step n + 1 while a slower peer still reads step n, never step n + 2
// (it needs that peer's step n + 1 row first).
constexpr int kMaxWorld = MPPI_MAX_WORLD;
struct XDesc {
    const void* peer[kMaxWorld];   // inbox base of every rank (own rank: local memory)
    double* row;                   // this rank's merged row, written by the launch's final merge
    unsigned* epoch;               // this rank's exchange epoch
    int rank, world, bytes;        // bytes: inbox size (2 x world rows of `stride` granules, 2 x world statuses)
    unsigned timeout_ticks;        // the exchange polls' bound in s_memrealtime ticks (10 ns; 0: the ~1 s spin
                                   // bound), MPPI_EXCHANGE_TIMEOUT_US at attach
};
// host timeout word, cause bits: an in-launch hand-off of this launch timed out (its results are invalid; not
// retryable) / the step's exchange failed on every rank (retryable over the all-gather) / this rank had every
// row but not every rank's status in time, so the other ranks may have applied the step (not retryable)
constexpr unsigned kTmoLocal = 1u, kTmoExchange = 2u, kTmoSplit = 4u;
__device__ __forceinline__ void st_gran_sys(__amdgpu_buffer_rsrc_t r, int idx, double v, unsigned tag) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const u32x4 x = {(unsigned)b, tag, (unsigned)(b >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(x, r, idx * 16, 0, kSC1 | 1);   // sc0 sc1: system scope
}

// Called by the final workgroup after its merge wrote x.row (put_final ends with
// a barrier, so the row is visible to the whole workgroup).
//
// Failure semantics (a rank late past the bound, or gone): after the row round,
// every rank writes a status granule (+1: it had every row in time, -1: not) to
// every inbox and polls all of them; the step holds only if every rank reports
// +1.  A rank that gave up wrote its -1 before leaving, so a late rank, whenever
// it arrives, finds that status next to the rows it needs: every rank of the
// step reaches the same verdict.  On failure the launch reports kTmoExchange
// (the host raises MPPI_E_EXCHANGE and keeps the nominal: no update is applied)
// and the caller runs the step again over the collective fallback.  The epoch
// advances either way, so the ranks stay in step for the next exchange.
//
// Two halves, so the caller can compute the fused update while the statuses
// travel: exchange_send_merge (rows out, merge, this rank's status out; returns
// the step's tag) and exchange_verdict (the statuses in).  The update written in
// between goes only to the ping-pong block the host has not yet made current and
// to outputs the host reads after the verdict; on failure the host keeps the
// block it had and ignores them.
template <int NT, int MAXCH, class SM>
__device__ __forceinline__ unsigned exchange_send_merge(const XDesc& x, const RowGeo& geo, double inv_lambda, SM& sm,
                                                        double* w_eps_out, unsigned* tmo) {
    // the previous exchange launch's final store; kernel boundaries order it
    const unsigned tag = (unsigned)__builtin_amdgcn_readfirstlane((int)*x.epoch) + 1u;
    const int par = (int)(tag & 1u), stride = geo.stride;
    for (int idx = threadIdx.x; idx < stride; idx += NT) {
        const double v = x.row[idx];
        for (int p = 0; p < x.world; ++p)
            st_gran_sys(rows_rsrc(x.peer[p], x.bytes), (par * x.world + x.rank) * stride + idx, v, tag);
    }
    bool late = false;
    const unsigned long long dl = x.timeout_ticks ? __builtin_amdgcn_s_memrealtime() + x.timeout_ticks : 0ull;
    merge_rows_block<NT, MAXCH, true, true>(rows_rsrc(x.peer[x.rank], x.bytes), par * x.world, x.world, geo,
                                            inv_lambda, sm, nullptr, 0, nullptr, w_eps_out, tag, nullptr, dl, &late);
    // this rank's own row is invalid if an in-launch hand-off of this launch timed out
    late = __syncthreads_or(late || (threadIdx.x == 0 && tmo &&
                                     __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u));
    const int sbase = 2 * x.world * stride + par * x.world;   // status granules follow the rows: [parity][rank]
    if ((int)threadIdx.x < x.world)
        st_gran_sys(rows_rsrc(x.peer[threadIdx.x], x.bytes), sbase + x.rank, late ? -1.0 : 1.0, tag);
    return tag;
}

template <int NT>
__device__ __forceinline__ bool exchange_verdict(const XDesc& x, const RowGeo& geo, unsigned tag, unsigned* tmo) {
    const int par = (int)(tag & 1u);
    const int sbase = 2 * x.world * geo.stride + par * x.world;
    const int tid = threadIdx.x, lane = tid & 63;
    bool bad = false, split = false;
    if (tid < 64) {   // wave 0 polls every rank's status (world <= 64)
        const __amdgpu_buffer_rsrc_t own = rows_rsrc(x.peer[x.rank], x.bytes);
        u32x4 g;
        bool missing = false;
        const unsigned long long dl = x.timeout_ticks ? __builtin_amdgcn_s_memrealtime() + x.timeout_ticks : 0ull;
        for (unsigned spins = 0;; ++spins) {
            asm volatile("" ::: "memory");
            g = ld_gran(own, lane < x.world ? sbase + lane : kOffRange);
            if (__all(lane >= x.world || gran_ok(g, tag))) break;
            MPPI_SPIN_OR_GIVE_UP_L(spins, dl, nullptr, lane, missing = true);
        }
        bad = __any(lane < x.world && !(gran_ok(g, tag) && gran_val(g) > 0.0)) || missing;
        // A status that never came while this rank's own is not a -1: the ranks whose statuses all arrived may
        // have applied the step, so re-running it here would pair this rank's retry with their next step.
        // Only a rank that reported -1 itself knows every rank fails (each waits for, or times out on, its -1).
        split = missing && !__any(lane == x.rank && gran_ok(g, tag) && gran_val(g) < 0.0);
    }
    bad = __syncthreads_or(bad);
    split = __syncthreads_or(split);
    if (tid == 0) {
        if (bad)
            __hip_atomic_store(tmo + 1, split ? kTmoExchange | kTmoSplit : kTmoExchange, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        *x.epoch = tag;
    }
    return !bad;
}

}  // namespace mppi

// Issue fairness between workgroups that share a CU.  The SIMD arbiter serves
// the oldest ready wave first, so of two co-resident rollout waves the younger
// one only fills the older one's issue gaps and then finishes alone at the
// single-wave rate (measured on the chain kernel: older workgroups 174 us,
// younger 277 us).  Each workgroup draws a per-CU ticket with one relaxed
// atomic (co-resident workgroups draw consecutive tickets: different
// parities), and waves raise their priority in alternate real-time phases of
// 2^kPrioShift ticks (100 MHz: ~41 us), the phase flipped by the ticket parity.
// Priority steers scheduling only; no result depends on it.
constexpr int kCuSlots = 2048;   // (XCC, SE, SH, CU) keys
constexpr int kPrioShift = 12;
__device__ __forceinline__ unsigned cu_key() {
    const unsigned hw = __builtin_amdgcn_s_getreg(0xF804);    // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(0xF814);   // XCC_ID
    return ((xcc & 7u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 0xFu);
}
// Thread 0 draws the ticket into *s_parity (read after the caller's next barrier).
__device__ __forceinline__ void draw_cu_ticket(unsigned* cu_ctr, unsigned* s_parity) {
    if (threadIdx.x == 0)
        *s_parity = __hip_atomic_fetch_add(cu_ctr + cu_key(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u;
}
__device__ __forceinline__ void fair_priority(unsigned parity) {
    if ((((unsigned)__builtin_amdgcn_s_memrealtime() >> kPrioShift) & 1u) ^ parity)
        __builtin_amdgcn_s_setprio(1);
    else
        __builtin_amdgcn_s_setprio(0);
}

