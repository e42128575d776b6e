// mppi_npgauss.hip — the reference's noise draw, NumPy's legacy global-RNG Gaussian stream, generated on the
// MI355X bit for bit (values and the RNG state left behind).
//
// control.py:163 draws eps with np.random.multivariate_normal(mu, Sigma, (K, T)) on the legacy RandomState:
// MT19937 words -> NumPy's legacy doubles (two words each) -> the polar method with rejection (legacy_gauss:
// one attempt = four words, accepted when 0 < r2 < 1, then a pair f x2, f x1 with f = sqrt(-2 log r2 / r2))
// -> the Sigma transform.  Sequential in NumPy; here every phase is parallel:
//
//   np_seq_kernel    the first 34 key arrays (blocks) after the state's: the word windows the jumps read.
//   np_jumpn_kernel  the state of every generator stream's start: MT19937 is linear over GF(2), so the block
//                    J words on is sum_d phi_d F^d(key) with phi = x^J mod P (P: the characteristic
//                    polynomial, found and powered on the host, np_legacy_gauss.c) and F^d(key) the window
//                    [d, d + 624) of the word sequence (Haramoto et al. 2008, the window form): a table product
//                    over 4-bit chunks of phi, the 16 entries of a chunk in each lane's registers.
//   np_gen_kernel    one workgroup per stream twists its range of blocks; the words 227 apart form one chain
//                    of the twist, so a thread computes three of them from the previous block (one mix each,
//                    in registers): one LDS round trip and one barrier per block.
//   np_write_kernel  the attempts, 2048 consecutive ones per workgroup; the index of the workgroup's first pair
//                    by look-back over its predecessors' published counts (one pass, no separate count and
//                    scan); each accepted pair's place from it; f with glibc's log
//                    reproduced (np_glibc_log.h), IEEE division and square root; the transform of the drop-in
//                    (a scaled column permutation, hostrng.monomial_transform, or for du = 2 any matrix through
//                    the host BLAS's 2-term rounding, hostrng.dot2_model) and the rounding to fp32, into the
//                    engine's noise layout for this rank's samples.
//   np_state_kernel  the state NumPy leaves: the key array holding the last consumed word, its position, and
//                    the cached Gaussian of an odd count.
//
// No contraction anywhere in this file: NumPy's r2 = x1 x1 + x2 x2, the transform's multiply and add are
// separately rounded; the log's fused multiply-adds are explicit.
//
// C ABI: include/mppi_rocm.h (mppi_np_*).  Reference: control.py:154-164.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <algorithm>
#include <vector>

#include "mppi_host.h"
#include "mppi_rocm.h"
#include "np_glibc_log.h"

#pragma clang fp contract(off)

namespace {

using mppi_host::fail;

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatA = 0x9908b0dfu, kUp = 0x80000000u, kLo = 0x7fffffffu;
constexpr int kDeg = 19937;
constexpr int kPolyWords = MPPI_NP_POLY_WORDS;        // 312 x 64 bits: a polynomial of degree < 19937
constexpr int kSeqBlocks = (kDeg + kN) / kN + 1;      // 34: the windows d + j < 19937 + 624 of the jumps
constexpr int kNT = 256;                              // threads of the attempt kernels
constexpr int kR = kN - kM;                           // 227: the twist's dependency distance
constexpr int kTT = 256;                              // threads of the twist kernels: thread t < 227 owns words t,
                                                      // t + 227 and (t < 170) t + 454 (twist3)
constexpr int kNibS = 32;                             // table jump: streams per workgroup
constexpr int kChunks = (kDeg + 3) / 4;               // 4-bit chunks of a jump polynomial
constexpr int kJNT = 640;                             // table jump threads: output word i per lane (< 624)
constexpr int kJTableWGs = 512;                       // table jump: chunk ranges x stream groups, about
constexpr int kAttRounds = 8;                         // attempts per thread, interleaved: attempt a0 + 256 r + t
constexpr int kAttPerWG = kNT * kAttRounds;

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
    const uint32_t y = (a & kUp) | (b & kLo);
    return (y >> 1) ^ ((0u - (y & 1u)) & kMatA);
}

// The key array after o (LDS), thread t's words.  NumPy's twist (in place, word order) is k[i] = o[i + 397] ^
// mix(o[i], o[i + 1]) for i < 227, k[i] = k[i - 227] ^ mix(o[i], o[i + 1]) up to 622, and k[623] =
// k[396] ^ mix(o[623], k[0]).  The words 227 apart are one chain, so thread t (< 227) computes k[t], k[t + 227]
// and k[t + 454] in order, each from its predecessor in a register: one mix per word, every LDS read of the block
// issued at once.  Word 623 is thread 169's third (its second is k[396]); the new k[0] it needs is recomputed
// from broadcast reads by every lane (cheaper than a branch on one lane).  Threads t >= 227 compute garbage that
// twist_block does not store.
__device__ __forceinline__ void twist3(const uint32_t* o, int t, uint32_t k[3]) {
    const int u = min(t, kR - 1);
    const uint32_t a0 = o[u], a1 = o[u + 1], am = o[u + kM];
    const uint32_t b0 = o[u + kR], b1 = o[u + kR + 1];
    const uint32_t c0 = o[min(u + 2 * kR, kN - 1)], c1 = o[min(u + 2 * kR + 1, kN - 1)];
    const uint32_t z0 = o[0], z1 = o[1], zm = o[kM];
    k[0] = am ^ mt_mix(a0, a1);
    k[1] = k[0] ^ mt_mix(b0, b1);
    const uint32_t knew0 = zm ^ mt_mix(z0, z1);
    k[2] = k[1] ^ mt_mix(c0, u == kN - 1 - 2 * kR ? knew0 : c1);
}

// words thread t stores: k[t], k[t + 227] for t < 227, k[t + 454] for t < 170
__device__ __forceinline__ int twist_words(int t) { return t < kN - 2 * kR ? 3 : t < kR ? 2 : 0; }

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ double legacy_double(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// attempt a: words [base + 4a, base + 4a + 4) of the untempered block sequence
__device__ __forceinline__ void attempt(const uint32_t* __restrict__ words, long long base, long long a, double& x1,
                                       double& x2, double& r2) {
    const uint32_t* w = words + base + 4 * a;
    const uint32_t w0 = temper(w[0]), w1 = temper(w[1]), w2 = temper(w[2]), w3 = temper(w[3]);
    x1 = 2.0 * legacy_double(w0, w1) - 1.0;
    x2 = 2.0 * legacy_double(w2, w3) - 1.0;
    r2 = x1 * x1 + x2 * x2;
}

__device__ __forceinline__ bool accepted(double r2) { return r2 < 1.0 && r2 != 0.0; }

struct NpResult {
    long long last_attempt;   // the attempt of the last wanted pair
    double last_fx1;          // its f x1 (cached by an odd count)
    long long total;          // accepted attempts among the generated ones
    int status;               // 1: fewer than the pairs wanted, 2: the look-back gave up (not written; the host
                              // draws again); np_state_kernel reports 3 if the last pair was not found
    int pad;
};

struct NpShape {
    float* out;
    unsigned per_k, du;         // T du normals per sample, du per step
    unsigned k_offset, K_local;
    long long st, sk, sd;       // out element (t, k - k_offset, d)
    int src[MPPI_NP_MAX_DU];
    double scale[MPPI_NP_MAX_DU], mean[MPPI_NP_MAX_DU];
    int dot2;                   // du = 2, a general transform: x_d = fma(z1, mat[2 + d], z0 mat[d]) (mppi_np_target)
    double mat[4];
};

// ------------------------------------------------------------------ generation
// One twist of buffer o into n (LDS) and, with kStore, into out (global); a barrier must follow before n is read.
template <bool kStore>
__device__ __forceinline__ void twist_block(const uint32_t* o, uint32_t* n, uint32_t* __restrict__ out, int t) {
    uint32_t k[3];
    twist3(o, t, k);
    const int m = twist_words(t);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        if (r < m) {
            n[t + r * kR] = k[r];
            if (kStore) out[t + r * kR] = k[r];
        }
}

__global__ __launch_bounds__(kTT) void np_seq_kernel(const uint32_t* __restrict__ key, uint32_t* __restrict__ seq) {
    __shared__ uint32_t buf[2][kN];
    for (int q = threadIdx.x; q < kN; q += kTT) {
        const uint32_t v = key[q];
        buf[0][q] = v;
        seq[q] = v;
    }
    __syncthreads();
    for (int b = 1; b < kSeqBlocks; ++b) {
        twist_block<true>(buf[(b - 1) & 1], buf[b & 1], seq + (size_t)b * kN, threadIdx.x);
        __syncthreads();   // the next twist reads this block and writes the buffer this one read
    }
}

// The same jumps as a table product (the Four Russians' method over GF(2), 4-bit chunks).  Output word i of
// jump j is the XOR over the chunks c of T_c[nib_j(c)][i], where nib_j(c) holds the polynomial's bits 4c .. 4c + 3
// and T_c[v][i] = XOR of seq[4c + b + i] over the set bits b of v: lane i builds its 16 table entries of a chunk in
// registers from four sequence words, and each of the workgroup's 32 jumps picks its entry by the chunk's
// (uniform) nibble — a register-indexed move and an XOR per jump and chunk, instead of ~2 LDS reads and XORs per
// set bit.  Workgroup (r, g): chunks [r cpw, (r + 1) cpw) for jumps [32 g, 32 g + 32); each writes its partial
// XOR of every output word, np_gen_kernel XORs the R parts.
__global__ __launch_bounds__(kJNT) void np_jumpn_kernel(const uint32_t* __restrict__ seq, const uint32_t* __restrict__ nibs,
                                                        int G, int cpw, int njumps, int R, uint32_t* __restrict__ parts) {
    extern __shared__ uint32_t s_w[];   // sequence words [4 c0, 4 c1 + 627)
    const int r = blockIdx.x, g = blockIdx.y, i = threadIdx.x;
    const int c0 = r * cpw, c1 = min(c0 + cpw, kChunks);
    const int w0 = 4 * c0, nw = 4 * (c1 - c0) + kN + 3;
    for (int q = i; q < nw; q += kJNT) s_w[q] = seq[w0 + q];
    __syncthreads();
    uint32_t o[kNibS];
#pragma unroll
    for (int j = 0; j < kNibS; ++j) o[j] = 0u;
    const int li = min(i, kN - 1);   // lanes past word 623 repeat it (never stored)
    for (int c = c0; c < c1; ++c) {
        const uint32_t* wp = s_w + 4 * (c - c0) + li;
        const uint32_t a = wp[0], b = wp[1], e = wp[2], d = wp[3];
        uint32_t T[16];
        T[0] = 0u;
        T[1] = a;
        T[2] = b;
        T[3] = a ^ b;
        T[4] = e;
        T[5] = e ^ a;
        T[6] = e ^ b;
        T[7] = e ^ T[3];
#pragma unroll
        for (int v = 0; v < 8; ++v) T[8 + v] = T[v] ^ d;
        // one word per jump, the nibble already extracted (< 16, set_jumps), scalar-loaded
        const uint32_t* nb = nibs + ((size_t)c * G + g) * kNibS;
#pragma unroll
        for (int j = 0; j < kNibS; ++j) o[j] ^= T[__builtin_amdgcn_readfirstlane(nb[j])];
    }
    if (i < kN) {
#pragma unroll
        for (int j = 0; j < kNibS; ++j) {
            const int jj = g * kNibS + j;
            if (jj < njumps) parts[((size_t)jj * R + r) * kN + i] = o[j];
        }
    }
}

// stream s: blocks [1 + P s, min(1 + P (s + 1), nblk)); stream 0 also writes block 0 (the state's key array)
__global__ __launch_bounds__(kTT) void np_gen_kernel(const uint32_t* __restrict__ key, const uint32_t* __restrict__ parts,
                                                     uint32_t* __restrict__ words, int P, int nblk, int nparts,
                                                     NpResult* res) {
    __shared__ uint32_t buf[2][kN];
    const int s = blockIdx.x, t = threadIdx.x;
    const int b0 = 1 + P * s, b1 = min(1 + P * (s + 1), nblk);
    constexpr int kQ = (kN + kTT - 1) / kTT;   // 3 words per thread in the coalesced prologue
    if (s == 0) {
        if (t == 0) {   // the draw's result, before np_write_kernel fills it
            res->last_attempt = -1;
            res->total = 0;
            res->status = 0;
        }
        for (int q = t; q < kN; q += kTT) {
            const uint32_t v = key[q];
            buf[0][q] = v;
            words[q] = v;
        }
        __syncthreads();
    } else {
        const uint32_t* base = parts + (size_t)(s - 1) * nparts * kN;
        uint32_t v[kQ];
        int qi[kQ];
#pragma unroll
        for (int r = 0; r < kQ; ++r) {
            v[r] = 0u;
            qi[r] = min(t + r * kTT, kN - 1);   // lanes past word 623 repeat it (not stored)
        }
        int h = 0;
        for (; h + 8 <= nparts; h += 8) {   // 8 parts x 3 words: 24 loads in flight
            uint32_t x[8][kQ];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int r = 0; r < kQ; ++r) x[u][r] = base[(size_t)(h + u) * kN + qi[r]];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int r = 0; r < kQ; ++r) v[r] ^= x[u][r];
        }
        for (; h < nparts; ++h)
#pragma unroll
            for (int r = 0; r < kQ; ++r) v[r] ^= base[(size_t)h * kN + qi[r]];
#pragma unroll
        for (int r = 0; r < kQ; ++r)
            if (t + r * kTT < kN) buf[1][t + r * kTT] = v[r];
        __syncthreads();
        twist_block<false>(buf[1], buf[0], nullptr, t);   // block P s, exactly
        __syncthreads();
    }
    int cur = 0;
    for (int b = b0; b < b1; ++b) {
        twist_block<true>(buf[cur], buf[cur ^ 1], words + (size_t)b * kN, t);
        __syncthreads();
        cur ^= 1;
    }
}

// ------------------------------------------------------------------ the polar method
// Workgroup look-back (single-pass prefix): workgroup w publishes its accepted-attempt count (kLookAgg) as soon
// as its attempts are in, then its inclusive prefix (kLookIncl) once wave 0 has summed the predecessors' counts
// back to the nearest published prefix, 64 workgroups per poll (kLookVoid: a predecessor gave up, and so does
// this workgroup).  A word: [epoch 24 | status 2 | value 38]; the
// draw's epoch tells this draw's words from an earlier draw's, so the array is not reset between draws.
// Workgroups are dispatched in order, so every predecessor a workgroup waits for is resident or done.
constexpr int kLookShift = 38;
constexpr unsigned long long kLookVal = (1ull << kLookShift) - 1ull;
constexpr unsigned long long kLookAgg = 1ull << kLookShift, kLookIncl = 2ull << kLookShift;
constexpr unsigned long long kLookVoid = 3ull << kLookShift, kLookStat = 3ull << kLookShift;
constexpr unsigned long long kLookEpoch = ~0ull << (kLookShift + 2);
constexpr int kLookPolls = 1 << 20;   // give up (status 2, the host draws again) rather than spin for ever

__device__ __forceinline__ void look_publish(unsigned long long* look, long long w, unsigned long long word) {
    __hip_atomic_store(look + w, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of workgroup w > 0: the exclusive prefix of its count (every lane returns it); -1 after kLookPolls polls
__device__ long long look_back(unsigned long long* look, long long w, unsigned long long epoch) {
    const int lane = threadIdx.x & 63;
    long long excl = 0, j = w - 1;
    for (int polls = 0; polls < kLookPolls; ++polls) {
        const long long idx = j - lane;
        unsigned long long v = idx >= 0 ? __hip_atomic_load(look + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : (epoch | kLookIncl);
        if ((v & kLookEpoch) != epoch) v = 0;   // an earlier draw's word: not published yet
        const unsigned long long incl = __ballot((v & kLookStat) == kLookIncl);
        const unsigned long long none = __ballot((v & kLookStat) == 0);
        const unsigned long long gone = __ballot((v & kLookStat) == kLookVoid);
        // lanes 0 .. the first inclusive prefix (or all 64) must be published
        const unsigned long long need = incl ? (2ull << (__builtin_ctzll(incl))) - 1ull : ~0ull;
        if (gone & need) return -1;
        if (none & need) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        long long part = ((1ull << lane) & need) ? (long long)(v & kLookVal) : 0;
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        excl += part;
        if (incl) return excl;
        j -= 64;
    }
    return -1;
}

// The attempts, their workgroup's count published and f computed (glibc's log reproduced, np_glibc_log.h; IEEE
// division and square root) while the look-back finds the workgroup's first pair.  The workgroup's normals m in [m0, m1) (NumPy's (K, T, du) order) are staged in
// LDS, then written through the transform in the engine's layout row by row: for each step t, the workgroup's
// samples are contiguous there, so consecutive threads write consecutive addresses (written straight from the
// attempts, every lane of a wave hit its own row: one cache line per 8 bytes).
// at most 128 VGPRs: four waves per SIMD (130 gave three)
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(4))) void np_write_kernel(const uint32_t* __restrict__ words, long long base, long long A,
                                                       unsigned long long* __restrict__ look,
                                                       unsigned long long epoch, const double* __restrict__ logd,
                                                       NpShape sh, long long pairs, long long n, int o, double cached,
                                                       NpResult* res) {
    __shared__ double s_log[NPLOG_NDATA];
    __shared__ int s_cnt[kAttRounds][kNT / 64];
    __shared__ long long s_qw;
    __shared__ double s_z[2 * kAttPerWG];
    __shared__ double s_next;   // dot2: the normal after this workgroup's (the next accepted pair's f x2)
    for (int i = threadIdx.x; i < NPLOG_NDATA; i += kNT) s_log[i] = logd[i];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long a0 = (long long)blockIdx.x * kAttPerWG + threadIdx.x;
    double x1[kAttRounds], x2[kAttRounds];   // r2 recomputed where f needs it (the same rounded operations)
    unsigned mask = 0;
#pragma unroll
    for (int r = 0; r < kAttRounds; ++r) {
        const long long a = a0 + (long long)r * kNT;
        double r2 = 2.0;
        if (a < A) attempt(words, base, a, x1[r], x2[r], r2);
        const bool acc = accepted(r2);
        mask |= (unsigned)acc << r;
        const unsigned long long bal = __ballot(acc);
        if (lane == 0) s_cnt[r][wave] = __popcll(bal);
    }
    __syncthreads();   // also publishes s_log
    const long long w = blockIdx.x;
    int agg = 0;   // the workgroup's accepted attempts
    for (int r = 0; r < kAttRounds; ++r)
        for (int v = 0; v < kNT / 64; ++v) agg += s_cnt[r][v];
    if (threadIdx.x == 0) look_publish(look, w, epoch | (w == 0 ? kLookIncl : kLookAgg) | (unsigned long long)agg);
    // local pair index of this thread's attempt in round r: all accepted attempts of the rounds before r, those of
    // round r in earlier waves, and those of earlier lanes of this wave; f while the predecessors publish
    int lq0 = 0;
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < kAttRounds; ++r) {
        const bool acc = (mask >> r) & 1u;
        const unsigned long long bal = __ballot(acc);
        int before = 0, round = 0;
        for (int v = 0; v < kNT / 64; ++v) {
            const int cw = s_cnt[r][v];
            before += v < wave ? cw : 0;
            round += cw;
        }
        const int lq = lq0 + before + __popcll(bal & lt);
        if (acc && lq < pairs) {
            const double r2 = x1[r] * x1[r] + x2[r] * x2[r];   // as attempt()
            const double f = sqrt(-2.0 * np_glibc_log(s_log, r2) / r2);
            s_z[2 * lq] = f * x2[r];       // normal o + 2 q: legacy_gauss returns f x2
            s_z[2 * lq + 1] = f * x1[r];   // o + 2 q + 1: and caches f x1
        }
        lq0 += round;
    }
    if (wave == 0) {   // the workgroup's first pair: the look-back
        if (w == 0) {
            if (lane == 0) s_qw = 0;
        } else {
            const long long ex = look_back(look, w, epoch);
            if (lane == 0) {
                if (ex >= 0) {
                    look_publish(look, w, epoch | kLookIncl | (unsigned long long)(ex + agg));
                } else {   // the look-back gave up: the draw is void, and the successors see it
                    look_publish(look, w, epoch | kLookVoid);
                    res->status = 2;
                }
                s_qw = ex;
            }
        }
        if (w == (long long)gridDim.x - 1 && lane == 0 && s_qw >= 0) {   // the last workgroup: the total
            res->total = s_qw + agg;
            if (s_qw + agg < pairs) res->status = 1;
        }
    }
    __syncthreads();   // s_qw and s_z
    const long long qw = s_qw;
    if (qw < 0) return;   // uniform
    const long long q0 = qw + agg;
    if (qw <= pairs - 1 && pairs - 1 < q0) {   // the last wanted pair is here (uniform): its attempt and f x1
        const int want = (int)(pairs - 1 - qw);
        int l0 = 0;
        for (int r = 0; r < kAttRounds; ++r) {   // the local indices again, as above
            const bool acc = (mask >> r) & 1u;
            const unsigned long long bal = __ballot(acc);
            int before = 0, round = 0;
            for (int v = 0; v < kNT / 64; ++v) {
                const int cw = s_cnt[r][v];
                before += v < wave ? cw : 0;
                round += cw;
            }
            if (acc && l0 + before + __popcll(bal & lt) == want) {
                res->last_attempt = a0 + (long long)r * kNT;
                res->last_fx1 = s_z[2 * want + 1];
            }
            l0 += round;
        }
    }
    // dot2: a step's two normals may straddle two workgroups; the workgroup holding the first writes the step,
    // and the second is then the next workgroup's first normal: its first accepted attempt's f x2, recomputed
    // here with the same operations (one or two attempts past this workgroup's, acceptance pi / 4)
    if (sh.dot2) {   // uniform
        if (threadIdx.x == 0 && q0 < pairs) {
            double y1 = 0.0, y2 = 0.0, rr = 2.0;
            for (long long a = (w + 1) * (long long)kAttPerWG; a < A; ++a) {
                attempt(words, base, a, y1, y2, rr);
                if (accepted(rr)) break;
            }
            const double r2 = y1 * y1 + y2 * y2;   // as attempt()
            s_next = y2 * sqrt(-2.0 * np_glibc_log(s_log, r2) / r2);
        }
        __syncthreads();
    }
    // normals [m0, m1) of this workgroup: pairs [qw, q0) below `pairs`; the cached Gaussian (m = 0) comes first
    const long long zb = o + 2 * qw;   // normal of s_z[0]
    const long long m0 = blockIdx.x == 0 ? 0 : zb;
    const long long m1 = min(o + 2 * min(q0, pairs), n);
    if (m1 <= m0) return;
    const long long k_lo = m0 / sh.per_k, k_hi = (m1 - 1) / sh.per_k;
    const long long s_lo = max(k_lo, (long long)sh.k_offset), s_hi = min(k_hi, (long long)sh.k_offset + sh.K_local - 1);
    if (s_hi < s_lo) return;
    const unsigned nk = (unsigned)(s_hi - s_lo + 1), du = sh.du, nt = sh.per_k / du;
    const bool k_inner = sh.sk == 1;   // a [T][du][K] layout: samples innermost; else (k, d) order within a step
    // element j of a step's nk du (one division each), then down the steps, G steps apart: G groups of per_t
    // threads when a step's elements fill less than the workgroup; for a fixed step the threads' addresses are
    // consecutive
    const unsigned per_t = nk * du, G = max(1u, (unsigned)kNT / per_t), g0 = threadIdx.x / per_t;
    if (g0 >= G) return;
    for (unsigned j = threadIdx.x - g0 * per_t; j < per_t; j += G == 1 ? kNT : per_t) {
        unsigned kk, d;
        if (k_inner) {
            d = j / nk;
            kk = j - d * nk;
        } else {
            kk = j / du;
            d = j - kk * du;
        }
        const long long k = s_lo + kk;
        // dot2: m is the step's first normal (the step is this workgroup's when m is in its range)
        long long m = k * sh.per_k + (sh.dot2 ? 0 : sh.src[d]) + (long long)g0 * du;
        float* op = sh.out + (k - sh.k_offset) * sh.sk + (long long)d * sh.sd + (long long)g0 * sh.st;
        const double sc = sh.dot2 ? sh.mat[d] : sh.scale[d], mu = sh.mean[d], sc1 = sh.mat[2 + (d & 1)];
        const long long dm = (long long)G * du, dop = (long long)G * sh.st;
        for (unsigned t = g0; t < nt; t += G, m += dm, op += dop) {
            if (m < m0 || m >= m1) continue;
            const double z = m < zb ? cached : s_z[m - zb];
            double x = z * sc;
            if (sh.dot2) x = fma(m + 1 < m1 ? s_z[m + 1 - zb] : s_next, sc1, x);   // np.dot's 2-term rounding
            *op = (float)(x + mu);
        }
    }
}

struct NpHostOut {
    mppi_np_state st;
    int status;
    long long blk;   // the words block holding st.key (its index in the draw's word buffer)
};

// the state NumPy leaves (the key array holding the last consumed word and the position after it) and the draw's
// status, written straight into the host-mapped result (no copies after the draw)
__global__ __launch_bounds__(kNT) void np_state_kernel(const uint32_t* __restrict__ words, long long base,
                                                       const NpResult* res, long long need, NpHostOut* out) {
    const int status = res->status ? res->status : res->last_attempt < 0 ? 3 : 0;
    if (threadIdx.x == 0) out->status = status;
    if (status) return;
    const long long qw = base + 4 * (res->last_attempt + 1) - 1;
    const long long blk = qw / kN;
    for (int i = threadIdx.x; i < kN; i += kNT) out->st.key[i] = words[blk * kN + i];
    if (threadIdx.x == 0) {
        out->blk = blk;
        out->st.pos = (int)(qw - blk * kN) + 1;
        out->st.has_gauss = (int)(need & 1);
        out->st.gauss = (need & 1) ? res->last_fx1 : 0.0;
    }
}

}  // namespace

struct mppi_np_ctx {
    int device = 0;
    double* d_log = nullptr;
    uint32_t* d_seq = nullptr;      // kSeqBlocks blocks
    int poly_P = 0, poly_streams = 0;
    uint32_t* d_nibs = nullptr;     // table jump: the polynomials' 4-bit chunks, [chunk][group][jump], one per word
    int jG = 0, jR = 0, jcpw = 0;   // table jump: stream groups, chunk ranges, chunks per range
    int jparts = 1;                 // partial XORs per stream that np_gen_kernel combines
    uint32_t* d_jumped = nullptr;
    uint32_t* d_words = nullptr;
    size_t words_cap = 0;           // words
    long long last_nblk = -1;       // blocks the last launched draw left in d_words (-1: none usable)
    unsigned long long* d_look = nullptr;   // np_write_kernel's look-back words, one per workgroup
    size_t look_cap = 0;            // workgroups
    unsigned long long epoch = 0;   // the last draw's epoch (24 bits; the words are cleared when it wraps)
    NpResult* d_res = nullptr;
    NpHostOut* h_out = nullptr;     // coherent host-mapped: the draw's state and status, written by np_state_kernel
    NpHostOut* d_out = nullptr;     // its device address
    uint32_t* h_key = nullptr;      // coherent host-mapped: the starting key array, read by the twist kernels
    uint32_t* d_key = nullptr;      // its device address
    hipEvent_t done = nullptr;
    bool pending = false;
};

namespace {

#define NP_CHECK(expr)                                                                    \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return fail(MPPI_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Plan {
    long long need, pairs, A, nblk;
    int P, streams;
};

// attempts generated: 4/3 of the pairs plus 4096 (acceptance pi/4: 1.27 attempts per pair expected), as the
// host path (np_legacy_gauss.c); the block stride P of the streams from a cost model of the two parallel
// phases, measured on MI355X (profiles/r16np2/, profiles/r16f/): the table jump costs ~0.42 us per stream, a
// stream twists its P blocks at ~0.225 us each (MPPI_NP_STRIDE forces P, for measurements).  Config 3 (8.4 M
// normals, 35.9 k blocks): P = 256, 141 streams.
constexpr double kBlockUs = 0.225;
constexpr double kJumpStreamUs = 0.42;   // ~linear in the streams (60.6 us for 140, 112.6 for 280)
Plan make_plan(long long n, int pos, int has_gauss) {
    Plan p;
    p.need = n - (has_gauss ? 1 : 0);
    p.pairs = (p.need + 1) / 2;
    p.A = p.pairs + p.pairs / 3 + 4096;
    p.nblk = (pos + 4 * p.A + kN - 1) / kN + 1;
    static const int forced = getenv("MPPI_NP_STRIDE") ? atoi(getenv("MPPI_NP_STRIDE")) : 0;
    double best = 1e30;
    p.P = 64;
    p.streams = 1;
    for (int P = 16; P <= (1 << 22); P <<= 1) {
        const long long streams = (p.nblk - 1 + P - 1) / P;
        if (streams > MPPI_NP_MAX_STREAMS || (forced && P != forced)) continue;
        const double jump = (double)(streams - 1) * kJumpStreamUs;
        const double cost = jump + P * kBlockUs;
        if (cost < best) {
            best = cost;
            p.P = P;
            p.streams = (int)(streams < 1 ? 1 : streams);
        }
    }
    return p;
}

}  // namespace

extern "C" {

int mppi_np_ctx_create(int device, const double* log_params, mppi_np_ctx** out) {
    if (!out || !log_params) return fail(MPPI_E_ARG, "null argument");
    *out = nullptr;
    NP_CHECK(hipSetDevice(device));
    mppi_np_ctx* c = new mppi_np_ctx();
    c->device = device;
    hipError_t e;
    if ((e = hipMalloc(&c->d_log, NPLOG_NDATA * sizeof(double))) != hipSuccess ||
        (e = hipMemcpy(c->d_log, log_params, NPLOG_NDATA * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMalloc(&c->d_seq, (size_t)kSeqBlocks * kN * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(&c->d_res, sizeof(NpResult))) != hipSuccess ||
        (e = hipHostMalloc(&c->h_out, sizeof(NpHostOut), hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->d_out, c->h_out, 0)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_key, kN * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void**)&c->d_key, c->h_key, 0)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming)) != hipSuccess) {
        mppi_np_ctx_destroy(c);
        return fail(MPPI_E_HIP, std::string("mppi_np_ctx_create: ") + hipGetErrorString(e));
    }
    *out = c;
    return MPPI_OK;
}

void mppi_np_ctx_destroy(mppi_np_ctx* c) {
    if (!c) return;
    if (c->pending && c->done) (void)hipEventSynchronize(c->done);
    (void)hipFree(c->d_log);
    (void)hipFree(c->d_seq);
    (void)hipFree(c->d_nibs);
    (void)hipFree(c->d_jumped);
    (void)hipFree(c->d_words);
    (void)hipFree(c->d_look);
    (void)hipFree(c->d_res);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->h_key) (void)hipHostFree(c->h_key);
    if (c->done) (void)hipEventDestroy(c->done);
    delete c;
}

int mppi_np_plan(const mppi_np_ctx* c, long long n, int pos, int has_gauss, int* block_stride, int* streams) {
    if (!c || !block_stride || !streams) return fail(MPPI_E_ARG, "null argument");
    if (n < 2 || n > MPPI_NP_MAX_NORMALS || pos < 0 || pos > kN) return fail(MPPI_E_ARG, "mppi_np_plan: bad n or pos");
    const Plan p = make_plan(n, pos, has_gauss);
    *block_stride = p.P;
    *streams = p.streams;
    return MPPI_OK;
}

int mppi_np_set_jumps(mppi_np_ctx* c, int block_stride, int streams, const unsigned long long* polys, int words) {
    if (!c || (streams > 1 && !polys)) return fail(MPPI_E_ARG, "null argument");
    if (words != kPolyWords || block_stride < 1 || streams < 1 || streams > MPPI_NP_MAX_STREAMS)
        return fail(MPPI_E_ARG, "mppi_np_set_jumps: bad stride, stream count or polynomial size");
    NP_CHECK(hipSetDevice(c->device));
    if (c->pending) NP_CHECK(hipEventSynchronize(c->done));   // the buffers may be in use by the last draw
    (void)hipFree(c->d_nibs);
    (void)hipFree(c->d_jumped);
    c->d_nibs = nullptr;
    c->d_jumped = nullptr;
    c->poly_P = c->poly_streams = 0;
    if (streams > 1) {
        const int ns = streams - 1;
        const int G = (ns + kNibS - 1) / kNibS;
        int R = std::max(1, std::min(128, (kJTableWGs + G - 1) / G));   // at most 128 parts for np_gen_kernel to XOR
        const int cpw = (kChunks + R - 1) / R;
        R = (kChunks + cpw - 1) / cpw;
        std::vector<uint32_t> nibs((size_t)kChunks * G * kNibS, 0u);
        for (int j = 0; j < ns; ++j)
            for (int w = 0; w < kPolyWords; ++w) {
                const uint64_t m = polys[(size_t)j * kPolyWords + w];
                if (!m) continue;
                if (64 * w + 63 - __builtin_clzll(m) >= kDeg)
                    return fail(MPPI_E_ARG, "mppi_np_set_jumps: a polynomial of degree >= 19937");
                for (int h = 0; h < 16; ++h) {   // the 16 chunks of this 64-bit word
                    const uint32_t v = (uint32_t)(m >> (4 * h)) & 15u;
                    const int ch = 16 * w + h;
                    if (v && ch < kChunks)
                        nibs[((size_t)ch * G + j / kNibS) * kNibS + j % kNibS] = v;
                }
            }
        NP_CHECK(hipMalloc(&c->d_nibs, nibs.size() * sizeof(uint32_t)));
        NP_CHECK(hipMemcpy(c->d_nibs, nibs.data(), nibs.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        NP_CHECK(hipMalloc(&c->d_jumped, (size_t)ns * R * kN * sizeof(uint32_t)));
        c->jG = G;
        c->jR = R;
        c->jcpw = cpw;
        c->jparts = R;
    }
    c->poly_P = block_stride;
    c->poly_streams = streams;
    return MPPI_OK;
}

int mppi_np_draw(mppi_np_ctx* c, void* stream, const mppi_np_state* st, long long n, const mppi_np_target* tgt) {
    if (!c || !st || !tgt || !tgt->out_dev) return fail(MPPI_E_ARG, "null argument");
    if (n < 2 || n > MPPI_NP_MAX_NORMALS || st->pos < 0 || st->pos > kN)
        return fail(MPPI_E_ARG, "mppi_np_draw: bad n or state position");
    if (tgt->du < 1 || tgt->du > MPPI_NP_MAX_DU || tgt->K < 1 || tgt->T < 1 || tgt->K * tgt->T * tgt->du != n ||
        tgt->k_offset < 0 || tgt->K_local < 0 || tgt->k_offset + tgt->K_local > tgt->K)
        return fail(MPPI_E_ARG, "mppi_np_draw: the target's (K, T, du) and slice must match n");
    for (int d = 0; d < tgt->du; ++d)
        if (!tgt->dot2 && (tgt->src[d] < 0 || tgt->src[d] >= tgt->du)) return fail(MPPI_E_ARG, "mppi_np_draw: bad src");
    if (tgt->dot2 && tgt->du != 2) return fail(MPPI_E_ARG, "mppi_np_draw: dot2 needs du = 2");
    const Plan p = make_plan(n, st->pos, st->has_gauss);
    if (p.P != c->poly_P || p.streams > c->poly_streams)
        return fail(MPPI_E_ARG, "mppi_np_draw: the jump polynomials of mppi_np_plan's stride and count are not set");
    NP_CHECK(hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    if (c->pending) NP_CHECK(hipEventSynchronize(c->done));
    // A draw that starts where the last one ended (the drop-ins' queued next-call draw does) finds its first 34
    // blocks in the last draw's words already (generated with ~1600 blocks of slack at c3): the jumps read that
    // slice and the sequence is not twisted again.
    long long reuse_blk = -1;
    if (p.streams > 1 && c->last_nblk > 0 && c->h_out->status == 0 && st->pos == c->h_out->st.pos &&
        c->h_out->blk >= 0 && c->h_out->blk + kSeqBlocks <= c->last_nblk &&
        !memcmp(st->key, c->h_out->st.key, kN * sizeof(uint32_t)))
        reuse_blk = c->h_out->blk;
    c->last_nblk = -1;   // until this draw's kernels are queued
    const size_t words = (size_t)p.nblk * kN;
    if (words > c->words_cap) {
        reuse_blk = -1;
        (void)hipFree(c->d_words);
        c->d_words = nullptr;
        c->words_cap = 0;
        NP_CHECK(hipMalloc(&c->d_words, words * sizeof(uint32_t)));
        c->words_cap = words;
    }
    const long long nwg = (p.A + kAttPerWG - 1) / kAttPerWG;
    if ((size_t)nwg > c->look_cap) {
        (void)hipFree(c->d_look);
        c->d_look = nullptr;
        c->look_cap = 0;
        NP_CHECK(hipMalloc(&c->d_look, nwg * sizeof(unsigned long long)));
        c->look_cap = (size_t)nwg;
        c->epoch = 0;   // cleared below
    }
    if (++c->epoch >= (1ull << (64 - kLookShift - 2)) || c->epoch == 1) {
        c->epoch = 1;
        NP_CHECK(hipMemsetAsync(c->d_look, 0, c->look_cap * sizeof(unsigned long long), s));
    }
    memcpy(c->h_key, st->key, kN * sizeof(uint32_t));   // read by the kernels over the link (no copy)
    if (p.streams > 1) {
        const uint32_t* seq = c->d_seq;
        if (reuse_blk >= 0)
            seq = c->d_words + (size_t)reuse_blk * kN;   // read before np_gen_kernel rewrites d_words (stream order)
        else
            hipLaunchKernelGGL(np_seq_kernel, dim3(1), dim3(kTT), 0, s, c->d_key, c->d_seq);
        hipLaunchKernelGGL(np_jumpn_kernel, dim3(c->jR, c->jG), dim3(kJNT), (4 * c->jcpw + kN + 3) * sizeof(uint32_t),
                           s, seq, c->d_nibs, c->jG, c->jcpw, p.streams - 1, c->jR, c->d_jumped);
    }
    hipLaunchKernelGGL(np_gen_kernel, dim3(p.streams), dim3(kTT), 0, s, c->d_key, c->d_jumped, c->d_words, p.P,
                       (int)p.nblk, c->jparts, c->d_res);
    NpShape sh;
    sh.out = (float*)tgt->out_dev;
    sh.per_k = (unsigned)(tgt->T * tgt->du);
    sh.du = (unsigned)tgt->du;
    sh.k_offset = (unsigned)tgt->k_offset;
    sh.K_local = (unsigned)tgt->K_local;
    sh.st = tgt->stride_t;
    sh.sk = tgt->stride_k;
    sh.sd = tgt->stride_d;
    sh.dot2 = tgt->dot2 ? 1 : 0;
    for (int i = 0; i < 4; ++i) sh.mat[i] = tgt->mat[i];
    for (int d = 0; d < MPPI_NP_MAX_DU; ++d) {
        sh.src[d] = d < tgt->du ? tgt->src[d] : 0;
        sh.scale[d] = d < tgt->du ? tgt->scale[d] : 0.0;
        sh.mean[d] = d < tgt->du ? tgt->mean[d] : 0.0;
    }
    hipLaunchKernelGGL(np_write_kernel, dim3((unsigned)nwg), dim3(kNT), 0, s, c->d_words, (long long)st->pos, p.A,
                       c->d_look, c->epoch << (kLookShift + 2), c->d_log, sh, p.pairs, n, st->has_gauss ? 1 : 0,
                       st->gauss, c->d_res);
    hipLaunchKernelGGL(np_state_kernel, dim3(1), dim3(kNT), 0, s, c->d_words, (long long)st->pos, c->d_res, p.need,
                       c->d_out);
    // the event marks the end of whatever was queued, even after a failed launch: the next draw waits for it
    // before it rewrites the host-mapped key the queued kernels read
    const hipError_t le = hipGetLastError();
    NP_CHECK(hipEventRecord(c->done, s));
    c->pending = true;
    if (le != hipSuccess) return fail(MPPI_E_HIP, std::string("mppi_np_draw: ") + hipGetErrorString(le));
    c->last_nblk = p.nblk;
    return MPPI_OK;
}

int mppi_np_draw_result(mppi_np_ctx* c, mppi_np_state* st_out) {
    if (!c || !st_out) return fail(MPPI_E_ARG, "null argument");
    if (!c->pending) return fail(MPPI_E_ARG, "mppi_np_draw_result: no draw pending");
    c->pending = false;
    NP_CHECK(hipEventSynchronize(c->done));
    if (c->h_out->status != 0)
        return fail(MPPI_E_RETRY, "mppi_np_draw: fewer accepted attempts than pairs wanted, or the look-back gave up (output incomplete)");
    *st_out = c->h_out->st;
    return MPPI_OK;
}

}  // extern "C"
