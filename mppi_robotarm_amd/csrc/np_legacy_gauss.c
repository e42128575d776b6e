// NumPy's legacy global-RNG Gaussian stream, continued bit-exactly with threads.
//
// The drop-in's default noise (noise="numpy") is the reference's own draw,
// np.random.multivariate_normal(mu, Sigma, (K, T)) on the legacy global
// RandomState (control.py:154-164).  Its cost is the standard-normal stream:
// MT19937 words -> legacy doubles -> the polar method with rejection, one
// Gaussian pair per accepted attempt (NumPy's legacy_gauss), sequential in
// NumPy.  Every attempt consumes exactly four 32-bit words, so attempt i
// reads words [4i, 4i + 4) of the stream: the words are generated first (the
// twist is the only sequential part), then threads test and convert disjoint
// attempt ranges and place their pairs after a prefix count of the accepted
// attempts before them.  Same libm log and IEEE sqrt, no contraction
// (-ffp-contract=off), so every value equals NumPy's; the state left behind
// (key, pos, the cached Gaussian) is the one NumPy would leave.
//
// The twist itself runs in parallel too: MT19937 is linear over GF(2), so the
// key array of any later block is a polynomial in the step map applied to the
// current one (jump-ahead: Haramoto, Matsumoto, Nishimura, L'Ecuyer, Panneton,
// "Efficient jump ahead for F2-linear random number generators", 2008).  The
// characteristic polynomial P of the per-word step is found once per process
// by Berlekamp-Massey on the generator's own output; a jump by J words is
// x^J mod P (binary powering, cached per J) evaluated on the state by Horner's
// rule; each thread jumps to the block before its range, twists once (which
// also fixes the 31 low bits of the oldest word, outside the 19937-bit state)
// and twists its own range.  A self-test against the sequential twist guards
// it; on any failure the twist stays sequential.
//
// Host code, never on the device path; the Python side (controller.py,
// legacy_multivariate_normal) does the rest of multivariate_normal with
// NumPy's own calls.
#define _GNU_SOURCE
#include <link.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

#include "np_glibc_log.h"

// AVX2 instances of the integer-only loops where the CPU has it (the same bits either way)
#if defined(__x86_64__) && defined(__GNUC__) && !defined(__clang__)
#define MT_CLONES __attribute__((target_clones("avx2", "default")))
#else
#define MT_CLONES
#endif

// next key array from the previous one, out of place (no aliasing: the loops vectorize); the same values as
// NumPy's in-place mt19937_gen
MT_CLONES static void mt_twist_to(const uint32_t* __restrict__ o, uint32_t* __restrict__ k) {
    const uint32_t A = 0x9908b0dfu, UP = 0x80000000u, LO = 0x7fffffffu;
    for (int i = 0; i < MT_N - MT_M; i++) {
        const uint32_t y = (o[i] & UP) | (o[i + 1] & LO);
        k[i] = o[i + MT_M] ^ (y >> 1) ^ (-(y & 1u) & A);
    }
    for (int i = MT_N - MT_M; i < MT_N - 1; i++) {
        const uint32_t y = (o[i] & UP) | (o[i + 1] & LO);
        k[i] = k[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1u) & A);
    }
    const uint32_t y = (o[MT_N - 1] & UP) | (k[0] & LO);
    k[MT_N - 1] = k[MT_M - 1] ^ (y >> 1) ^ (-(y & 1u) & A);
}

// the block buffer, kept across calls (a fresh 90 MB allocation per draw costs its page faults every call)
static uint32_t* g_blocks = NULL;
static int64_t g_cap = 0;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static inline uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

static inline double legacy_double(uint32_t a, uint32_t b) {
    return ((a >> 5) * 67108864.0 + (b >> 6)) / 9007199254740992.0;
}

// ------------------------------------------------------------------ worker pool
// Threads made once and kept (a draw has three parallel phases; creating and joining 15 threads for each cost
// more than some phases); a child after fork() starts without them.
typedef void* (*TaskFn)(void*);
typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    int made;            // workers created (ids 1 .. made)
    unsigned long gen;   // task generation
    int active;          // workers 1 .. active - 1 take part in the current task
    int pending;         // of those, not finished
    TaskFn fn;
    char* args;
    size_t stride;
    unsigned long born[64];   // the generation before a worker's first task (set when it is made)
} Pool;
static Pool g_pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0, 0, 0, NULL,
                      NULL, 0, {0}};

static void pool_child_reset(void) {
    pthread_mutex_init(&g_pool.mu, NULL);
    pthread_cond_init(&g_pool.go, NULL);
    pthread_cond_init(&g_pool.done, NULL);
    g_pool.made = 0;
    g_pool.pending = 0;
}

static void* pool_worker(void* p) {
    const int id = (int)(intptr_t)p;
    pthread_mutex_lock(&g_pool.mu);
    unsigned long seen = g_pool.born[id];   // not the current one: the task it was made for may be posted already
    for (;;) {
        while (g_pool.gen == seen) pthread_cond_wait(&g_pool.go, &g_pool.mu);
        seen = g_pool.gen;
        if (id < g_pool.active) {
            const TaskFn fn = g_pool.fn;
            void* arg = g_pool.args + (size_t)id * g_pool.stride;
            pthread_mutex_unlock(&g_pool.mu);
            fn(arg);
            pthread_mutex_lock(&g_pool.mu);
            if (--g_pool.pending == 0) pthread_cond_signal(&g_pool.done);
        }
    }
    return NULL;
}

// fn(args + t * stride) for t = 0 .. nt - 1, t = 0 on the calling thread; returns once all are done.  Falls
// back to fewer threads (down to the caller alone) when workers cannot be made.
static void pool_run(TaskFn fn, void* args, size_t stride, int nt_req) {
    int nt = nt_req;
    pthread_mutex_lock(&g_pool.mu);
    static int atfork_set = 0;
    if (!atfork_set) {
        pthread_atfork(NULL, NULL, pool_child_reset);
        atfork_set = 1;
    }
    while (g_pool.made < nt - 1 && g_pool.made < 63) {
        g_pool.born[g_pool.made + 1] = g_pool.gen;
        pthread_t th;
        pthread_attr_t at;
        pthread_attr_init(&at);
        pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
        const int rc = pthread_create(&th, &at, pool_worker, (void*)(intptr_t)(g_pool.made + 1));
        pthread_attr_destroy(&at);
        if (rc != 0) break;
        ++g_pool.made;
    }
    if (nt - 1 > g_pool.made) nt = g_pool.made + 1;
    g_pool.fn = fn;
    g_pool.args = (char*)args;
    g_pool.stride = stride;
    g_pool.active = nt;
    g_pool.pending = nt - 1;
    ++g_pool.gen;
    pthread_cond_broadcast(&g_pool.go);
    pthread_mutex_unlock(&g_pool.mu);
    // the caller's share, then the rest: a task left unstarted by a worker that could not be made runs here
    fn(args);
    for (int t = nt; t < nt_req; ++t) fn((char*)args + (size_t)t * stride);
    pthread_mutex_lock(&g_pool.mu);
    while (g_pool.pending > 0) pthread_cond_wait(&g_pool.done, &g_pool.mu);
    pthread_mutex_unlock(&g_pool.mu);
}

// ------------------------------------------------------------------ jump-ahead
#define MT_DEG 19937                       // dimension of the state (the oldest word's top bit + 623 words)
#define PW ((MT_DEG + 64) / 64)            // 64-bit words of a polynomial of degree <= MT_DEG
typedef struct {
    int ready;                             // 1: P below is valid; -1: unavailable (sequential twist)
    uint64_t p[PW];                        // the characteristic polynomial, bit e = coefficient of x^e
    int nterms;                            // its terms below x^MT_DEG
    int terms[MT_DEG];
} CharPoly;
static CharPoly g_cp;

static inline int bit_get(const uint64_t* a, int64_t i) { return (int)((a[i >> 6] >> (i & 63)) & 1u); }
static inline void bit_flip(uint64_t* a, int64_t i) { a[i >> 6] ^= 1ull << (i & 63); }
// 64 bits of a starting at bit i (bits past nwords*64 read as 0)
static inline uint64_t bits64(const uint64_t* a, int64_t nwords, int64_t i) {
    const int64_t w = i >> 6;
    const int sh = (int)(i & 63);
    const uint64_t lo = w < nwords ? a[w] : 0, hi = w + 1 < nwords ? a[w + 1] : 0;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// Berlekamp-Massey over GF(2) on the bit-0 sequence of the untempered words from a seeded state: the minimal
// polynomial of that sequence is the characteristic polynomial of the step map (irreducible for MT19937,
// degree 19937).  P(x) = x^L C(1/x) for the connection polynomial C.
static int char_poly_init(void) {
    enum { NB = 2 * MT_DEG + 128, CW = (NB + 63) / 64 + 2 };
    static uint64_t seq[CW], C[CW], B[CW], T[CW];
    const int nblk = NB / MT_N + 3;
    uint32_t* w = (uint32_t*)malloc((size_t)nblk * MT_N * sizeof(uint32_t));
    if (!w) return -1;
    w[0] = 5489u;   // init_genrand(5489)
    for (int i = 1; i < MT_N; ++i) w[i] = 1812433253u * (w[i - 1] ^ (w[i - 1] >> 30)) + (uint32_t)i;
    for (int b = 1; b < nblk; ++b) mt_twist_to(w + (size_t)(b - 1) * MT_N, w + (size_t)b * MT_N);
    // s_n = bit 0 of word MT_N + n (generated words only), stored reversed: seq bit j = s_{NB-1-j}
    memset(seq, 0, sizeof(seq));
    for (int64_t n = 0; n < NB; ++n)
        if (w[MT_N + n] & 1u) bit_flip(seq, NB - 1 - n);
    free(w);
    memset(C, 0, sizeof(C));
    memset(B, 0, sizeof(B));
    C[0] = B[0] = 1;
    int64_t L = 0, m = 1;
    for (int64_t n = 0; n < NB; ++n) {
        // d = sum_{i=0..L} c_i s_{n-i} = parity of C[0..L] & seq[NB-1-n ..]
        const int64_t off = NB - 1 - n, words = (L + 64) / 64;
        uint64_t acc = 0;
        for (int64_t q = 0; q < words; ++q) {
            uint64_t c = C[q];
            if (q == words - 1 && ((L + 1) & 63)) c &= (1ull << ((L + 1) & 63)) - 1;
            acc ^= c & bits64(seq, CW, off + 64 * q);
        }
        if (!(__builtin_popcountll(acc) & 1)) {
            ++m;
            continue;
        }
        const int ws = (int)(m >> 6), bs = (int)(m & 63);
        if (2 * L <= n) memcpy(T, C, sizeof(C));
        for (int64_t q = CW - 1; q >= ws; --q) {   // C ^= B << m
            const uint64_t v = (B[q - ws] << bs) | (bs && q - ws - 1 >= 0 ? B[q - ws - 1] >> (64 - bs) : 0);
            C[q] ^= v;
        }
        if (2 * L <= n) {
            L = n + 1 - L;
            memcpy(B, T, sizeof(C));
            m = 1;
        } else {
            ++m;
        }
    }
    if (L != MT_DEG) return -1;
    memset(g_cp.p, 0, sizeof(g_cp.p));
    g_cp.nterms = 0;
    int top = 0;
    for (int64_t i = 0; i <= L; ++i)
        if (bit_get(C, i)) {   // c_i x^i  ->  x^(L - i)
            bit_flip(g_cp.p, L - i);
            if (L - i < MT_DEG) {
                g_cp.terms[g_cp.nterms++] = (int)(L - i);
                if (L - i > top) top = (int)(L - i);
            }
        }
    // reduce_mod's word-at-a-time order needs a gap of more than 64 below the leading term (it is 623)
    return bit_get(g_cp.p, MT_DEG) && bit_get(g_cp.p, 0) && MT_DEG - top > 64 ? 0 : -1;
}

// a (bits 0 .. 2 MT_DEG, 2 PW words) reduced mod P in place: each set bit i >= MT_DEG is replaced by the
// terms of P below x^MT_DEG shifted by i - MT_DEG (the leading term cancels it).  A word at a time, top down:
// P's highest term below x^MT_DEG is x^19314 (623 below), so the bits a word's high part maps to lie at least
// 623 positions lower, in words not yet visited (checked when P is found: MT_DEG - top > 64).  In the lowest
// word (w0 = 311) only bits >= 33 are set, so a term below 33 lands at a negative word offset pos: its low half
// (q = -1) is all zero and skipped, its high half goes to word 0.
static void reduce_mod(uint64_t* a) {
    const int64_t w0 = MT_DEG >> 6;
    for (int64_t w = (2 * MT_DEG) >> 6; w >= w0; --w) {
        uint64_t v = a[w];
        if (w == w0) v &= ~0ull << (MT_DEG & 63);   // the bits >= MT_DEG of the lowest such word
        if (!v) continue;
        a[w] ^= v;
        for (int e = 0; e < g_cp.nterms; ++e) {   // v x^(64 w) -> v x^(64 w - MT_DEG + term)
            const int64_t pos = 64 * w - MT_DEG + g_cp.terms[e];
            const int64_t q = pos >> 6;
            const int sh = (int)(pos & 63);
            if (q >= 0) a[q] ^= v << sh;
            if (sh) a[q + 1] ^= v >> (64 - sh);
        }
    }
}

// x^J mod P by binary powering (squaring is the bit spread; multiplying by x a shift)
static void pow_x_mod(uint64_t J, uint64_t* out /* PW words */) {
    uint64_t r[2 * PW], t[2 * PW];
    memset(r, 0, sizeof(r));
    r[0] = 1;
    int top = 63;
    while (top > 0 && !((J >> top) & 1)) --top;
    for (int b = top; b >= 0; --b) {
        memset(t, 0, sizeof(t));   // t = r^2: bit i -> bit 2i
        for (int q = 0; q < PW; ++q) {
            uint64_t v = r[q];
            while (v) {
                const int k = __builtin_ctzll(v);
                v &= v - 1;
                bit_flip(t, 2 * (64 * (int64_t)q + k));
            }
        }
        reduce_mod(t);
        memcpy(r, t, sizeof(r));
        if ((J >> b) & 1) {   // r *= x
            for (int q = 2 * PW - 1; q > 0; --q) r[q] = (r[q] << 1) | (r[q - 1] >> 63);
            r[0] <<= 1;
            reduce_mod(r);
        }
    }
    memcpy(out, r, PW * sizeof(uint64_t));
}

// jump polynomials already computed, keyed by J (words); guarded by g_jmu
#define JCACHE 128
static uint64_t g_jkey[JCACHE];
static uint64_t* g_jpoly[JCACHE];
static int g_jn = 0;
static pthread_mutex_t g_jmu = PTHREAD_MUTEX_INITIALIZER;     // the cache
static pthread_mutex_t g_initmu = PTHREAD_MUTEX_INITIALIZER;  // jump_init_locked

static const uint64_t* jump_poly(uint64_t J) {
    pthread_mutex_lock(&g_jmu);
    for (int i = 0; i < g_jn; ++i)
        if (g_jkey[i] == J) {
            const uint64_t* p = g_jpoly[i];
            pthread_mutex_unlock(&g_jmu);
            return p;
        }
    pthread_mutex_unlock(&g_jmu);
    uint64_t* p = (uint64_t*)malloc(PW * sizeof(uint64_t));   // computed outside the lock (threads in parallel)
    if (!p) return NULL;
    pow_x_mod(J, p);
    pthread_mutex_lock(&g_jmu);
    if (g_jn == JCACHE) {   // full: start over (the drop-in uses a handful of draw sizes)
        for (int i = 0; i < g_jn; ++i) free(g_jpoly[i]);
        g_jn = 0;
    }
    g_jkey[g_jn] = J;
    g_jpoly[g_jn++] = p;
    pthread_mutex_unlock(&g_jmu);
    return p;
}

// The key array J words-steps after `key` (J = 624 b: the key array of block b), up to the 31 low bits of its
// oldest word, which lie outside the state: sum_d phi_d F^d(key) with F the one-word step.  F^d(key) is the
// window [d, d + 624) of the word sequence that starts with key (block 0, then the blocks the twist makes), so
// the sum is the XOR of the windows at phi's set bits: the sequence's first 34 blocks are made once (~20 us),
// then each 48-word slice of the result is accumulated in registers over every set bit (loads and XORs only;
// the same value as Horner's rule on the circular state, 5x fewer memory operations).
#define JW_CH 48                                     // 624 = 13 x 48 words per slice
#define JW_NB ((MT_DEG + MT_N) / MT_N + 1)           // blocks covering words [0, MT_DEG + MT_N)
MT_CLONES static void jw_slice(const uint32_t* seq, const int* bits, int nb, int c, uint32_t* out) {
    uint32_t acc[JW_CH];
    memset(acc, 0, sizeof(acc));
    for (int b = 0; b < nb; ++b) {
        const uint32_t* w = seq + bits[b] + c;
        for (int q = 0; q < JW_CH; ++q) acc[q] ^= w[q];
    }
    memcpy(out + c, acc, sizeof(acc));
}

static int jump_state(const uint32_t* key, const uint64_t* phi, uint32_t* out) {
    uint32_t* seq = (uint32_t*)malloc((size_t)JW_NB * MT_N * sizeof(uint32_t));
    int* bits = (int*)malloc((MT_DEG + 1) * sizeof(int));
    if (!seq || !bits) {
        free(seq);
        free(bits);
        return -1;
    }
    memcpy(seq, key, MT_N * sizeof(uint32_t));
    for (int b = 1; b < JW_NB; ++b) mt_twist_to(seq + (size_t)(b - 1) * MT_N, seq + (size_t)b * MT_N);
    int nb = 0;
    for (int i = 0; i < PW; ++i)
        for (uint64_t m = phi[i]; m; m &= m - 1) {
            const int d = i * 64 + __builtin_ctzll(m);
            if (d <= MT_DEG) bits[nb++] = d;
        }
    for (int c = 0; c < MT_N; c += JW_CH) jw_slice(seq, bits, nb, c, out);
    free(seq);
    free(bits);
    return 0;
}

// once per process (under g_initmu): P, then a self-test of two jumps (to blocks 3 and 1000) against the
// sequential twist
static void jump_init_locked(void) {
    if (g_cp.ready) return;
    if (char_poly_init() != 0) {
        g_cp.ready = -1;
        return;
    }
    g_cp.ready = 1;
    enum { NBT = 1001 };
    uint32_t* w = (uint32_t*)malloc((size_t)NBT * MT_N * sizeof(uint32_t));
    uint32_t j[MT_N], k[MT_N];
    if (!w) {
        g_cp.ready = -1;
        return;
    }
    w[0] = 19650218u;
    for (int i = 1; i < MT_N; ++i) w[i] = 1812433253u * (w[i - 1] ^ (w[i - 1] >> 30)) + (uint32_t)i;
    for (int b = 1; b < NBT; ++b) mt_twist_to(w + (size_t)(b - 1) * MT_N, w + (size_t)b * MT_N);
    const int tb[2] = {3, NBT - 1};
    for (int q = 0; q < 2; ++q) {
        const uint64_t* phi = jump_poly((uint64_t)MT_N * (tb[q] - 1));
        if (!phi) {
            g_cp.ready = -1;
            break;
        }
        if (jump_state(w, phi, j) != 0) {   // block tb - 1, up to its oldest word's low bits
            g_cp.ready = -1;
            break;
        }
        mt_twist_to(j, k);       // block tb, exactly
        if (memcmp(k, w + (size_t)tb[q] * MT_N, sizeof(k)) != 0) g_cp.ready = -1;
    }
    free(w);
}

typedef struct {
    uint32_t* blocks;
    int64_t b0, b1;   // blocks [b0, b1) to fill; block b0 - 1 from a jump when b0 > 1
    int ok;
} GenWork;

static void* gen_pass(void* p) {
    GenWork* g = (GenWork*)p;
    uint32_t prev[MT_N];
    const uint32_t* src = g->blocks + (size_t)(g->b0 - 1) * MT_N;
    if (g->b0 > 1) {   // the block before the range: a jump from block 0 to block b0 - 2, one twist
        const uint64_t* phi = jump_poly((uint64_t)MT_N * (uint64_t)(g->b0 - 2));
        if (!phi) return NULL;
        uint32_t j[MT_N];
        if (g->b0 - 2 > 0) {
            if (jump_state(g->blocks, phi, j) != 0) return NULL;
        } else {
            memcpy(j, g->blocks, sizeof(j));
        }
        mt_twist_to(j, prev);
        src = prev;
    }
    for (int64_t b = g->b0; b < g->b1; ++b) {
        mt_twist_to(src, g->blocks + (size_t)b * MT_N);
        src = g->blocks + (size_t)b * MT_N;
    }
    g->ok = 1;
    return NULL;
}

// blocks 1 .. nblk - 1 from block 0; in parallel when there are enough of them
static int g_jump_min_blocks = 4096;   // below this the sequential twist (~0.5 us per block) is as fast

static void twist_blocks(uint32_t* blocks, int64_t nblk, int nthreads) {
    int nt = nthreads;
    if (nblk < g_jump_min_blocks || nt < 2) nt = 1;
    if (nt > 1) {
        pthread_mutex_lock(&g_initmu);
        jump_init_locked();
        const int ready = g_cp.ready;
        pthread_mutex_unlock(&g_initmu);
        if (ready != 1) nt = 1;
    }
    if (nt == 1) {
        for (int64_t b = 1; b < nblk; ++b) mt_twist_to(blocks + (b - 1) * MT_N, blocks + b * MT_N);
        return;
    }
    GenWork gw[64];
    // blocks per thread rounded up to a multiple of 64, so that the jump lengths (cached per length) stay the
    // same from draw to draw although the state's position moves the block count by one
    const int64_t per = ((nblk - 1 + nt - 1) / nt + 63) / 64 * 64;
    for (int t = 0; t < nt; ++t) {
        gw[t].blocks = blocks;
        gw[t].b0 = 1 + per * t < nblk ? 1 + per * t : nblk;
        gw[t].b1 = 1 + per * (t + 1) < nblk ? 1 + per * (t + 1) : nblk;
        gw[t].ok = 0;
    }
    pool_run(gen_pass, gw, sizeof(GenWork), nt);
    for (int t = 0; t < nt; ++t)
        if (!gw[t].ok) {   // a failed allocation: the sequential twist
            for (int64_t b = 1; b < nblk; ++b) mt_twist_to(blocks + (b - 1) * MT_N, blocks + b * MT_N);
            return;
        }
}

typedef struct {
    const uint32_t* blocks;   // untempered key arrays, block 0 = the state's current key
    int64_t base;             // absolute word index of stream word 0 (the state's pos)
    int64_t a0, a1;           // attempt range of this worker
    int64_t count;            // accepted attempts in [a0, a1)
    int64_t first_pair;       // pass 2: index of this range's first pair
    int64_t pairs;            // pass 2: pairs wanted overall
    double* out;              // pass 2: pair p -> out[2p] = f x2, out[2p + 1] = f x1 (if inside n)
    int64_t n_out;
    int64_t last_attempt;     // pass 2: attempt of the last wanted pair, if in this range
    double last_fx1;
} Work;

static inline void attempt(const uint32_t* blocks, int64_t base, int64_t i, double* x1, double* x2, double* r2) {
    const int64_t w = base + 4 * i;
    const uint32_t a = temper(blocks[w]), b = temper(blocks[w + 1]);
    const uint32_t c = temper(blocks[w + 2]), d = temper(blocks[w + 3]);
    *x1 = 2.0 * legacy_double(a, b) - 1.0;
    *x2 = 2.0 * legacy_double(c, d) - 1.0;
    *r2 = *x1 * *x1 + *x2 * *x2;
}

MT_CLONES static void* count_pass(void* p) {
    Work* w = (Work*)p;
    int64_t n = 0;
    for (int64_t i = w->a0; i < w->a1; ++i) {
        double x1, x2, r2;
        attempt(w->blocks, w->base, i, &x1, &x2, &r2);
        n += (r2 < 1.0 && r2 != 0.0);
    }
    w->count = n;
    return NULL;
}

static void* write_pass(void* p) {
    Work* w = (Work*)p;
    int64_t q = w->first_pair;
    for (int64_t i = w->a0; i < w->a1 && q < w->pairs; ++i) {
        double x1, x2, r2;
        attempt(w->blocks, w->base, i, &x1, &x2, &r2);
        if (r2 >= 1.0 || r2 == 0.0) continue;
        const double f = sqrt(-2.0 * log(r2) / r2);
        const double g1 = f * x1, g2 = f * x2;
        w->out[2 * q] = g2;
        if (2 * q + 1 < w->n_out) w->out[2 * q + 1] = g1;
        if (q == w->pairs - 1) {
            w->last_attempt = i;
            w->last_fx1 = g1;
        }
        ++q;
    }
    return NULL;
}

// key[624] / *pos: the MT19937 state (NumPy's get_state()[1:3]); *has_gauss / *gauss: the cached Gaussian
// (get_state()[3:5]).  Writes n standard normals exactly as n calls of legacy_gauss would, and leaves the
// state those calls would leave.  Returns 0, or -1 on bad arguments / allocation failure (state untouched).
static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

static int legacy_gauss_locked(uint32_t* key, int* pos, int* has_gauss, double* gauss, double* out, int64_t n,
                               int nthreads) {
    static int timing = -1;   // MPPI_NP_TIMING=1: the phases' wall times on stderr (diagnostics)
    if (timing < 0) timing = getenv("MPPI_NP_TIMING") != NULL;
    const double t_start = timing ? now_ms() : 0.0;
    if (!key || !pos || !has_gauss || !gauss || (n > 0 && !out) || n < 0 || *pos < 0 || *pos > MT_N) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    int64_t o = 0;
    const int cached = *has_gauss != 0;
    if (n > 0 && cached) out[o++] = *gauss;
    const int64_t need = n - o, pairs = (need + 1) / 2;
    if (pairs == 0) {
        if (n > 0 && cached) {
            *has_gauss = 0;
            *gauss = 0.0;
        }
        return 0;
    }
    int64_t A = pairs + pairs / 3 + 4096;   // acceptance pi/4: 1.27 attempts per pair expected
    for (;;) {
        const int64_t words = 4 * A;
        const int64_t nblk = (*pos + words + MT_N - 1) / MT_N + 1;
        if (nblk > g_cap) {
            free(g_blocks);
            g_blocks = (uint32_t*)malloc((size_t)nblk * MT_N * sizeof(uint32_t));
            g_cap = g_blocks ? nblk : 0;
            if (!g_blocks) return -1;
        }
        uint32_t* blocks = g_blocks;
        memcpy(blocks, key, MT_N * sizeof(uint32_t));
        const double t_tw = timing ? now_ms() : 0.0;
        twist_blocks(blocks, nblk, nthreads);
        const double t_cnt = timing ? now_ms() : 0.0;
        Work wk[64];
        const int nt = (int)(A < nthreads * 4096 ? 1 : nthreads);
        for (int t = 0; t < nt; ++t) {
            memset(&wk[t], 0, sizeof(Work));
            wk[t].blocks = blocks;
            wk[t].base = *pos;
            wk[t].a0 = A * t / nt;
            wk[t].a1 = A * (t + 1) / nt;
            wk[t].out = out + o;
            wk[t].n_out = need;
            wk[t].pairs = pairs;
            wk[t].last_attempt = -1;
        }
        pool_run(count_pass, wk, sizeof(Work), nt);
        int64_t total = 0;
        for (int t = 0; t < nt; ++t) {
            wk[t].first_pair = total;
            total += wk[t].count;
        }
        if (total < pairs) {   // too few attempts generated (vanishingly rare): more, from the same state
            A = A + A / 2;
            continue;
        }
        const double t_wr = timing ? now_ms() : 0.0;
        pool_run(write_pass, wk, sizeof(Work), nt);
        if (timing)
            fprintf(stderr, "np_legacy_gauss n=%lld threads=%d: setup %.3f twist %.3f count %.3f write %.3f ms\n",
                    (long long)n, nt, t_tw - t_start, t_cnt - t_tw, t_wr - t_cnt, now_ms() - t_wr);
        int64_t last = -1;
        double fx1 = 0.0;
        for (int t = 0; t < nt; ++t)
            if (wk[t].last_attempt >= 0) {
                last = wk[t].last_attempt;
                fx1 = wk[t].last_fx1;
            }
        // state after the last consumed word (absolute index q): the key array of its block, pos past it
        const int64_t q = *pos + 4 * (last + 1) - 1;
        memcpy(key, blocks + (q / MT_N) * MT_N, MT_N * sizeof(uint32_t));
        *pos = (int)(q % MT_N) + 1;
        if (need & 1) {   // an odd count leaves the last pair's f x1 cached
            *has_gauss = 1;
            *gauss = fx1;
        } else {
            *has_gauss = 0;
            *gauss = 0.0;
        }
        return 0;
    }
}

int mppi_np_legacy_gauss(uint32_t* key, int* pos, int* has_gauss, double* gauss, double* out, int64_t n,
                         int nthreads) {
    pthread_mutex_lock(&g_mu);
    const int rc = legacy_gauss_locked(key, pos, has_gauss, gauss, out, n, nthreads);
    if (g_cap * MT_N * (int64_t)sizeof(uint32_t) > ((int64_t)256 << 20)) {   // not kept past 256 MB (config 5's
        free(g_blocks);                                                        // 1.2 GB draw buffer)
        g_blocks = NULL;
        g_cap = 0;
    }
    pthread_mutex_unlock(&g_mu);
    return rc;
}

// Tests: the block count from which the twist runs in parallel (jump-ahead), and whether the jump machinery
// passed its self-test (1), failed (-1) or has not run (0).
int mppi_np_jump_config(int min_blocks) {
    pthread_mutex_lock(&g_mu);
    if (min_blocks > 0) g_jump_min_blocks = min_blocks;
    pthread_mutex_lock(&g_initmu);
    jump_init_locked();
    const int r = g_cp.ready;
    pthread_mutex_unlock(&g_initmu);
    pthread_mutex_unlock(&g_mu);
    return r;
}

// ------------------------------------------------------------------ the device draw's inputs
// The device draw of the same stream (mppi_rocm.h mppi_np_*) needs two things only the host has: the jump
// polynomials (x^J mod P for the block offsets its generator streams start at) and glibc's log constants.

// x^J mod P into out[PW] (bit e = coefficient of x^e); 0, or -1 when the jump machinery is unavailable
int mppi_np_jump_poly(uint64_t J, uint64_t* out) {
    pthread_mutex_lock(&g_initmu);
    jump_init_locked();
    const int ready = g_cp.ready;
    pthread_mutex_unlock(&g_initmu);
    if (ready != 1 || !out) return -1;
    const uint64_t* p = jump_poly(J);
    if (!p) return -1;
    memcpy(out, p, PW * sizeof(uint64_t));
    return 0;
}

int mppi_np_poly_words(void) { return PW; }

// glibc's struct log_data in the loaded libm: ln2hi, ln2lo, then poly[5] (poly[0] = -0x1.0000000000001p-1) and
// poly1[11] (poly1[0] = -0.5) — found by that signature in libm's read-only segments.
typedef struct {
    const double* hit[4];
    int n;
} LogScan;

static int log_scan_cb(struct dl_phdr_info* info, size_t size, void* data) {
    (void)size;
    LogScan* sc = (LogScan*)data;
    if (!info->dlpi_name || !strstr(info->dlpi_name, "libm.so")) return 0;
    const double sig[3] = {0x1.62e42fefa3800p-1, 0x1.ef35793c76730p-45, -0x1.0000000000001p-1};
    for (int h = 0; h < info->dlpi_phnum; ++h) {
        const ElfW(Phdr)* ph = &info->dlpi_phdr[h];
        if (ph->p_type != PT_LOAD || !(ph->p_flags & PF_R) || (ph->p_flags & PF_X) || ph->p_memsz < sizeof(sig))
            continue;
        const char* b = (const char*)(info->dlpi_addr + ph->p_vaddr);
        for (size_t o = 0; o + NPLOG_NDATA * sizeof(double) <= ph->p_memsz; o += 8) {
            if (memcmp(b + o, sig, sizeof(sig)) != 0) continue;
            const double* d = (const double*)(b + o);
            if (d[7] == -0.5 && sc->n < 4) sc->hit[sc->n++] = d;
        }
    }
    return 0;
}

// values the check compares: accepted polar r2 (the draw's domain), the near-1 band, spread exponents
static double log_check_value(uint64_t* st, int kind) {
    *st ^= *st << 13;
    *st ^= *st >> 7;
    *st ^= *st << 17;
    const uint64_t r = *st;
    if (kind == 0) {   // r2 = x1^2 + x2^2 of two legacy doubles, as an accepted attempt makes it
        const double x1 = 2.0 * legacy_double((uint32_t)r, (uint32_t)(r >> 32)) - 1.0;
        *st ^= *st << 13;
        *st ^= *st >> 7;
        *st ^= *st << 17;
        const double x2 = 2.0 * legacy_double((uint32_t)*st, (uint32_t)(*st >> 32)) - 1.0;
        const double r2 = x1 * x1 + x2 * x2;
        return r2 < 1.0 && r2 != 0.0 ? r2 : 0.5;
    }
    if (kind == 1) return 0.93 + (double)(r >> 11) * 0x1p-53 * 0.07;   // [0.93, 1): glibc's near-1 branch
    const uint64_t e = 1023 - 1 - (r % 105);                            // [2^-105, 1)
    return nplog_asdouble((e << 52) | (r >> 12));
}

// The constants of np_glibc_log (NPLOG_NDATA doubles) into out, after np_glibc_log on them equalled libm's
// log() bit for bit on `samples` inputs of each kind above.  0, or -1 (not found, or a mismatch: the libm in
// this process is not the variant np_glibc_log reproduces, and the device draw must not be used).
int mppi_np_log_params(double* out, int samples) {
    LogScan sc;
    memset(&sc, 0, sizeof(sc));
    dl_iterate_phdr(log_scan_cb, &sc);
    for (int h = 0; h < sc.n; ++h) {
        const double* D = sc.hit[h];
        uint64_t st = 0x9E3779B97F4A7C15ull;
        int ok = 1;
        for (int kind = 0; kind < 3 && ok; ++kind)
            for (int i = 0; i < samples; ++i) {
                volatile double x = log_check_value(&st, kind);   // volatile: log() on run-time values
                const double a = log(x), b = np_glibc_log(D, x);
                if (memcmp(&a, &b, 8) != 0) {
                    ok = 0;
                    break;
                }
            }
        if (ok) {
            memcpy(out, D, NPLOG_NDATA * sizeof(double));
            return 0;
        }
    }
    return -1;
}

// Tests: np_glibc_log against libm's log on n given values; returns the number that differ
int64_t mppi_np_log_mismatches(const double* D, const double* x, int64_t n) {
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double a = log(x[i]), b = np_glibc_log(D, x[i]);
        bad += memcmp(&a, &b, 8) != 0;
    }
    return bad;
}

// np.dot(z, M) of an (n, 2) by (2, 2) product as one candidate rounding of the host BLAS: out[i][j] =
// fma(z[i][1], M[1][j], z[i][0] * M[0][j]) (the product z0 M0j rounded, the second term fused into it: OpenBLAS's
// dgemm kernels accumulate k = 0, 1 with FMAs from a zero accumulator).  hostrng.dot2_model compares it with
// np.dot bit for bit at run time before the device draw applies the same operations (mppi_npgauss.hip).
void mppi_np_dot2_fma(const double* z, int64_t n, const double* M, double* out) {
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < 2; ++j) {
            const double p = z[2 * i] * M[j];
            out[2 * i + j] = fma(z[2 * i + 1], M[2 + j], p);
        }
}
