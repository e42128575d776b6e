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
// Host code, never on the device path; the Python side (controller.py,
// legacy_multivariate_normal) does the rest of multivariate_normal with
// NumPy's own calls.
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

// next key array from the previous one, out of place (no aliasing: the loops vectorize); the same values as
// NumPy's in-place mt19937_gen
static void mt_twist_to(const uint32_t* __restrict__ o, uint32_t* __restrict__ k) {
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

static void* count_pass(void* p) {
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
static int legacy_gauss_locked(uint32_t* key, int* pos, int* has_gauss, double* gauss, double* out, int64_t n,
                               int nthreads) {
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
        for (int64_t b = 1; b < nblk; ++b) mt_twist_to(blocks + (b - 1) * MT_N, blocks + b * MT_N);
        Work wk[64];
        pthread_t th[64];
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
        for (int t = 1; t < nt; ++t) pthread_create(&th[t], NULL, count_pass, &wk[t]);
        count_pass(&wk[0]);
        for (int t = 1; t < nt; ++t) pthread_join(th[t], NULL);
        int64_t total = 0;
        for (int t = 0; t < nt; ++t) {
            wk[t].first_pair = total;
            total += wk[t].count;
        }
        if (total < pairs) {   // too few attempts generated (vanishingly rare): more, from the same state
            A = A + A / 2;
            continue;
        }
        for (int t = 1; t < nt; ++t) pthread_create(&th[t], NULL, write_pass, &wk[t]);
        write_pass(&wk[0]);
        for (int t = 1; t < nt; ++t) pthread_join(th[t], NULL);
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
