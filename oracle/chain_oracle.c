/* CPU ORACLE — test infrastructure only, never shipped, never on the product path.
 *
 * Plain-C fp64 restatement of the n-link planar-chain MPPI loop defined in
 * oracle/chain_oracle.py (the build-defined model for SURVEY §8 f4 / BASELINE
 * config 5; see that file for the equations and what pins them: at n = 2 with
 * inertia := length the model is the reference _F, control.py:234-263).
 * OpenMP over samples.  Used by tests/ for full-size parity of the chain kernel
 * and by bench.py's cpu_baseline leg for the chain workload.
 *
 * Noise addressing is strided so both the reference-style (K,T,n) layout and
 * the device-native (T,n,K) layout can be read: eps[k][t][d] = eps[k*sk + t*st + d*sd].
 */
#include <math.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define CH_MAX 8
#define SEARCH_IDX_LEN 30 /* control.py:203 */

typedef struct {
    int n;
    double mu[CH_MAX][CH_MAX], nu[CH_MAX], Dd[CH_MAX], fk[CH_MAX], J[CH_MAX], b[CH_MAX], g;
} chain_model;

/* chain[] = m[n], l[n], lc[n], I[n], fk[n], J[n], b[n], g  (chain_oracle.py ChainParams) */
static int chain_setup(chain_model *M, const double *chain, int n) {
    if (n < 1 || n > CH_MAX) return -1;
    const double *m = chain, *l = chain + n, *lc = chain + 2 * n, *I = chain + 3 * n, *fk = chain + 4 * n;
    const double *J = chain + 5 * n, *b = chain + 6 * n;
    memset(M, 0, sizeof(*M));
    M->n = n;
    M->g = chain[7 * n];
    for (int a = 0; a < n; ++a) {
        double tail = 0.0;
        for (int k = a + 1; k < n; ++k) tail += m[k];
        M->mu[a][a] = m[a] * lc[a] * lc[a] + l[a] * l[a] * tail;
        M->nu[a] = m[a] * lc[a] + l[a] * tail;
        M->Dd[a] = M->mu[a][a] + I[a] + J[a] + (a + 1 < n ? J[a + 1] : 0.0);  /* + S^-T diag(J) S^-1 */
        M->fk[a] = fk[a];
        M->J[a] = J[a];
        M->b[a] = b[a];
        for (int b = a + 1; b < n; ++b) {
            double tb = 0.0;
            for (int k = b + 1; k < n; ++k) tb += m[k];
            M->mu[a][b] = M->mu[b][a] = l[a] * (m[b] * lc[b] + l[b] * tb);
        }
    }
    return 0;
}

/* one semi-implicit Euler step: x = [q(n), dq(n)], v = joint torques (n) */
static void chain_step(double *x, const double *v, double dt, const chain_model *M) {
    const int n = M->n;
    double thd[CH_MAX], s[CH_MAX], c[CH_MAX], D[CH_MAX][CH_MAX], r[CH_MAX];
    double acc = 0.0, accd = 0.0;
    for (int a = 0; a < n; ++a) {
        acc += x[a];
        accd += x[n + a];
        thd[a] = accd;
        s[a] = sin(acc);
        c[a] = cos(acc);
    }
    for (int a = 0; a < n; ++a) {
        D[a][a] = M->Dd[a];
        double bias = 0.0;
        for (int b = 0; b < n; ++b) {
            if (b == a) continue;
            const double cab = c[a] * c[b] + s[a] * s[b]; /* cos(th_a - th_b) */
            const double sab = s[a] * c[b] - c[a] * s[b]; /* sin(th_a - th_b) */
            D[a][b] = M->mu[a][b] * cab - (b == a + 1 ? M->J[b] : 0.0) - (a == b + 1 ? M->J[a] : 0.0);
            bias += M->mu[a][b] * sab * thd[b] * thd[b];
        }
        const double va = v[a] - M->b[a] * x[n + a];                      /* joint torque - damping */
        const double vn = a + 1 < n ? v[a + 1] - M->b[a + 1] * x[n + a + 1] : 0.0;
        const double tau = va - vn;
        r[a] = tau - bias - M->g * M->nu[a] * c[a];
    }
    /* Cholesky D = L L^T (in place, lower), then L y = r, L^T z = y */
    for (int j = 0; j < n; ++j) {
        double d = D[j][j];
        for (int k = 0; k < j; ++k) d -= D[j][k] * D[j][k];
        d = sqrt(d);
        D[j][j] = d;
        for (int i = j + 1; i < n; ++i) {
            double e = D[i][j];
            for (int k = 0; k < j; ++k) e -= D[i][k] * D[j][k];
            D[i][j] = e / d;
        }
    }
    for (int i = 0; i < n; ++i) {
        double e = r[i];
        for (int k = 0; k < i; ++k) e -= D[i][k] * r[k];
        r[i] = e / D[i][i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double e = r[i];
        for (int k = i + 1; k < n; ++k) e -= D[k][i] * r[k];
        r[i] = e / D[i][i];
    }
    double prev = 0.0;
    for (int a = 0; a < n; ++a) {
        const double qdd = r[a] - prev;
        prev = r[a];
        x[n + a] += qdd * dt;
        x[a] += x[n + a] * dt;
    }
}

/* control.py:174-232 on the chain: end effector (x, y), windowed first argmin,
 * weighted squared error x 10000 on (x, y, dq_1, dq_2). */
static double chain_cost(const double *x, const double *win, int W, const double *w, const chain_model *M) {
    double px = 0.0, py = 0.0, acc = 0.0;
    for (int a = 0; a < M->n; ++a) {
        acc += x[a];
        px += M->fk[a] * cos(acc);
        py += M->fk[a] * sin(acc);
    }
    int jmin = 0;
    double dmin = INFINITY;
    for (int j = 0; j < W; ++j) {
        const double dx = px - win[4 * j], dy = py - win[4 * j + 1];
        const double d = (dx * dx + dy * dy) * 100;
        if (j == 0 || d < dmin) { dmin = d; jmin = j; }   /* control.py:213-215, as mppi_oracle.c */
    }
    const double *r = win + 4 * jmin;
    const double ex = px - r[0], ey = py - r[1], e1 = x[M->n] - r[2], e2 = x[M->n + 1] - r[3];
    return (w[0] * ex * ex + w[1] * ey * ey + w[2] * e1 * e1 + w[3] * e2 * e2) * 10000;
}

/* S[k] for samples [k_begin, k_end): x0[2n], u[T*n] (nominal), sigma_inv[n*n] row-major. */
int oracle_chain_rollout_costs_f64(const double *x0, const double *u, const float *eps, long sk, long st, long sd,
                                   int k_begin, int k_end, int T, int n, const double *win, int W, double dt,
                                   double lambda, double alpha, const double *sigma_inv, const double *stage_w,
                                   const double *term_w, long k_exploit, long k_offset, const double *chain,
                                   double *S_out, int nthreads) {
    chain_model M;
    if (chain_setup(&M, chain, n) != 0 || T <= 0 || W <= 0 || W > SEARCH_IDX_LEN || k_end < k_begin) return -1;
    const double gamma = lambda * (1.0 - alpha);
    double a[128 * CH_MAX];
    if (T > 128) return -1;
    for (int t = 0; t < T; ++t)
        for (int d = 0; d < n; ++d) {
            double acc = 0.0;
            for (int e = 0; e < n; ++e) acc += (gamma * u[t * n + e]) * sigma_inv[e * n + d];
            a[t * n + d] = acc;
        }
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int k = k_begin; k < k_end; ++k) {
        double x[2 * CH_MAX], v[CH_MAX];
        memcpy(x, x0, 2 * n * sizeof(double));
        double S = 0.0;
        const int exploit = (k + k_offset) < k_exploit;
        for (int t = 0; t < T; ++t) {
            double g = 0.0;
            for (int d = 0; d < n; ++d) {
                const double e = (double)eps[(long)k * sk + (long)t * st + (long)d * sd];
                v[d] = exploit ? u[t * n + d] + e : e;
                g += a[t * n + d] * v[d];
            }
            chain_step(x, v, dt, &M);
            S = S + (chain_cost(x, win, W, stage_w, &M) + g);
        }
        S_out[k - k_begin] = S + chain_cost(x, win, W, term_w, &M);
    }
    return 0;
}

/* control.py:112-118: w_eps[t*n + d] = sum_k w_k eps[k][t][d], sequential in k. */
int oracle_chain_weighted_noise_f64(const double *S, const float *eps, long sk, long st, long sd, int K, int T,
                                    int n, double lambda, double *w_out, double *w_eps_out) {
    if (K <= 0) return -1;
    double rho = S[0];
    for (int k = 1; k < K; ++k) rho = S[k] < rho ? S[k] : rho;
    double eta = 0.0;
    for (int k = 0; k < K; ++k) eta += exp((-1.0 / lambda) * (S[k] - rho));
    for (int i = 0; i < n * T; ++i) w_eps_out[i] = 0.0;
    for (int k = 0; k < K; ++k) {
        const double w = (1.0 / eta) * exp((-1.0 / lambda) * (S[k] - rho));
        if (w_out) w_out[k] = w;
        if (w == 0.0) continue;
        for (int t = 0; t < T; ++t)
            for (int d = 0; d < n; ++d)
                w_eps_out[t * n + d] += w * (double)eps[(long)k * sk + (long)t * st + (long)d * sd];
    }
    return 0;
}

/* States after each step for control rows ctrl[N][T][n]; out[N][T][2n]. */
int oracle_chain_traj_f64(const double *x0, const double *ctrl, int N, int T, int n, double dt, const double *chain,
                          double *out) {
    chain_model M;
    if (chain_setup(&M, chain, n) != 0) return -1;
    for (int i = 0; i < N; ++i) {
        double x[2 * CH_MAX];
        memcpy(x, x0, 2 * n * sizeof(double));
        for (int t = 0; t < T; ++t) {
            chain_step(x, ctrl + ((long)i * T + t) * n, dt, &M);
            memcpy(out + ((long)i * T + t) * 2 * n, x, 2 * n * sizeof(double));
        }
    }
    return 0;
}
