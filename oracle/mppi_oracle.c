/* CPU ORACLE — test infrastructure only, never shipped, never on the product path.
 *
 * Plain-C fp64 restatement of the reference MPPI hot loop
 * (junofficial/mppi_RobotArm control.py:81-118), OpenMP over samples.  Used by
 * tests/ (large-size parity on sample subsets) and by bench.py's cpu_baseline
 * leg (kind "port").  The HIP product library never links or loads this.
 *
 * Parity is pinned through oracle/mppi_oracle.py (itself checked against the
 * golden fixtures captured from the imported reference); tests compare the two
 * restatements sample by sample.  The only intended difference from the
 * reference arithmetic is the 2x2 inverse: closed form here, LAPACK getrf/getri
 * via np.linalg.inv in the reference (control.py:252) — ~1 ulp.
 *
 * Noise addressing is strided so both the reference (K,T,2) layout and the
 * device-native (T,K,2) layout can be read: eps[k][t][d] = eps[k*sk + t*st + d].
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define SEARCH_IDX_LEN 30 /* control.py:203 */

typedef struct {
    double m1, m2, l1, l2, lc1, lc2, g; /* sys_params.py:1-13 */
    double fk_l1, fk_l2;                /* control.py:55-56 */
} oracle_arm;

/* _F, control.py:234-263 (semi-implicit Euler, mass matrix as written) */
static inline void oracle_F(double x[4], double u1, double u2, double dt, const oracle_arm *p) {
    const double q1 = x[0], q2 = x[1], dq1 = x[2], dq2 = x[3];
    const double c2 = cos(q2);
    const double M11 = p->m1 * p->lc1 * p->lc1 + p->l1 +
                       p->m2 * (p->l1 * p->l1 + p->lc2 * p->lc2 + 2 * p->l1 * p->lc2 * c2) + p->l2;
    const double M22 = p->m2 * p->lc2 * p->lc2 + p->l2;
    const double M12 = p->m2 * p->l1 * p->lc2 * c2 + p->m2 * p->lc2 * p->lc2 + p->l2;
    const double h = p->m2 * p->l1 * p->lc2 * sin(q2);
    const double g1 = p->m1 * p->lc1 * p->g * cos(q1) + p->m2 * p->g * (p->lc2 * cos(q1 + q2) + p->l1 * cos(q1));
    const double g2 = p->m2 * p->lc2 * p->g * cos(q1 + q2);
    const double cdq1 = (-h * dq2) * dq1 + (-h * dq1 - h * dq2) * dq2;
    const double cdq2 = (h * dq1) * dq1;
    const double r1 = (u1 - cdq1) - g1, r2 = (u2 - cdq2) - g2;
    const double det = M11 * M22 - M12 * M12;
    const double ddq1 = (M22 * r1 - M12 * r2) / det;
    const double ddq2 = (-M12 * r1 + M11 * r2) / det;
    const double ndq1 = dq1 + ddq1 * dt, ndq2 = dq2 + ddq2 * dt;
    x[0] = q1 + ndq1 * dt;
    x[1] = q2 + ndq2 * dt;
    x[2] = ndq1;
    x[3] = ndq2;
}

/* _c / _phi with _get_nearest_waypoint (control.py:174-232); window = W rows of
 * [x, y, dq1, dq2] already sliced at prev_waypoints_idx.  Returns the cost and
 * writes the window-relative argmin. */
static inline double oracle_cost(const double x[4], const double *win, int W, const double w[4],
                                 const oracle_arm *p, int *jmin_out) {
    const double q1 = x[0], q2 = x[1];
    const double px = p->fk_l1 * cos(q1) + p->fk_l2 * cos(q1 + q2);
    const double py = p->fk_l1 * sin(q1) + p->fk_l2 * sin(q1 + q2);
    int jmin = 0;
    double dmin = INFINITY;
    for (int j = 0; j < W; ++j) {
        const double dx = px - win[4 * j], dy = py - win[4 * j + 1];
        const double d = (dx * dx + dy * dy) * 100;
        if (j == 0 || d < dmin) { dmin = d; jmin = j; } /* min(d): d[0], replaced on a strict <; list.index */
    }
    const double *r = win + 4 * jmin;
    const double ex = px - r[0], ey = py - r[1], e1 = x[2] - r[2], e2 = x[3] - r[3];
    if (jmin_out) *jmin_out = jmin;
    return (w[0] * ex * ex + w[1] * ey * ey + w[2] * e1 * e1 + w[3] * e2 * e2) * 10000;
}

/* S[k] for samples [k_begin, k_end) of one control step (control.py:81-109).
 *   x0[4], u[T*2] (nominal, fp64), sigma_inv[4] row-major,
 *   k_exploit: global samples k < k_exploit use u + eps, others eps only (control.py:98),
 *   k_offset: global index of local sample 0. */
int oracle_rollout_costs_f64(const double *x0, const double *u, const float *eps, long sk, long st,
                             int k_begin, int k_end, int T, const double *win, int W, double dt,
                             double lambda, double alpha, const double *sigma_inv,
                             const double *stage_w, const double *term_w, long k_exploit,
                             long k_offset, const double *arm, double *S_out, int nthreads) {
    if (T <= 0 || W <= 0 || W > SEARCH_IDX_LEN || k_end < k_begin) return -1;
    oracle_arm p;
    memcpy(&p, arm, sizeof(p));
    const double gamma = lambda * (1.0 - alpha);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int k = k_begin; k < k_end; ++k) {
        double x[4] = {x0[0], x0[1], x0[2], x0[3]};
        double S = 0.0;
        const int exploit = (k + k_offset) < k_exploit;
        for (int t = 0; t < T; ++t) {
            const float *e = eps + (long)k * sk + (long)t * st;
            const double v1 = exploit ? u[2 * t] + (double)e[0] : (double)e[0];
            const double v2 = exploit ? u[2 * t + 1] + (double)e[1] : (double)e[1];
            oracle_F(x, v1, v2, dt, &p);
            const double c = oracle_cost(x, win, W, stage_w, &p, NULL);
            const double a0 = (gamma * u[2 * t]) * sigma_inv[0] + (gamma * u[2 * t + 1]) * sigma_inv[2];
            const double a1 = (gamma * u[2 * t]) * sigma_inv[1] + (gamma * u[2 * t + 1]) * sigma_inv[3];
            S = S + (c + (a0 * v1 + a1 * v2));
        }
        S = S + oracle_cost(x, win, W, term_w, &p, NULL);
        S_out[k - k_begin] = S;
    }
    return 0;
}

/* _compute_weights + weighted noise (control.py:112-118) over K samples:
 * w_eps[t*2+d] = sum_k w_k eps[k][t][d], sequential in k. */
int oracle_weighted_noise_f64(const double *S, const float *eps, long sk, long st, int K, int T,
                              double lambda, double *w_out, double *w_eps_out) {
    if (K <= 0) return -1;
    double rho = S[0];
    for (int k = 1; k < K; ++k) rho = S[k] < rho ? S[k] : rho;
    double eta = 0.0;
    for (int k = 0; k < K; ++k) eta += exp((-1.0 / lambda) * (S[k] - rho));
    for (int i = 0; i < 2 * T; ++i) w_eps_out[i] = 0.0;
    for (int k = 0; k < K; ++k) {
        const double w = (1.0 / eta) * exp((-1.0 / lambda) * (S[k] - rho));
        if (w_out) w_out[k] = w;
        for (int t = 0; t < T; ++t)
            for (int d = 0; d < 2; ++d) w_eps_out[2 * t + d] += w * (double)eps[(long)k * sk + (long)t * st + d];
    }
    return 0;
}

/* Trajectory re-roll (control.py:129-145): states after each step for control
 * rows ctrl[n][t][2]; out[n][t][4]. */
int oracle_rollout_traj_f64(const double *x0, const double *ctrl, int N, int T, double dt,
                            const double *arm, double *out) {
    oracle_arm p;
    memcpy(&p, arm, sizeof(p));
    for (int n = 0; n < N; ++n) {
        double x[4] = {x0[0], x0[1], x0[2], x0[3]};
        for (int t = 0; t < T; ++t) {
            oracle_F(x, ctrl[((long)n * T + t) * 2], ctrl[((long)n * T + t) * 2 + 1], dt, &p);
            memcpy(out + ((long)n * T + t) * 4, x, sizeof(x));
        }
    }
    return 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
