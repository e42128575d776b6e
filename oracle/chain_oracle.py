"""CPU ORACLE — test infrastructure only, never shipped, never on the product path.

fp64 NumPy restatement of the n-link planar-chain MPPI step that this build
defines for SURVEY §8 f4 / BASELINE config 5 ("7-DoF arm dynamics (extended
sys_params.py), K=131072 T=128, xydq_circle.txt reference").  The reference has
no 7-DoF model, so the model is BUILD-DEFINED and parity at n = 7 is UNPINNED by
the reference.  What IS pinned: at n = 2 with the reference's constants and its
mass-matrix convention (link inertia I_i := l_i, control.py:241-245) the chain
dynamics reduce term by term to the reference ``_F`` (control.py:234-263);
``tests/test_chain_oracle.py`` checks that against ``mppi_oracle`` (itself pinned
to the reference fixtures) and checks the whole n = 2 chain step against the
reference's golden steps.

Model (planar chain, joint angles q, absolute angles theta = S q, S = lower-
triangular ones, so theta_a = q_1 + ... + q_a):

  kinetic energy  T = 1/2 theta_dot^T D(theta) theta_dot,
                  D_ab = mu_ab cos(theta_a - theta_b) + delta_ab I_a
  mu_ab (a < b)   = l_a (m_b lc_b + l_b sum_{k>b} m_k)          (constant)
  mu_aa           = m_a lc_a^2 + l_a^2 sum_{k>a} m_k
  bias            c_a = sum_b mu_ab sin(theta_a - theta_b) theta_dot_b^2
  gravity         g_a = g nu_a cos theta_a,  nu_a = m_a lc_a + l_a sum_{k>a} m_k
  joint drives    armature (rotor inertia) J_a and viscous damping b_a per joint: the
                  joint-space mass matrix S^T D S + diag(J) is, in theta-space,
                  D' = D + S^-T diag(J) S^-1  (diagonal + J_a + J_{a+1}, first
                  off-diagonal - J_{a+1}); the joint torques are u - b dq
  joint torques   u' = u - b dq map to theta-space as tau_a = u'_a - u'_{a+1}  (u'_{n+1} = 0)
  D' theta_ddot = tau - c - g;  q_ddot_1 = theta_ddot_1, q_ddot_a = theta_ddot_a - theta_ddot_{a-1}
  semi-implicit Euler as control.py:256-259: dq += q_ddot dt; q += dq dt

(At n = 2 with J = b = 0: M = S^T D S gives M11 = m1 lc1^2 + m2 l1^2 + I1 + 2 m2 l1 lc2 c2 + m2 lc2^2 + I2,
M12 = m2 l1 lc2 c2 + m2 lc2^2 + I2, M22 = m2 lc2^2 + I2 — control.py:241-245 with I = l.)

Cost: end-effector (x, y) from forward kinematics with the fk
lengths, the windowed nearest waypoint of control.py:200-232, and the
reference's 4-term weighted squared error x 10000 on (x, y, dq_1, dq_2) against
xydq_circle.txt's (x, y, dq1, dq2) columns; control cost (gamma u_t^T Sigma^-1) v
(control.py:106) with the n x n Sigma; weights / weighted noise / median filter /
update / shift exactly as the 2-DoF step (control.py:112-152).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

import mppi_oracle as O

MAX_DOF = 8


def _default(v):
    return field(default_factory=lambda: tuple(v))


@dataclass(frozen=True)
class ChainParams:
    """Link constants of an n-link planar chain (build-defined 'extended sys_params')."""
    m: tuple = _default([1.0] * 7)
    l: tuple = _default([2.0 / 7.0] * 7)
    lc: tuple = _default([1.0 / 7.0] * 7)
    I: tuple = _default([(2.0 / 7.0) ** 2 / 12.0] * 7)   # slender rods, m l^2 / 12
    fk: tuple = _default([2.0 / 7.0] * 7)                # lengths used by the cost's kinematics
    J: tuple = _default([0.1] * 7)                       # joint armature (rotor inertia), kg m^2
    b: tuple = _default([1.0] * 7)                       # joint viscous damping, N m s / rad
    g: float = 9.81

    @property
    def n(self) -> int:
        return len(self.m)

    @staticmethod
    def from_arm2(a: O.ArmParams = O.ArmParams()) -> "ChainParams":
        """The reference 2-link model (control.py:11-18, 241-245): inertia := link length."""
        return ChainParams(m=(a.m1, a.m2), l=(a.l1, a.l2), lc=(a.lc1, a.lc2), I=(a.l1, a.l2),
                           fk=(a.fk_l1, a.fk_l2), J=(0.0, 0.0), b=(0.0, 0.0), g=a.g)


def coefficients(P: ChainParams):
    """(mu n x n, nu n, D' diagonal n): the constant parts of D' and gravity."""
    n = P.n
    m, l, lc = map(np.asarray, (P.m, P.l, P.lc))
    tail = np.array([m[k + 1:].sum() for k in range(n)])        # sum_{k>a} m_k
    mu = np.zeros((n, n))
    for a in range(n):
        mu[a, a] = m[a] * lc[a] ** 2 + l[a] ** 2 * tail[a]
        for b in range(a + 1, n):
            mu[a, b] = mu[b, a] = l[a] * (m[b] * lc[b] + l[b] * tail[b])
    nu = m * lc + l * tail
    J = np.asarray(P.J, dtype=np.float64)
    return mu, nu, np.diag(mu) + np.asarray(P.I) + J + np.append(J[1:], 0.0)


def chain_forward_dynamics(q, dq, v, dt, P: ChainParams):
    """One semi-implicit Euler step of the chain, vectorised over leading dims (..., n)."""
    mu, nu, Dd = coefficients(P)
    th = np.cumsum(q, axis=-1)
    thd = np.cumsum(dq, axis=-1)
    dth = th[..., :, None] - th[..., None, :]                   # theta_a - theta_b
    D = mu * np.cos(dth)
    idx = np.arange(P.n)
    D[..., idx, idx] = Dd
    J = np.asarray(P.J, dtype=np.float64)
    D[..., idx[:-1], idx[1:]] -= J[1:]
    D[..., idx[1:], idx[:-1]] -= J[1:]
    c = np.einsum("ab,...ab,...b->...a", mu, np.sin(dth), thd ** 2)
    gt = P.g * nu * np.cos(th)
    ve = v - np.asarray(P.b) * dq
    tau = ve - np.concatenate([ve[..., 1:], np.zeros(ve.shape[:-1] + (1,))], axis=-1)
    thdd = np.linalg.solve(D, (tau - c - gt)[..., None])[..., 0]
    qdd = np.diff(thdd, axis=-1, prepend=0.0)
    dq_n = dq + qdd * dt
    q_n = q + dq_n * dt
    return q_n, dq_n


def chain_fk(q, P: ChainParams):
    """End effector (x, y) with the cost's link lengths."""
    th = np.cumsum(q, axis=-1)
    fk = np.asarray(P.fk)
    return (fk * np.cos(th)).sum(-1), (fk * np.sin(th)).sum(-1)


def nearest_waypoint_xy(x, y, ref_path, prev_idx):
    """control.py:200-232 on an end-effector position (d.index(min(d)), O.first_min_index)."""
    win = ref_path[prev_idx:prev_idx + O.SEARCH_IDX_LEN]
    d = ((np.asarray(x)[..., None] - win[:, 0]) ** 2 + (np.asarray(y)[..., None] - win[:, 1]) ** 2) * 100
    idx = O.first_min_index(d) + prev_idx
    return idx, ref_path[idx, 0], ref_path[idx, 1], ref_path[idx, 2], ref_path[idx, 3]


def chain_state_cost(q, dq, ref_path, prev_idx, weight, P: ChainParams):
    """control.py:174-198 on (x, y, dq_1, dq_2) of the chain."""
    x, y = chain_fk(q, P)
    _, rx, ry, r1, r2 = nearest_waypoint_xy(x, y, ref_path, prev_idx)
    c = weight[0] * (x - rx) ** 2 + weight[1] * (y - ry) ** 2 + \
        weight[2] * (dq[..., 0] - r1) ** 2 + weight[3] * (dq[..., 1] - r2) ** 2
    return c * 10000


def chain_rollout_costs(x0, u, eps, ref_path, prev_idx, dt, lam, alpha, sigma, stage_w, term_w,
                        expl=0.0, P: ChainParams = ChainParams(), k_offset=0, K_total=None):
    """The K x T loop (control.py:81-109 with the chain model).  eps (K, T, n); returns S (K,)."""
    K, T, n = eps.shape
    K_total = K if K_total is None else K_total
    gamma = lam * (1.0 - alpha)
    sig_inv = np.linalg.inv(sigma)
    exploit = (np.arange(K) + k_offset) < (1.0 - expl) * K_total
    q = np.tile(np.asarray(x0[:n], dtype=np.float64), (K, 1))
    dq = np.tile(np.asarray(x0[n:], dtype=np.float64), (K, 1))
    S = np.zeros(K)
    for t in range(T):
        e = eps[:, t, :].astype(np.float64)
        v = np.where(exploit[:, None], u[t] + e, e)
        q, dq = chain_forward_dynamics(q, dq, v, dt, P)
        a = (gamma * u[t]) @ sig_inv
        S = S + (chain_state_cost(q, dq, ref_path, prev_idx, stage_w, P) + v @ a)
    return S + chain_state_cost(q, dq, ref_path, prev_idx, term_w, P)


def chain_rollout_trajectory(x0, controls, dt, P: ChainParams = ChainParams()):
    """States (..., T, 2n) driven by ``controls`` (..., T, n) (control.py:129-145 analogue)."""
    controls = np.asarray(controls, dtype=np.float64)
    n = P.n
    lead, T = controls.shape[:-2], controls.shape[-2]
    q = np.broadcast_to(np.asarray(x0[:n], dtype=np.float64), lead + (n,)).copy()
    dq = np.broadcast_to(np.asarray(x0[n:], dtype=np.float64), lead + (n,)).copy()
    out = np.zeros(lead + (T, 2 * n))
    for t in range(T):
        q, dq = chain_forward_dynamics(q, dq, controls[..., t, :], dt, P)
        out[..., t, :n] = q
        out[..., t, n:] = dq
    return out


def gravity_torque(q, P: ChainParams = ChainParams()):
    """Joint torques holding the chain still at q (tau = S^T g_theta): a natural u_prev init."""
    _, nu, _ = coefficients(P)
    g_th = P.g * nu * np.cos(np.cumsum(q))
    return np.cumsum(g_th[::-1])[::-1]


class ChainOracleController:
    """Stateful fp64 restatement of the chain controller (control.py:20-152 with the chain model)."""

    def __init__(self, delta_t, ref_path, horizon_step_T, number_of_samples_K, param_exploration, param_lambda,
                 param_alpha, sigma, stage_cost_weight, terminal_cost_weight, chain: ChainParams = ChainParams(),
                 u_init=None, visualize_optimal_traj=True, visualze_sampled_trajs=False):
        self.chain = chain
        self.dim_u, self.dim_x = chain.n, 2 * chain.n
        self.T, self.K = horizon_step_T, number_of_samples_K
        self.param_exploration, self.param_lambda, self.param_alpha = param_exploration, param_lambda, param_alpha
        self.Sigma = np.asarray(sigma, dtype=np.float64)
        self.stage_cost_weight, self.terminal_cost_weight = stage_cost_weight, terminal_cost_weight
        self.delta_t, self.ref_path = delta_t, ref_path
        self.visualize_optimal_traj, self.visualze_sampled_trajs = visualize_optimal_traj, visualze_sampled_trajs
        u0 = np.zeros(self.dim_u) if u_init is None else np.asarray(u_init, dtype=np.float64)
        self.u_prev = np.tile(u0, (self.T, 1)) if u0.ndim == 1 else u0.copy()
        self.prev_waypoints_idx = 0
        self.last = {}

    def calc_control_input(self, observed_x, epsilon):
        n = self.dim_u
        u = self.u_prev
        x0 = np.asarray(observed_x, dtype=np.float64)
        ex, ey = chain_fk(x0[:n], self.chain)
        idx, *_ = nearest_waypoint_xy(ex, ey, self.ref_path, self.prev_waypoints_idx)
        self.prev_waypoints_idx = int(idx)
        if self.prev_waypoints_idx >= self.ref_path.shape[0] - 1:
            raise IndexError
        eps = np.asarray(epsilon, dtype=np.float64)
        S = chain_rollout_costs(x0, u, eps, self.ref_path, self.prev_waypoints_idx, self.delta_t,
                                self.param_lambda, self.param_alpha, self.Sigma, self.stage_cost_weight,
                                self.terminal_cost_weight, self.param_exploration, self.chain)
        w = O.compute_weights(S, self.param_lambda)
        w_eps_raw = O.weighted_noise(w, eps)
        w_eps = O.moving_median_filter(w_eps_raw, 10)
        u_before = u.copy()
        u += w_eps
        u_new = u.copy()
        optimal = np.zeros((self.T, self.dim_x))
        if self.visualize_optimal_traj:
            optimal = chain_rollout_trajectory(x0, np.roll(u, 1, axis=0), self.delta_t, self.chain)
        sampled = np.zeros((self.K, self.T, self.dim_x))
        if self.visualze_sampled_trajs:
            kx = (np.arange(self.K) < (1.0 - self.param_exploration) * self.K)[:, None, None]
            v = np.where(kx, u_before[None] + eps, eps)
            sampled = chain_rollout_trajectory(x0, np.roll(v, 1, axis=1), self.delta_t, self.chain)
        self.u_prev[:-1] = u[1:]
        self.u_prev[-1] = u[-1]
        self.last = dict(S=S, w=w, w_eps_raw=w_eps_raw, w_eps_filt=w_eps, u_new=u_new, eps=eps)
        return u[0], u, optimal, sampled
