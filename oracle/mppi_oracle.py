"""CPU ORACLE — test infrastructure only, never shipped, never on the product path.

A vectorised fp64 NumPy restatement of the reference MPPI step
(junofficial/mppi_RobotArm ``control.py:67-152``), used ONLY by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the
checker.  The HIP product path (``mppi_robotarm_amd``) never imports this file.

Parity is PINNED: ``tests/test_oracle_golden.py`` checks this restatement
against the golden fixtures captured from the imported reference
(``tests/golden/make_golden.py``) — S to ~1e-15 relative, u bit-for-bit in the
one-hot regime, closed loops tick by tick.

Every function cites the reference line it restates.  Quirks kept on purpose
(SURVEY §3.3): the returned ``u0`` is the post-shift row, ``u_seq`` aliases
``u_prev``, the median filter is scipy's upper median with ``reflect``
boundaries, the optimal / sampled trajectories use the off-by-one control
``u[t-1]`` (``t = 0`` reads ``u[-1]``), the weighted noise uses ``eps`` (not
``v``), the nearest-waypoint window is shared by every sample and step of one
control step, and ``_F`` (link lengths from ``sys_params``) and the
kinematics in the cost (``self.l1 = self.l2 = 1``) keep separate lengths.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

SEARCH_IDX_LEN = 30  # control.py:203


@dataclass(frozen=True)
class ArmParams:
    """sys_params.py:1-13 (constants used by ``_F``, control.py:11-18)."""
    m1: float = 1.0
    m2: float = 1.0
    l1: float = 1.0
    l2: float = 1.0
    lc1: float = 0.5
    lc2: float = 0.5
    g: float = 9.81
    # forward kinematics inside the cost / waypoint search: control.py:55-56
    fk_l1: float = 1.0
    fk_l2: float = 1.0


def forward_dynamics(q1, q2, dq1, dq2, u1, u2, dt, p: ArmParams):
    """``_F`` (control.py:234-263), vectorised over samples.

    Mass matrix exactly as written (control.py:241-245: link lengths stand in
    for the link inertias); ``np.linalg.inv`` of the stacked 2x2 matrices as at
    control.py:252; semi-implicit Euler (control.py:256, 259).
    """
    c2 = np.cos(q2)
    M11 = p.m1 * p.lc1 ** 2 + p.l1 + p.m2 * (p.l1 ** 2 + p.lc2 ** 2 + 2 * p.l1 * p.lc2 * c2) + p.l2
    M22 = p.m2 * p.lc2 ** 2 + p.l2
    M12 = p.m2 * p.l1 * p.lc2 * c2 + p.m2 * p.lc2 ** 2 + p.l2
    M21 = M12
    h = p.m2 * p.l1 * p.lc2 * np.sin(q2)
    g1 = p.m1 * p.lc1 * p.g * np.cos(q1) + p.m2 * p.g * (p.lc2 * np.cos(q1 + q2) + p.l1 * np.cos(q1))
    g2 = p.m2 * p.lc2 * p.g * np.cos(q1 + q2)
    # C.dot(dq) with C = [[-h dq2, -h dq1 - h dq2], [h dq1, 0]]   (control.py:251)
    cdq1 = (-h * dq2) * dq1 + (-h * dq1 - h * dq2) * dq2
    cdq2 = (h * dq1) * dq1 + 0.0 * dq2
    r1 = (u1 - cdq1) - g1
    r2 = (u2 - cdq2) - g2
    n = np.broadcast(q1, q2).shape
    M = np.empty(n + (2, 2))
    M[..., 0, 0] = M11
    M[..., 0, 1] = M12
    M[..., 1, 0] = M21
    M[..., 1, 1] = M22
    Mi = np.linalg.inv(M)
    ddq1 = Mi[..., 0, 0] * r1 + Mi[..., 0, 1] * r2
    ddq2 = Mi[..., 1, 0] * r1 + Mi[..., 1, 1] * r2
    dq1n = dq1 + ddq1 * dt
    dq2n = dq2 + ddq2 * dt
    q1n = q1 + dq1n * dt
    q2n = q2 + dq2n * dt
    return q1n, q2n, dq1n, dq2n


def arm_dynamic(q, dq, u, p: ArmParams = ArmParams()):
    """Plant ``Arm_Dynamic`` (utils.py:14-29): returns ddq for the host loop."""
    c2 = np.cos(q[1])
    M11 = p.m1 * p.lc1 ** 2 + p.l1 + p.m2 * (p.l1 ** 2 + p.lc2 ** 2 + 2 * p.l1 * p.lc2 * c2) + p.l2
    M22 = p.m2 * p.lc2 ** 2 + p.l2
    M12 = p.m2 * p.l1 * p.lc2 * c2 + p.m2 * p.lc2 ** 2 + p.l2
    M = np.array([[M11, M12], [M12, M22]])
    h = p.m2 * p.l1 * p.lc2 * np.sin(q[1])
    g1 = p.m1 * p.lc1 * p.g * np.cos(q[0]) + p.m2 * p.g * (p.lc2 * np.cos(q[0] + q[1]) + p.l1 * np.cos(q[0]))
    g2 = p.m2 * p.lc2 * p.g * np.cos(q[0] + q[1])
    C = np.array([[-h * dq[1], -h * dq[0] - h * dq[1]], [h * dq[0], 0]])
    return np.linalg.inv(M).dot(u - C.dot(dq) - np.array([g1, g2]))


def forward_kinematics(q, p: ArmParams = ArmParams()):
    """``Forward_Kinemetic`` (utils.py:32-38)."""
    x1 = p.l1 * np.cos(q[0])
    y1 = p.l1 * np.sin(q[0])
    x2 = p.l1 * np.cos(q[0]) + p.l2 * np.cos(q[0] + q[1])
    y2 = p.l1 * np.sin(q[0]) + p.l2 * np.sin(q[0] + q[1])
    return x1, y1, x2, y2


def first_min_index(d):
    """``d.index(min(d))`` (control.py:213-215) along the last axis.  Python's
    min() keeps d[0] and replaces it only on a strict '<': a NaN at j > 0 is
    never chosen, a NaN at j = 0 always is (np.argmin returns the first NaN)."""
    j = np.argmin(d, axis=-1)
    nan = np.isnan(np.take_along_axis(d, np.asarray(j)[..., None], axis=-1)[..., 0])
    if np.any(nan):
        alt = np.argmin(np.where(np.isnan(d), np.inf, d), axis=-1)   # the first minimum of the numbers
        alt = np.where(np.isnan(d[..., 0]), 0, alt)
        j = np.where(nan, alt, j)
    return j


def nearest_waypoint(q1, q2, ref_path, prev_idx, p: ArmParams):
    """``_get_nearest_waypoint`` (control.py:200-232) vectorised over samples.

    Window ``ref_path[prev:prev+30]`` (slice-truncated at the path end),
    ``d.index(min(d))`` of ``((x-rx)^2 + (y-ry)^2) * 100`` (control.py:212-215).
    Returns (nearest_idx, ref_x, ref_y, ref_dq1, ref_dq2).
    """
    x = p.fk_l1 * np.cos(q1) + p.fk_l2 * np.cos(q1 + q2)
    y = p.fk_l1 * np.sin(q1) + p.fk_l2 * np.sin(q1 + q2)
    win = ref_path[prev_idx:prev_idx + SEARCH_IDX_LEN]
    dx = np.asarray(x)[..., None] - win[:, 0]
    dy = np.asarray(y)[..., None] - win[:, 1]
    d = (dx ** 2 + dy ** 2) * 100
    j = first_min_index(d)
    idx = j + prev_idx
    return idx, ref_path[idx, 0], ref_path[idx, 1], ref_path[idx, 2], ref_path[idx, 3]


def state_cost(q1, q2, dq1, dq2, ref_path, prev_idx, weight, p: ArmParams):
    """``_c`` / ``_phi`` (control.py:174-198): weighted squared error x 10000."""
    x = p.fk_l1 * np.cos(q1) + p.fk_l2 * np.cos(q1 + q2)
    y = p.fk_l1 * np.sin(q1) + p.fk_l2 * np.sin(q1 + q2)
    _, rx, ry, rdq1, rdq2 = nearest_waypoint(q1, q2, ref_path, prev_idx, p)
    c = weight[0] * (x - rx) ** 2 + weight[1] * (y - ry) ** 2 + \
        weight[2] * (dq1 - rdq1) ** 2 + weight[3] * (dq2 - rdq2) ** 2
    return c * 10000


def rollout_costs(x0, u, eps, ref_path, prev_idx, dt, lam, alpha, sigma, stage_w, term_w,
                  expl=0.0, p: ArmParams = ArmParams(), k_offset=0, K_total=None, gamma=None):
    """The K x T hot loop, control.py:81-109.  Returns S (K,) fp64.

    ``k_offset`` / ``K_total`` restate the exploration split
    ``k < (1 - expl) * K`` (control.py:98) for a shard of a larger sample set.
    ``gamma``: the controller's ``param_gamma`` (fixed at construction,
    control.py:45, read at :106); default lam (1 - alpha).
    """
    K, T, _ = eps.shape
    K_total = K if K_total is None else K_total
    if gamma is None:
        gamma = lam * (1.0 - alpha)                   # control.py:45
    sig_inv = np.linalg.inv(sigma)                    # control.py:106 (raises on singular)
    kg = np.arange(K) + k_offset
    exploit = kg < (1.0 - expl) * K_total             # control.py:98
    S = np.zeros(K)
    q1 = np.full(K, float(x0[0]))
    q2 = np.full(K, float(x0[1]))
    dq1 = np.full(K, float(x0[2]))
    dq2 = np.full(K, float(x0[3]))
    for t in range(1, T + 1):
        e = eps[:, t - 1, :].astype(np.float64)
        v1 = np.where(exploit, u[t - 1, 0] + e[:, 0], e[:, 0])   # control.py:99-101
        v2 = np.where(exploit, u[t - 1, 1] + e[:, 1], e[:, 1])
        q1, q2, dq1, dq2 = forward_dynamics(q1, q2, dq1, dq2, v1, v2, dt, p)
        c = state_cost(q1, q2, dq1, dq2, ref_path, prev_idx, stage_w, p)
        a = (gamma * u[t - 1].T) @ sig_inv            # ((γ uᵀ) Σ⁻¹) v, left-to-right
        S = S + (c + (a[0] * v1 + a[1] * v2))
    S = S + state_cost(q1, q2, dq1, dq2, ref_path, prev_idx, term_w, p)   # control.py:109
    return S


def compute_weights(S, lam):
    """``_compute_weights`` (control.py:297-314), sequential sums as in the loops."""
    rho = S.min()
    e = np.exp((-1.0 / lam) * (S - rho))
    eta = np.cumsum(e)[-1] if e.size else 0.0
    return (1.0 / eta) * e


def weighted_noise(w, eps):
    """control.py:115-118: w_eps[t] = sum_k w[k] eps[k,t], k in order."""
    return np.cumsum(w[:, None, None] * eps.astype(np.float64), axis=0)[-1]


def median_filter_reflect(x, size=10):
    """``scipy.ndimage.median_filter(x, size, mode='reflect')`` (control.py:325).

    Window [i - size//2, i + size - size//2 - 1], half-sample-symmetric
    ('reflect': d c b a | a b c d | d c b a) boundaries, rank size//2 of the
    sorted window (the UPPER median for even sizes).
    """
    x = np.asarray(x, dtype=np.float64)
    n = x.shape[0]
    if n < 5 and size == 10:
        # SciPy 1.15.3's 1-D rank filter does not follow its own 'reflect'
        # definition when the input is shorter than half the window (n <= 3
        # returns zeros, n = 4 differs); the reference inherits that, so the
        # pinned dependency itself is the oracle for horizons T < 5.
        from scipy.ndimage import median_filter
        return median_filter(x, size=size, mode="reflect")
    lo = size // 2
    out = np.empty(n)
    for i in range(n):
        idx = np.arange(i - lo, i - lo + size)
        # reflect with period 2n: index -1 -> 0, -2 -> 1, n -> n-1, ...
        m = np.mod(idx, 2 * n)
        m = np.where(m >= n, 2 * n - 1 - m, m)
        out[i] = np.sort(x[m])[size // 2]
    return out


def moving_median_filter(xx, window_size=10):
    """``_moving_median_filter`` (control.py:319-327): per column."""
    out = np.zeros(xx.shape)
    for d in range(xx.shape[1]):
        out[:, d] = median_filter_reflect(xx[:, d], window_size)
    return out


def rollout_trajectory(x0, controls, dt, p: ArmParams = ArmParams()):
    """control.py:129-145: states after each of T steps driven by ``controls`` (..., T, 2)."""
    controls = np.asarray(controls, dtype=np.float64)
    lead = controls.shape[:-2]
    T = controls.shape[-2]
    q1 = np.full(lead, float(x0[0]))
    q2 = np.full(lead, float(x0[1]))
    dq1 = np.full(lead, float(x0[2]))
    dq2 = np.full(lead, float(x0[3]))
    out = np.zeros(lead + (T, 4))
    for t in range(T):
        q1, q2, dq1, dq2 = forward_dynamics(q1, q2, dq1, dq2, controls[..., t, 0], controls[..., t, 1], dt, p)
        out[..., t, 0] = q1
        out[..., t, 1] = q2
        out[..., t, 2] = dq1
        out[..., t, 3] = dq2
    return out


class OracleController:
    """Stateful restatement of ``MPPIControllerForPathTracking`` (control.py:20-152)."""

    def __init__(self, delta_t=0.01, ref_path=0, horizon_step_T=20, number_of_samples_K=500,
                 param_exploration=0.0, param_lambda=50.0, param_alpha=1.0,
                 sigma=np.array([[10.0, 10.0], [100.0, 100.0]]),
                 stage_cost_weight=np.array([10.0, 10.0, 10.0, 10.0]),
                 terminal_cost_weight=np.array([10.0, 10.0, 10.0, 10.0]),
                 visualize_optimal_traj=True, visualze_sampled_trajs=False,
                 arm: ArmParams = ArmParams()):
        self.dim_x, self.dim_u = 4, 2
        self.T, self.K = horizon_step_T, number_of_samples_K
        self.param_exploration = param_exploration
        self.param_lambda = param_lambda
        self.param_alpha = param_alpha
        self.param_gamma = param_lambda * (1.0 - param_alpha)
        self.Sigma = sigma
        self.stage_cost_weight = stage_cost_weight
        self.terminal_cost_weight = terminal_cost_weight
        self.visualize_optimal_traj = visualize_optimal_traj
        self.visualze_sampled_trajs = visualze_sampled_trajs
        self.delta_t = delta_t
        self.ref_path = ref_path
        self.arm = arm
        self.u_prev = np.array([[10.0, -2.0] for _ in range(self.T)])
        self.prev_waypoints_idx = 0
        self.last = {}

    def _calc_epsilon(self, sigma, size_sample, size_time_step, size_dim_u):
        """control.py:154-164."""
        if sigma.shape[0] != sigma.shape[1] or sigma.shape[0] != size_dim_u or size_dim_u < 1:
            raise ValueError
        return np.random.multivariate_normal(np.zeros(size_dim_u), sigma, (size_sample, size_time_step))

    def calc_control_input(self, observed_x, epsilon=None):
        u = self.u_prev
        x0 = np.asarray(observed_x, dtype=np.float64)
        idx, *_ = nearest_waypoint(x0[0], x0[1], self.ref_path, self.prev_waypoints_idx, self.arm)
        self.prev_waypoints_idx = int(idx)                              # control.py:75,230
        if self.prev_waypoints_idx >= self.ref_path.shape[0] - 1:      # control.py:76-78
            raise IndexError
        eps = self._calc_epsilon(self.Sigma, self.K, self.T, self.dim_u) if epsilon is None else \
            np.asarray(epsilon, dtype=np.float64)
        S = rollout_costs(x0, u, eps, self.ref_path, self.prev_waypoints_idx, self.delta_t,
                          self.param_lambda, self.param_alpha, self.Sigma,
                          self.stage_cost_weight, self.terminal_cost_weight,
                          self.param_exploration, self.arm, gamma=self.param_gamma)
        w = compute_weights(S, self.param_lambda)
        w_eps_raw = weighted_noise(w, eps)
        w_eps = moving_median_filter(w_eps_raw, 10)
        u_before = u.copy()
        u += w_eps                                                       # control.py:126
        u_new = u.copy()
        optimal_traj = np.zeros((self.T, self.dim_x))
        if self.visualize_optimal_traj:                                  # control.py:129-134
            optimal_traj = rollout_trajectory(x0, np.roll(u, 1, axis=0), self.delta_t, self.arm)
        sampled = np.zeros((self.K, self.T, self.dim_x))
        if self.visualze_sampled_trajs:                                  # control.py:137-145
            K_exp = (np.arange(self.K) < (1.0 - self.param_exploration) * self.K)[:, None, None]
            v = np.where(K_exp, u_before[None] + eps, eps)                # pre-update u
            sampled = rollout_trajectory(x0, np.roll(v, 1, axis=1), self.delta_t, self.arm)
        self.u_prev[:-1] = u[1:]                                         # control.py:148-149
        self.u_prev[-1] = u[-1]
        self.last = dict(S=S, w=w, w_eps_raw=w_eps_raw, w_eps_filt=w_eps, u_new=u_new, eps=eps)
        return u[0], u, optimal_traj, sampled
