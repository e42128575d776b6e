"""CPU: the n-link chain oracle (BASELINE config 5).

The 7-DoF model is build-defined (the reference has none), so its parity is
unpinned by the reference at n = 7.  These tests pin what can be pinned:
at n = 2 with the reference constants and inertia := length
(control.py:241-245) the chain IS the reference model — dynamics, the whole
K x T cost, and the full controller update — checked against the 2-DoF oracle
and the reference's own golden steps; and the two chain restatements (NumPy,
C) agree at n = 7.
"""
import numpy as np
import pytest

import chain_oracle as CO
import coracle
import mppi_oracle as O
from conftest import STEP_FIXTURES, load_step

P7 = CO.ChainParams()
P2 = CO.ChainParams.from_arm2()


def test_chain_dynamics_reduce_to_reference_F_at_n2():
    rng = np.random.default_rng(0)
    q, dq, v = rng.normal(0, 1, (500, 2)), rng.normal(0, 2, (500, 2)), rng.normal(0, 20, (500, 2))
    ref = np.stack(O.forward_dynamics(q[:, 0], q[:, 1], dq[:, 0], dq[:, 1], v[:, 0], v[:, 1], 0.006, O.ArmParams()), 1)
    qn, dqn = CO.chain_forward_dynamics(q, dq, v, 0.006, P2)
    np.testing.assert_allclose(np.concatenate([qn, dqn], 1), ref, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_chain_step_at_n2_matches_reference_golden(name, paths):
    """S and the updated control of the reference's golden steps, through the chain model."""
    g = load_step(name)
    ref_path = paths[str(g["path"])]
    c = CO.ChainOracleController(float(g["delta_t"]), ref_path, int(g["T"]), int(g["K"]),
                                 float(g["param_exploration"]), float(g["param_lambda"]), float(g["param_alpha"]),
                                 g["sigma"], g["stage_cost_weight"], g["terminal_cost_weight"], chain=P2,
                                 visualize_optimal_traj=False)
    c.u_prev = g["u_prev"].copy()
    c.prev_waypoints_idx = int(g["prev_idx"])
    _, u_seq, _, _ = c.calc_control_input(g["x0"], epsilon=g["eps"].astype(np.float64))
    S = c.last["S"]
    assert int(np.argmin(S)) == int(np.argmin(g["S"]))
    assert float(np.max(np.abs(S - g["S"]) / np.abs(g["S"]))) < 1e-13
    assert float(np.max(np.abs(u_seq - g["u_seq"]))) < 1e-10 * max(1.0, float(np.max(np.abs(g["u_seq"]))))
    assert c.prev_waypoints_idx == int(g["prev_idx_after"])


def _c5_inputs(K, T, seed=3):
    rng = np.random.default_rng(seed)
    x0 = np.concatenate([[1.481492] + [-0.320757] * 6, [0.0] * 7])
    u = np.tile(CO.gravity_torque(x0[:7], P7), (T, 1)) + rng.normal(0, 0.5, (T, 7))
    sig = np.diag([20.0, 16.0, 12.0, 8.0, 4.0, 2.0, 1.0])
    eps = (rng.normal(0, 1, (K, T, 7)) * np.sqrt(np.diag(sig))).astype(np.float32)
    return x0, u, sig, eps


def test_c_chain_oracle_matches_numpy_at_n7(paths):
    K, T = 96, 24
    x0, u, sig, eps = _c5_inputs(K, T)
    win = paths["xydq_circle"][:30]
    S = CO.chain_rollout_costs(x0, u, eps.astype(np.float64), paths["xydq_circle"], 0, 0.006, 100.0, 0.98, sig,
                               [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.25, P7)
    Sc = coracle.chain_rollout_costs(x0, u, eps, win, 0.006, 100.0, 0.98, sig, [0.5, 0.5, 5, 5], [5, 5, 50, 50], P7,
                                     k_exploit=int(np.ceil(0.75 * K)))
    np.testing.assert_allclose(Sc, S, rtol=1e-11)
    Sd = coracle.chain_rollout_costs(x0, u, np.ascontiguousarray(eps.transpose(1, 2, 0)), win, 0.006, 100.0, 0.98,
                                     sig, [0.5, 0.5, 5, 5], [5, 5, 50, 50], P7, k_exploit=int(np.ceil(0.75 * K)),
                                     layout="TNK")
    assert np.array_equal(Sc, Sd)                      # device [T][n][K] layout reads the same values
    w, we = coracle.chain_weighted_noise(Sc, eps, 1.0e7)
    np.testing.assert_allclose(we, O.weighted_noise(O.compute_weights(Sc, 1.0e7), eps), rtol=1e-12, atol=1e-15)
    traj = coracle.chain_traj(x0, np.repeat(u[None], 3, 0), 0.006, P7)
    np.testing.assert_allclose(traj[0], CO.chain_rollout_trajectory(x0, u, 0.006, P7), rtol=1e-12, atol=1e-12)


def test_gravity_torque_holds_the_chain():
    q = np.array([1.481492] + [-0.320757] * 6)
    qn, dqn = CO.chain_forward_dynamics(q[None], np.zeros((1, 7)), CO.gravity_torque(q, P7)[None], 0.006, P7)
    assert np.max(np.abs(dqn)) < 1e-12 and np.max(np.abs(qn - q)) < 1e-14


def test_c5_start_pose_is_on_the_path(paths):
    x, y = CO.chain_fk(np.array([1.481492] + [-0.320757] * 6), P7)
    assert np.hypot(x - paths["xydq_circle"][0, 0], y - paths["xydq_circle"][0, 1]) < 1e-5


def test_theta_space_dynamics_equal_the_joint_space_equations():
    """D' (with the armature) and tau (with the damping) in absolute angles give the
    accelerations of M q_ddot = u - b dq - S^T (c + g), M = S^T D S + diag(J)."""
    rng = np.random.default_rng(2)
    q, dq, v = rng.normal(0, 1, 7), rng.normal(0, 2, 7), rng.normal(0, 5, 7)
    mu, nu, _ = CO.coefficients(CO.ChainParams(J=(0.0,) * 7, b=(0.0,) * 7))
    th, thd = np.cumsum(q), np.cumsum(dq)
    D = mu * np.cos(th[:, None] - th[None, :])
    np.fill_diagonal(D, np.diag(mu) + np.asarray(P7.I))
    S = np.tril(np.ones((7, 7)))
    M = S.T @ D @ S + np.diag(P7.J)
    rhs = v - np.asarray(P7.b) * dq - S.T @ ((mu * np.sin(th[:, None] - th[None, :])) @ thd ** 2 + P7.g * nu * np.cos(th))
    qn, dqn = CO.chain_forward_dynamics(q[None], dq[None], v[None], 0.006, P7)
    np.testing.assert_allclose((dqn[0] - dq) / 0.006, np.linalg.solve(M, rhs), rtol=1e-10, atol=1e-10)


def test_tie_flip_helper_explains_a_neighbour_pick(paths):
    """tests/tieflip.py: a cost equal to the fp64 one with the neighbour slot taken
    at the closest-tie step is explained (residual ~0, that step's gap reported)."""
    from tieflip import tie_flip_residual, tie_table
    rng = np.random.default_rng(3)
    K, T = 64, 8
    win = paths["xydq_circle"][:30]
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, gravity_torque
    x0 = CHAIN7_X0
    u = np.tile(gravity_torque(x0[:7]), (T, 1))
    eps = (rng.standard_normal((T, 7, K)) * np.sqrt(np.diag(CHAIN7_SIGMA))[None, :, None]).astype(np.float32)
    W, TW = [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0]
    Sr = coracle.chain_rollout_costs(x0, u, eps, win, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, P7, layout="TNK")
    idx = np.array([3, 17, 40])
    gap, delta = tie_table(idx, x0, u, eps, win, 0.006, W, TW, P7)
    S_dev = Sr.copy()
    t1 = int(np.argmin(gap[0]))
    S_dev[3] += delta[0, t1]                       # sample 3: the neighbour at its closest tie
    res, used = tie_flip_residual(S_dev, Sr, idx, x0, u, eps, win, 0.006, W, TW, P7)
    assert res[0] < 1e-12 and used[0] == gap[0, t1]
    assert res[1] < 1e-12 and used[1] == 0.0       # unflipped samples need no flip
    assert np.all(gap >= 0)


def test_device_pick_helper_recomputes_with_given_slots(paths):
    """tests/tieflip.py device_pick_residual: with the fp64 argmin everywhere it returns S_ref itself
    (residual 0, no differing pick); with the second-nearest slot forced at one step, S_ref plus
    exactly that step's cost step (tie_table's delta), that step's gap and one differing pick."""
    from tieflip import device_pick_residual, tie_table
    rng = np.random.default_rng(4)
    K, T = 32, 6
    win = paths["xydq_circle"][:30]
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, gravity_torque
    x0 = CHAIN7_X0
    u = np.tile(gravity_torque(x0[:7]), (T, 1))
    eps = (rng.standard_normal((T, 7, K)) * np.sqrt(np.diag(CHAIN7_SIGMA))[None, :, None]).astype(np.float32)
    W, TW = [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0]
    Sr = coracle.chain_rollout_costs(x0, u, eps, win, 0.006, 100.0, 0.98, CHAIN7_SIGMA, W, TW, P7, layout="TNK")
    idx = np.arange(K)
    # the fp64 picks (first minimum) from the oracle's own walk
    slots = np.zeros((K, T), dtype=np.int32)
    from tieflip import _walk
    second = np.zeros((K, T), dtype=np.int32)
    for t, x, y, dq in _walk(idx, x0, u, eps, 0.006, P7, None):
        d = (x[:, None] - win[:, 0]) ** 2 + (y[:, None] - win[:, 1]) ** 2
        o = np.argsort(d, axis=1, kind="stable")
        slots[:, t], second[:, t] = o[:, 0], o[:, 1]
    res, gap, nd = device_pick_residual(Sr, Sr, idx, x0, u, eps, win, 0.006, W, TW, P7, slots)
    assert np.all(res < 1e-13) and np.all(gap == 0) and np.all(nd == 0)
    gap2, delta = tie_table([5], x0, u, eps, win, 0.006, W, TW, P7)
    forced = slots.copy()
    forced[5, 2] = second[5, 2]
    S_dev = Sr.copy()
    S_dev[5] += delta[0, 2]
    res, gap, nd = device_pick_residual(S_dev, Sr, idx, x0, u, eps, win, 0.006, W, TW, P7, forced)
    assert res[5] < 1e-12 and nd[5] == 1 and abs(gap[5] - gap2[0, 2]) < 1e-15
    assert np.all(np.delete(nd, 5) == 0)
