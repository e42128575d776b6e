"""CPU: pin the oracles (NumPy fp64 + C fp64) to the golden fixtures captured
from the imported reference (tests/golden/make_golden.py)."""
import json
import math
import os

import numpy as np
import pytest

import coracle
import mppi_oracle as O
from conftest import GOLDEN, LOOP_FIXTURES, STEP_FIXTURES, ctor_kwargs, load_loop, load_step

RUNPY = dict(param_exploration=0.0, param_lambda=100.0, param_alpha=0.98, sigma=np.eye(2) * 20.0,
             stage_cost_weight=np.array([0.5, 0.5, 5.0, 5.0]),
             terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]))


def _run_oracle(g, paths):
    c = O.OracleController(ref_path=paths[str(g["path"])], **ctor_kwargs(g))
    c.prev_waypoints_idx = int(g["prev_idx"])
    c.u_prev = g["u_prev"].copy()
    u_prev = c.u_prev
    out = c.calc_control_input(g["x0"], epsilon=g["eps"].astype(np.float64))
    return c, u_prev, out


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_numpy_oracle_matches_reference(name, paths):
    g = load_step(name)
    c, u_prev, (u0, u_seq, opt, samp) = _run_oracle(g, paths)
    L = c.last
    assert np.max(np.abs(L["S"] - g["S"]) / np.abs(g["S"])) < 1e-14
    assert int(np.argmin(L["S"])) == int(np.argmin(g["S"]))
    np.testing.assert_allclose(L["w"], g["w"], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(L["w_eps_raw"], g["w_eps_raw"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(L["w_eps_filt"], g["w_eps_filt"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(L["u_new"], g["u_new"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(u_seq, g["u_seq"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(u0, g["u0"], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(opt, g["optimal_traj"], rtol=1e-13, atol=1e-14)
    if "sampled_traj" in g:
        np.testing.assert_allclose(samp, g["sampled_traj"], rtol=1e-12, atol=1e-14)
    assert c.prev_waypoints_idx == int(g["prev_idx_after"])
    # aliasing semantics of the return (control.py:70,126,148-152)
    assert u_seq is u_prev and np.shares_memory(u0, u_prev)
    if float(np.sum(g["w"] ** 2)) > 0.999999:  # one-hot weights: bit-exact update
        assert np.array_equal(L["u_new"], g["u_new"])


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_c_oracle_matches_reference(name, paths):
    g = load_step(name)
    ref = paths[str(g["path"])]
    prev = int(g["prev_idx_after"])
    K = int(g["K"])
    S = coracle.rollout_costs(g["x0"], g["u_prev"], g["eps"], ref[prev:prev + 30], float(g["delta_t"]),
                              float(g["param_lambda"]), float(g["param_alpha"]), g["sigma"],
                              g["stage_cost_weight"], g["terminal_cost_weight"], O.ArmParams(),
                              k_exploit=math.ceil((1 - float(g["param_exploration"])) * K))
    assert np.max(np.abs(S - g["S"]) / np.abs(g["S"])) < 1e-13
    w, w_eps = coracle.weighted_noise(S, g["eps"], float(g["param_lambda"]))
    np.testing.assert_allclose(w_eps, g["w_eps_raw"], rtol=1e-9, atol=1e-12)
    # device layout [T][K][2] reads the same numbers
    S2 = coracle.rollout_costs(g["x0"], g["u_prev"], np.ascontiguousarray(g["eps"].transpose(1, 0, 2)),
                               ref[prev:prev + 30], float(g["delta_t"]), float(g["param_lambda"]),
                               float(g["param_alpha"]), g["sigma"], g["stage_cost_weight"],
                               g["terminal_cost_weight"], O.ArmParams(),
                               k_exploit=math.ceil((1 - float(g["param_exploration"])) * K), layout="TK")
    assert np.array_equal(S, S2)


@pytest.mark.parametrize("name", LOOP_FIXTURES)
def test_closed_loop_oracle(name, paths):
    """run.py:48-71 tick by tick (plant utils.py:14-38) on the fixture's noise."""
    g = load_loop(name)
    T, K = int(g["T"]), int(g["K"])
    c = O.OracleController(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=T,
                           number_of_samples_K=K, visualize_optimal_traj=False, **RUNPY)
    q = g["states"][0][:2].copy()
    dq = g["states"][0][2:].copy()
    state = np.concatenate([q, dq])
    for i in range(int(g["ticks"])):
        np.testing.assert_allclose(state, g["states"][i], rtol=1e-9, atol=1e-11)
        u, u_seq, _, _ = c.calc_control_input(state, epsilon=g["eps"][i].astype(np.float64))
        np.testing.assert_allclose(u, g["u"][i], rtol=1e-9, atol=1e-9)  # fp64 drift through the plant
        assert c.prev_waypoints_idx == int(g["prev_idx"][i])
        dq = dq + 0.003 * O.arm_dynamic(q, dq, u)
        q = q + 0.003 * dq
        state = np.concatenate([q, dq])
    np.testing.assert_allclose(state, g["final_state"], rtol=1e-9, atol=1e-11)


def test_median_filter_known_answers():
    m = np.load(os.path.join(GOLDEN, "medfilt.npz"))
    for n in (1, 2, 3, 5, 9, 10, 11, 20, 30, 64):
        assert np.array_equal(O.median_filter_reflect(m[f"x{n}"]), m[f"y{n}"]), n


def test_error_classes_match_reference(paths):
    errs = json.load(open(os.path.join(GOLDEN, "errors.json")))
    assert errs == {"end_of_path": "IndexError", "default_sigma": "numpy.linalg.LinAlgError",
                    "sigma_shape": "ValueError"}
    c = O.OracleController(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=8,
                           number_of_samples_K=4, **RUNPY)
    c.prev_waypoints_idx = paths["xydq_circle"].shape[0] - 1
    with pytest.raises(IndexError):
        c.calc_control_input(np.zeros(4))
    c = O.OracleController(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=8,
                           number_of_samples_K=4)
    with pytest.raises(np.linalg.LinAlgError):
        c.calc_control_input(O.np.array([1.15, -1.27, 0.0, 0.0]), epsilon=np.zeros((4, 8, 2)))
