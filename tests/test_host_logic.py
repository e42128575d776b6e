"""CPU: the host-side half of the drop-in controller (control.py:67-78, 122-164)
against the golden fixtures and the reference's semantics — everything that
runs before / after the device call, without a GPU."""
import contextlib
import io
import math
import os
import sys

import numpy as np
import pytest

import mppi_oracle as O
from conftest import STEP_FIXTURES, ctor_kwargs, load_step
from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
from mppi_robotarm_amd.distributed import shard_geometry
from mppi_robotarm_amd.engine import exploit_count
from mppi_robotarm_amd.params import SYS_PARAMS, ArmParams, runpy_config

RUNPY = dict(param_exploration=0.0, param_lambda=100.0, param_alpha=0.98, sigma=np.eye(2) * 20.0,
             stage_cost_weight=np.array([0.5, 0.5, 5.0, 5.0]),
             terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]))


def test_constructor_state_matches_reference(paths):
    c = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], **runpy_config())
    assert (c.dim_x, c.dim_u, c.T, c.K) == (4, 2, 30, 100)
    assert c.param_gamma == pytest.approx(100.0 * (1 - 0.98))           # control.py:45
    assert np.array_equal(c.u_prev, np.array([[10.0, -2.0]] * 30))      # control.py:59
    assert c.prev_waypoints_idx == 0 and c.l1 == 1 and c.l2 == 1
    assert c.visualze_sampled_trajs is True and c.visualize_optimal_traj is True
    assert c.ref_path is paths["xydq_circle"]                           # held by reference


def test_sys_params_and_arm():
    assert SYS_PARAMS() == {"Ts": 0.0025, "m1": 1, "m2": 1, "l1": 1, "l2": 1, "lc1": 0.5, "lc2": 0.5, "g": 9.81}
    assert ArmParams.from_sys_params() == ArmParams()


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_nearest_waypoint_update_matches_fixture(name, paths):
    g = load_step(name)
    c = MPPIControllerForPathTracking(ref_path=paths[str(g["path"])], verbose=False, **ctor_kwargs(g))
    c.prev_waypoints_idx = int(g["prev_idx"])
    idx, rx, ry, rdq1, rdq2 = c._get_nearest_waypoint(g["x0"][0], g["x0"][1], update_prev_idx=True)
    assert idx == int(g["prev_idx_after"]) == c.prev_waypoints_idx
    oi, *ref = O.nearest_waypoint(g["x0"][0], g["x0"][1], paths[str(g["path"])], int(g["prev_idx"]), O.ArmParams())
    assert int(oi) == idx and np.allclose(ref, [rx, ry, rdq1, rdq2], rtol=0, atol=0)


def test_progress_prints_like_reference(paths):
    c = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], **runpy_config())
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        c._get_nearest_waypoint(1.152198236517471885, -1.266101672070702344, update_prev_idx=True)
    assert buf.getvalue().splitlines() == ["0     prev_idx = 0", "0     nearest_idx = 0",
                                          "======================updated======================="]


@pytest.mark.parametrize("name", STEP_FIXTURES)
def test_median_filter_and_update_match_fixture(name, paths):
    g = load_step(name)
    c = MPPIControllerForPathTracking(ref_path=paths[str(g["path"])], verbose=False, **ctor_kwargs(g))
    filt = c._moving_median_filter(g["w_eps_raw"], 10)
    assert np.array_equal(filt, g["w_eps_filt"])
    assert np.array_equal(g["u_prev"] + filt, g["u_new"])


@pytest.mark.parametrize("name", ["c1_circle_k128_t20", "sigma_k128_t20", "runpy_k100_t30"])
def test_noise_draw_is_the_reference_stream(name, paths):
    """_calc_epsilon consumes np.random exactly as control.py:163 does."""
    g = load_step(name)
    c = MPPIControllerForPathTracking(ref_path=paths[str(g["path"])], verbose=False, **ctor_kwargs(g))
    np.random.seed(int(g["seed"]))
    eps = c._calc_epsilon(c.Sigma, c.K, c.T, c.dim_u)
    assert np.array_equal(eps.astype(np.float32), g["eps"])


def test_error_paths_before_the_device(paths):
    # end of path (control.py:76-78): IndexError, after the print
    c = MPPIControllerForPathTracking(ref_path=paths["xydq_circle"], verbose=False, **runpy_config())
    c.prev_waypoints_idx = paths["xydq_circle"].shape[0] - 1
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), pytest.raises(IndexError):
        c.calc_control_input(np.array([0.0, 0.0, 0.0, 0.0]))
    assert "[ERROR] Reached the end of the reference path." in buf.getvalue()
    # sigma shape (control.py:157-159): ValueError
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=8,
                                      number_of_samples_K=4, verbose=False, **{**RUNPY, "sigma": np.eye(3)})
    with contextlib.redirect_stdout(io.StringIO()), pytest.raises(ValueError):
        c.calc_control_input(np.array([1.15, -1.27, 0.0, 0.0]))
    # default sigma is singular (control.py:30, :106): LinAlgError after the noise draw
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=8,
                                      number_of_samples_K=4, verbose=False)
    np.random.seed(0)
    import warnings
    with warnings.catch_warnings(), pytest.raises(np.linalg.LinAlgError):
        warnings.simplefilter("ignore")
        c.calc_control_input(np.array([1.15, -1.27, 0.0, 0.0]))


@pytest.mark.parametrize("expl,K", [(0.0, 100), (0.25, 128), (0.37, 1000), (1.0, 64), (0.999, 7), (-0.5, 10),
                                    (0.3, 10), (0.1, 10)])
def test_exploit_count_is_the_reference_split(expl, K):
    """k < (1 - expl) * K evaluated in fp64 exactly as control.py:98."""
    assert exploit_count(expl, K) == sum(1 for k in range(K) if k < (1.0 - expl) * K)


@pytest.mark.parametrize("K,world", [(65536, 8), (100, 3), (7, 7), (524288, 8), (1000, 6)])
def test_shard_geometry_partitions_samples(K, world):
    seen = []
    for r in range(world):
        n, off = shard_geometry(K, world, r)
        seen.extend(range(off, off + n))
    assert seen == list(range(K))
    with pytest.raises(ValueError):
        shard_geometry(2, 3, 0)


def test_exploration_split_is_shard_invariant():
    """The device rule (k_offset + k) < k_exploit reproduces control.py:98 per shard."""
    K, expl, world = 1000, 0.37, 3
    kx = exploit_count(expl, K)
    ref = [k < (1.0 - expl) * K for k in range(K)]
    got = []
    for r in range(world):
        n, off = shard_geometry(K, world, r)
        got.extend((off + k) < kx for k in range(n))
    assert got == ref


def test_oracle_reproduces_exploration_fixture(paths):
    g = load_step("expl_k128_t20")
    K = int(g["K"])
    assert exploit_count(float(g["param_exploration"]), K) == math.ceil(0.75 * K)


def test_harness_plant_matches_reference_loop():
    """utils.py:14-38 plant + run.py:53-59 integration, replayed on the fixture's controls."""
    from conftest import load_loop
    from mppi_robotarm_amd.harness import arm_dynamic, forward_kinematics
    g = load_loop("runpy_k100_t30")
    q = g["states"][0][:2].copy()
    dq = g["states"][0][2:].copy()
    for i in range(int(g["ticks"])):
        dq += 0.003 * arm_dynamic(q, dq, g["u"][i])
        q += 0.003 * dq
        nxt = g["states"][i + 1] if i + 1 < int(g["ticks"]) else g["final_state"]
        assert np.array_equal(np.concatenate([q, dq]), nxt)
    x1, y1, x2, y2 = forward_kinematics(np.array([0.3, -0.4]))
    assert np.allclose([x2, y2], [np.cos(0.3) + np.cos(-0.1), np.sin(0.3) + np.sin(-0.1)])


def test_bench_valu_roofline_from_committed_counters():
    """bench.py's VALU issue roofline from the committed PMC summary against the committed issue-rate
    microbenchmark (profiles/ubench_issue.json, tools/ubench_issue.hip): one wave per SIMD at c3 (priced also
    against the lone-wave rate), two at c5; fractions in (0, 1]."""
    import json
    import os
    import bench
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lone_ns, simd_ns = bench.issue_ceilings()
    assert simd_ns < lone_ns   # more waves per SIMD issue faster than one alone
    for name, kern_ms, wps in (("traffic.json", 0.0293, 1.0), ("traffic_c5.json", 0.250, 2.0)):
        tj = json.load(open(os.path.join(root, "profiles", name)))
        v = bench.valu_roofline(tj, kern_ms)
        assert v["waves_per_simd"] == wps and 0.0 < v["frac"] <= 1.0
        per_simd = tj["valu_insts_per_launch"] / min(tj["waves_per_launch"], bench.SIMDS)
        assert v["frac"] == pytest.approx(per_simd / (kern_ms * 1e6) * simd_ns)
        assert ("frac_one_wave_ceiling" in v) == (wps == 1.0)
        if wps == 1.0:
            assert 0.0 < v["frac_one_wave_ceiling"] <= 1.0
            assert v["frac_one_wave_ceiling"] == pytest.approx(per_simd / (kern_ms * 1e6) * lone_ns)
    assert bench.valu_roofline({}, 0.03) is None


def test_bench_numpy_baseline_runs(paths):
    """bench.py's single-thread NumPy fp64 baseline on a tiny sample."""
    import bench
    eps = (np.random.default_rng(0).standard_normal((64, 4, 2)) * math.sqrt(20.0)).astype(np.float32)
    out = bench.numpy_baseline(eps, paths["xydq_circle"][:30], np.array([1.15, -1.27, 0.0, 0.0]),
                               np.array([[10.0, -2.0]] * 4), 100.0, 0.0)
    assert out["value"] > 0 and out["cores"] == 1 and "K=64 T=4" in out["sample"]


def test_bench_launches_ranks_itself(monkeypatch):
    """`bench.py --gpus N` without WORLD_SIZE starts N ranks itself (the driver's
    N = 1, 2, 4, 8 calls then need no external launcher): a torch.distributed.run
    child on 127.0.0.1 with the same arguments, before any GPU call; ranks own one
    GPU each under nccl (RCCL) when there are enough, else share under gloo."""
    import bench
    cmd = bench.launcher_cmd(4, 29999, ["--gpus", "4", "--steps", "50"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "127.0.0.1" in cmd
    assert "--master-port=29999" in cmd
    assert cmd[-5:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "50"]
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    monkeypatch.setattr(bench, "launch_ranks", lambda a: seen.setdefault("n", a.gpus) and 0)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and seen["n"] == 2
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    assert bench.default_backend(8) == "nccl" and bench.default_backend(2) == "nccl"
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    assert bench.default_backend(2) == "gloo" and bench.default_backend(1) == "nccl"


def test_bench_host_cores_is_the_affinity_mask():
    import bench
    assert bench.host_cores() == len(os.sched_getaffinity(0))


@pytest.mark.parametrize("d", [[3.0, 1.0, 2.0, 1.0], [3.0, np.nan, 1.0, 1.0], [np.nan, 2.0, 1.0],
                               [2.0, np.nan, np.nan], [np.nan, np.nan], [1.0, 1.0, np.nan, 0.5],
                               [np.inf, np.nan, np.inf]])
def test_nearest_waypoint_nan_rule_is_python_min(d):
    """control.py:212-215 builds a list and takes d.index(min(d)): min() keeps d[0]
    and replaces it only on a strict '<', so a NaN at j > 0 is never chosen and a
    NaN at j = 0 always is — unlike np.argmin (first NaN).  Host drop-in, NumPy
    oracle (vectorised) and the chain oracle all follow it."""
    import chain_oracle as CO
    from mppi_robotarm_amd.controller import first_min_index
    lst = [np.float64(v) for v in d]
    want = lst.index(min(lst))
    arr = np.array(d)
    assert first_min_index(arr) == want
    assert int(O.first_min_index(arr)) == want
    assert O.first_min_index(np.stack([arr, arr[::-1]])).tolist() == [want, [*lst[::-1]].index(min(lst[::-1]))]
    path = np.zeros((len(d), 4))
    path[:len(d), 0] = np.sqrt(np.where(np.isnan(arr), np.nan, arr) / 100.0)   # (x - rx)^2 * 100 == d at x = 0
    idx = CO.nearest_waypoint_xy(0.0, 0.0, path, 0)[0]
    assert int(idx) == want


def test_host_nearest_waypoint_skips_nan_rows(paths):
    """The drop-in's host update (control.py:200-232) on a ref_path with NaN rows."""
    path = paths["xydq_circle"].copy()
    c = MPPIControllerForPathTracking(ref_path=path, verbose=False)
    x0 = np.array([1.152198236517471885, -1.266101672070702344, 0.0, 0.0])
    want = c._get_nearest_waypoint(x0[0], x0[1])[0]
    path[want + 1] = np.nan                     # a NaN after the nearest row: never chosen
    assert c._get_nearest_waypoint(x0[0], x0[1])[0] == want
    path[0] = np.nan                            # a NaN in row 0 of the window: chosen
    assert c._get_nearest_waypoint(x0[0], x0[1])[0] == 0


def test_sampled_readback_buffers_are_never_shared_with_a_live_array():
    """sampled_traj_list comes from a pool of read-back buffers (widened on the host from a chunked fp32 DMA on the GPU); a buffer is reused only
    once the caller holds neither its array nor any view of it, so each returned array behaves as the fresh
    np.zeros of control.py:137 (CPU tensors here: the pool logic, torch widening)."""
    import torch
    from mppi_robotarm_amd.controller import SampledReadback
    rb = SampledReadback()
    tr = [torch.full((6, 5, 4), float(i) + 0.25, dtype=torch.float32) for i in range(8)]
    a1 = rb(tr[1])
    assert a1.dtype == np.float64 and a1.shape == (6, 5, 4) and a1.flags.writeable and np.all(a1 == 1.25)
    a2 = rb(tr[2])
    assert not np.shares_memory(a1, a2) and np.all(a1 == 1.25)
    p1 = a1.__array_interface__["data"][0]
    del a1
    a3 = rb(tr[3])                                 # a1's buffer is free again
    assert a3.__array_interface__["data"][0] == p1 and np.all(a3 == 3.25) and np.all(a2 == 2.25)
    v = a2[2:, 1]                                  # a view keeps a2's buffer out of reuse
    del a2
    a4 = rb(tr[4])
    assert np.all(v == 2.25) and not np.shares_memory(a4, v) and not np.shares_memory(a4, a3)
    a5 = rb(tr[5])                                 # pool full (3 held): a plain read-back
    assert np.all(a5 == 5.25) and len(rb) == 3
    assert not any(np.shares_memory(a5, x) for x in (a3, a4, v))
    a5[:] = -1.0                                   # writable, and nobody else's
    assert np.all(a3 == 3.25) and np.all(a4 == 4.25) and np.all(v == 2.25)
    a6 = rb(torch.zeros((3, 5, 4)))                # K changed: new buffers, held arrays intact
    assert a6.shape == (3, 5, 4) and np.all(a3 == 3.25) and np.all(v == 2.25)


# the chain's fused update (mppi_chain.hip chain_update_block): four consecutive windows of scipy's median of 10
# from one sorted 7-value core; restated here against scipy.ndimage.median_filter (control.py:319-327)
_SORT7 = [(0, 6), (2, 3), (4, 5), (0, 2), (1, 4), (3, 6), (0, 1), (2, 5), (3, 4), (1, 2), (4, 6), (2, 3), (4, 5),
          (1, 2), (3, 4), (5, 6)]


def _sliding_median10(col):
    T = len(col)
    out = np.empty(T)
    for t0 in range(0, T, 4):
        idx = np.arange(t0 - 5, t0 + 8)
        idx = np.where(idx < 0, -idx - 1, idx)
        idx = np.where(idx >= T, 2 * T - 1 - idx, idx)
        e = col[np.clip(idx, 0, T - 1)]
        A = list(e[3:10])
        for i, j in _SORT7:
            A[i], A[j] = min(A[i], A[j]), max(A[i], A[j])
        for j in range(4):
            if t0 + j < T:
                B = sorted(e[[k if k < 3 else k + 7 for k in range(j, j + 3)]])
                out[t0 + j] = min(A[5], max(A[4], B[0]), max(A[3], B[1]), max(A[2], B[2]))
    return out


@pytest.mark.parametrize("T", [5, 6, 7, 9, 32, 127, 128])
def test_chain_sliding_median_equals_scipy(T):
    from scipy.ndimage import median_filter
    rng = np.random.default_rng(T)
    for x in (rng.standard_normal((T, 7)), rng.integers(-3, 4, (T, 7)).astype(float)):   # ties included
        ref = median_filter(x, size=(10, 1), mode="reflect")
        got = np.stack([_sliding_median10(x[:, d]) for d in range(7)], axis=1)
        assert np.array_equal(got, ref)


# the rank-5 selection network measured for median10 (the full 10-sort minus 5 comparators)
_SEL10 = [(4, 9), (3, 8), (2, 7), (1, 6), (0, 5), (1, 4), (6, 9), (0, 3), (5, 8), (0, 2), (3, 6), (2, 4), (5, 7), (8, 9),
          (1, 2), (4, 6), (7, 8), (3, 5), (2, 5), (6, 8), (4, 7), (6, 7), (5, 6), (4, 5)]


def test_median10_selection_network_is_rank5():
    import itertools
    for bits in itertools.product([0, 1], repeat=10):   # 0-1 principle
        v = list(bits)
        for i, j in _SEL10:
            v[i], v[j] = min(v[i], v[j]), max(v[i], v[j])
        assert v[5] == sorted(bits)[5]
