"""GPU: the multi-GPU drop-in — MPPIControllerForPathTracking / ChainMPPIController
constructed with ``process_group`` — rehearsed with 2 ranks on ONE GPU (gloo
carries the one-time setup collectives; on a node the in-launch exchange's
stores cross xGMI, the pool's boxes have one GPU).

Every rank builds the controller with the same arguments and feeds it the same
``observed_x`` (run.py's loop replicated, run.py:49); with NumPy noise every rank
seeds ``np.random`` identically, draws the reference's full (K, T, 2) stream and
keeps its slice (control.py:91-118 over a shard of the samples).  Checked:

  * the reference fixtures: ``step_runpy_k100_t30`` (run.py's config with
    sampled trajectories on, so the sharded re-roll is gathered across ranks,
    control.py:137-145) reached through ``np.random.seed`` + the reference RNG
    stream, and the ``loop_k64_t20`` ticks — at U_TOL (BASELINE.json's 1e-4);
  * the single-process controller on the same inputs — at 1e-10 (the shards'
    rows are merged in another order; nothing else differs);
  * both exchanges: "auto" (must pick the in-launch one: one launch per rank
    per step, and with device noise the one-call native tick) and "rccl"
    (rollout + all-gather + merge launch);
  * the chain controller at n = 2 against the reference's step fixture.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from conftest import ctor_kwargs, load_loop, load_paths, load_step  # noqa: E402

U_TOL = 1e-4
X_TOL = 1e-10
RUNPY = dict(param_exploration=0.0, param_lambda=100.0, param_alpha=0.98, sigma=np.eye(2) * 20.0,
             stage_cost_weight=np.array([0.5, 0.5, 5.0, 5.0]),
             terminal_cost_weight=np.array([5.0, 5.0, 50.0, 50.0]))
DEV_K, DEV_T, DEV_TICKS, DEV_SEED = 8192, 32, 6, 3


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _urel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


# ---------------------------------------------------------------- scenarios
# Each runs identically in a rank (pg = the process group) and in the parent (pg = None).

def _step_runpy(pg, exchange):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g, paths = load_step("runpy_k100_t30"), load_paths()
    c = MPPIControllerForPathTracking(ref_path=paths[str(g["path"])], verbose=False, process_group=pg,
                                      exchange=exchange, **ctor_kwargs(g))
    c.prev_waypoints_idx = int(g["prev_idx"])
    c.u_prev = g["u_prev"].copy()
    u_prev = c.u_prev
    np.random.seed(int(g["seed"]))
    u0, u_seq, opt, samp = c.calc_control_input(g["x0"])
    alias = bool(u_seq is u_prev and np.shares_memory(u0, u_prev))
    out = dict(u_seq=u_seq.copy(), u0=np.array(u0), opt=opt, samp=samp, prev=c.prev_waypoints_idx, alias=alias,
               xmode=str(c._xmode))
    c.close()
    return out


def _loop(pg, exchange):
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g, paths = load_loop("k64_t20"), load_paths()
    T, K = int(g["T"]), int(g["K"])
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=T,
                                      number_of_samples_K=K, verbose=False, visualize_optimal_traj=False,
                                      process_group=pg, exchange=exchange, **RUNPY)
    u_prev, prev, useq, idx = np.array([[10.0, -2.0]] * T), 0, [], []
    for i in range(int(g["ticks"])):
        c.u_prev = u_prev.copy()
        c.prev_waypoints_idx = prev
        eps = g["eps"][i].astype(np.float64)
        c._calc_epsilon = lambda *a, e=eps, **k: e
        _, u_seq, _, _ = c.calc_control_input(g["states"][i])
        useq.append(u_seq.copy())
        idx.append(c.prev_waypoints_idx)
        u_prev, prev = g["u_seq"][i].copy(), int(g["prev_idx"][i])
    out = dict(u_seq=np.array(useq), prev=np.array(idx), xmode=str(c._xmode))
    c.close()
    return out


def _device_ticks(pg, exchange):
    """Device Philox noise, closed loop on the loop fixture's recorded states: after
    the first (general-path) call the tick is the bound one-call native step."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g, paths = load_loop("k64_t20"), load_paths()
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=DEV_T,
                                      number_of_samples_K=DEV_K, verbose=False, noise="device", seed=DEV_SEED,
                                      process_group=pg, exchange=exchange, **RUNPY)
    useq, u0s, opts, idx = [], [], [], []
    for i in range(DEV_TICKS):
        u0, u_seq, opt, samp = c.calc_control_input(g["states"][i])
        assert u_seq is c.u_prev and samp.shape == (DEV_K, DEV_T, 4) and samp.flags.writeable
        useq.append(u_seq.copy())
        u0s.append(np.array(u0))
        opts.append(opt.copy())
        idx.append(c.prev_waypoints_idx)
    out = dict(u_seq=np.array(useq), u0=np.array(u0s), opt=np.array(opts), prev=np.array(idx),
               xmode=str(c._xmode), bound=c._bound is not None)
    c.close()
    return out


def _chain_step(pg, exchange, sampled=True):
    from mppi_robotarm_amd.chain import ChainMPPIController, ChainParams
    g, paths = load_step("runpy_k100_t30"), load_paths()
    c = ChainMPPIController(float(g["delta_t"]), paths[str(g["path"])], int(g["T"]), int(g["K"]),
                            float(g["param_exploration"]), float(g["param_lambda"]), float(g["param_alpha"]),
                            g["sigma"], g["stage_cost_weight"], g["terminal_cost_weight"],
                            visualze_sampled_trajs=sampled, chain=ChainParams.from_arm2(), u_init=g["u_prev"],
                            process_group=pg, exchange=exchange)
    c.prev_waypoints_idx = int(g["prev_idx"])
    np.random.seed(int(g["seed"]))
    u0, u_seq, opt, samp = c.calc_control_input(g["x0"])
    out = dict(u_seq=u_seq.copy(), opt=opt, samp=samp, prev=c.prev_waypoints_idx, xmode=str(c._xmode))
    c.close()
    return out


LATE_TIMEOUT_US = "30000"   # MPPI_EXCHANGE_TIMEOUT_US of the late-rank scenarios: a 30 ms poll bound
LATE_TICK, LATE_SLEEP_S = 2, 0.5


def _late_rank_ticks(pg, exchange):
    """Failure semantics of the in-launch exchange: rank 1 starts its tick LATE_TICK LATE_SLEEP_S late, far
    past the poll bound.  Every rank must see the step fail (ExchangeError inside the call, no update applied
    anywhere), run it again over the all-gather and return the single-process result; the later ticks run
    over the all-gather and match too (the state left by the failed launch is consistent)."""
    import time
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g, paths = load_loop("k64_t20"), load_paths()
    rank = pg.rank() if pg is not None else 0
    os.environ["MPPI_EXCHANGE_TIMEOUT_US"] = LATE_TIMEOUT_US
    try:
        c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=DEV_T,
                                          number_of_samples_K=DEV_K, verbose=False, noise="device", seed=DEV_SEED,
                                          process_group=pg, exchange=exchange, **RUNPY)
        useq, idx, modes = [], [], []
        for i in range(DEV_TICKS):
            if i == LATE_TICK and rank == 1:
                time.sleep(LATE_SLEEP_S)
            _, u_seq, _, _ = c.calc_control_input(g["states"][i])
            useq.append(u_seq.copy())
            idx.append(c.prev_waypoints_idx)
            modes.append(str(c._xmode))
        out = dict(u_seq=np.array(useq), prev=np.array(idx), modes=np.array(modes), xmode=str(c._xmode))
        c.close()
    finally:
        del os.environ["MPPI_EXCHANGE_TIMEOUT_US"]
    return out


def _late_rank_chain(pg, exchange):
    """The same for the chain controller's fused step (n = 2, the reference's step fixture, device noise)."""
    import time
    from mppi_robotarm_amd.chain import ChainMPPIController, ChainParams
    g, paths = load_step("runpy_k100_t30"), load_paths()
    rank = pg.rank() if pg is not None else 0
    os.environ["MPPI_EXCHANGE_TIMEOUT_US"] = LATE_TIMEOUT_US
    try:
        c = ChainMPPIController(float(g["delta_t"]), paths[str(g["path"])], int(g["T"]), 4096,
                                float(g["param_exploration"]), float(g["param_lambda"]), float(g["param_alpha"]),
                                g["sigma"], g["stage_cost_weight"], g["terminal_cost_weight"],
                                chain=ChainParams.from_arm2(), u_init=g["u_prev"], noise="device", seed=5,
                                process_group=pg, exchange=exchange)
        useq, modes = [], []
        for i in range(4):
            c.prev_waypoints_idx = int(g["prev_idx"])
            if i == LATE_TICK and rank == 1:
                time.sleep(LATE_SLEEP_S)
            _, u_seq, _, _ = c.calc_control_input(g["x0"])
            useq.append(u_seq.copy())
            modes.append(str(c._xmode))
        out = dict(u_seq=np.array(useq), modes=np.array(modes), xmode=str(c._xmode))
        c.close()
    finally:
        del os.environ["MPPI_EXCHANGE_TIMEOUT_US"]
    return out


def _mixed_draw(pg, exchange):
    """The drop-in's default NumPy noise with rank 1 on the host draw (numpy_noise_on_device=False) and rank 0
    on the device draw: the ranks' first-step check compares the RNG state each draw leaves (the same for both),
    so they agree and take the in-launch exchange; the steps equal the single-process controller's."""
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    g, paths = load_loop("k64_t20"), load_paths()
    rank = pg.rank() if pg is not None else 0
    c = MPPIControllerForPathTracking(delta_t=0.006, ref_path=paths["xydq_circle"], horizon_step_T=DEV_T,
                                      number_of_samples_K=DEV_K, verbose=False, process_group=pg, exchange=exchange,
                                      numpy_noise_on_device=rank == 0, **RUNPY)
    np.random.seed(17)
    useq = []
    for i in range(3):
        _, u_seq, _, _ = c.calc_control_input(g["states"][i])
        useq.append(u_seq.copy())
    out = dict(u_seq=np.array(useq), rng=np.random.get_state()[1][:8].astype(np.int64), xmode=str(c._xmode),
               rankonly_devdraw=bool(c._npdev))
    c.close()
    return out


SCENARIOS = {
    "step_auto": (_step_runpy, "auto"), "step_rccl": (_step_runpy, "rccl"),
    "loop_auto": (_loop, "auto"),
    "dev_auto": (_device_ticks, "auto"), "dev_rccl": (_device_ticks, "rccl"),
    "chain_auto": (_chain_step, "auto"), "chain_rccl": (_chain_step, "rccl"),
    # no sampled re-roll: the chain's fused step (update in the launch, after the in-launch exchange)
    "chainfused_auto": (lambda pg, ex: _chain_step(pg, ex, sampled=False), "auto"),
    "late_auto": (_late_rank_ticks, "auto"),
    "latechain_auto": (_late_rank_chain, "auto"),
    "mixdraw_auto": (_mixed_draw, "auto"),
}


def _rank(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        res = {}
        for name, (fn, ex) in SCENARIOS.items():
            for k, v in fn(dist.group.WORLD, ex).items():
                res[f"{name}.{k}"] = np.asarray(v)
        np.savez(f"{out}.{rank}.npz", **res)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    import torch.multiprocessing as mp
    out = str(tmp_path_factory.mktemp("mgpu") / "r")
    mp.start_processes(_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    return [dict(np.load(f"{out}.{r}.npz")) for r in range(2)]


@pytest.fixture(scope="module")
def single():
    return {name: fn(None, "auto") for name, (fn, _) in SCENARIOS.items()}


def _get(res, name):
    p = name + "."
    return {k[len(p):]: v for k, v in res.items() if k.startswith(p)}


@pytest.mark.parametrize("name", list(SCENARIOS))
def test_ranks_agree_and_match_single_process(ranks, single, name):
    r0, r1, s = _get(ranks[0], name), _get(ranks[1], name), single[name]
    for k in r0:
        if not k.startswith("rankonly_"):
            np.testing.assert_array_equal(r0[k], r1[k], err_msg=f"{name}.{k}: ranks differ")
    want = "rccl" if name.endswith("rccl") or name.startswith("late") else "launch"
    assert str(r0["xmode"]) == want, "exchange='auto' must pick the in-launch exchange when its check passes"
    for k, v in s.items():
        if k in ("xmode", "bound", "modes") or k.startswith("rankonly_"):
            continue
        if np.asarray(v).dtype.kind == "f":
            np.testing.assert_allclose(r0[k], v, rtol=X_TOL, atol=X_TOL, err_msg=f"{name}.{k}")
        else:
            np.testing.assert_array_equal(r0[k], v, err_msg=f"{name}.{k}")


@pytest.mark.parametrize("mode", ["auto", "rccl"])
def test_sharded_step_matches_reference_fixture(ranks, mode):
    """run.py's config, np.random.seed + the reference RNG stream, sampled trajectories gathered."""
    g = load_step("runpy_k100_t30")
    r = _get(ranks[0], f"step_{mode}")
    assert _urel(r["u_seq"], g["u_seq"]) < U_TOL
    assert _urel(r["u0"], g["u0"]) < U_TOL
    assert bool(r["alias"])                                              # control.py:70,148-152
    assert int(r["prev"]) == int(g["prev_idx_after"])
    np.testing.assert_allclose(r["opt"], g["optimal_traj"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(r["samp"], g["sampled_traj"], rtol=1e-4, atol=1e-4)


def test_sharded_loop_matches_reference_fixture(ranks):
    g = load_loop("k64_t20")
    r = _get(ranks[0], "loop_auto")
    for i in range(int(g["ticks"])):
        assert _urel(r["u_seq"][i], g["u_seq"][i]) < U_TOL, i
    np.testing.assert_array_equal(r["prev"], g["prev_idx"])


def test_device_noise_ticks_take_the_one_call_native_tick(ranks):
    r = _get(ranks[0], "dev_auto")
    assert bool(r["bound"]), "the multi-GPU drop-in did not reach mppi_dropin_tick"


@pytest.mark.parametrize("mode", ["auto", "rccl", "fused"])
def test_sharded_chain_n2_matches_reference_fixture(ranks, mode):
    g = load_step("runpy_k100_t30")
    r = _get(ranks[0], "chainfused_auto" if mode == "fused" else f"chain_{mode}")
    assert _urel(r["u_seq"], g["u_seq"]) < U_TOL
    assert int(r["prev"]) == int(g["prev_idx_after"])
    np.testing.assert_allclose(r["opt"], g["optimal_traj"], rtol=1e-4, atol=1e-4)
    if mode == "fused":
        assert not np.any(r["samp"])                  # control.py:135 zeros without the re-roll
    else:
        np.testing.assert_allclose(r["samp"], g["sampled_traj"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name", ["late_auto", "latechain_auto"])
def test_late_rank_falls_back_on_every_rank(ranks, name):
    """The in-launch exchange on its poll bound: both ranks ran the ticks before the late one in-launch, took
    the collective fallback in the late tick itself (no exception reached the caller) and stayed on it; the
    results are the single-process controller's at every tick (test_ranks_agree_and_match_single_process)."""
    for r in ranks:
        modes = list(_get(r, name)["modes"])
        assert modes[:LATE_TICK] == ["launch"] * LATE_TICK, modes
        assert all(m == "rccl" for m in modes[LATE_TICK:]), modes


def test_ranks_agree_on_the_noise_stream_whichever_way_they_drew(ranks):
    """one rank on the device NumPy draw, the other on the host draw — the first-step check passed
    (no 'ranks disagree' error, the in-launch exchange taken) and every step matched
    (test_ranks_agree_and_match_single_process[mixdraw_auto])."""
    assert bool(_get(ranks[0], "mixdraw_auto")["rankonly_devdraw"])
    assert not bool(_get(ranks[1], "mixdraw_auto")["rankonly_devdraw"])
