"""GPU: the in-launch multi-GPU exchange at world 2, 4 and 8, rehearsed on ONE GPU.

Config 4 runs the exchange with 8 ranks (one per GPU of a node): the [parity][rank]
inbox slots, the status round over world ranks, 7 peer stores per granule and the
8-row merge (mppi_device.h exchange_send_merge / exchange_verdict).  The pool's
boxes have one GPU, so the ranks share it: every rank's grid must be resident at
the same time as every other rank's (the exchange polls for the peers' rows inside
the launch).  The grids are therefore small — K_total = 8 x 1536 samples at one lane
per sample is 6 workgroups per rank at world 8 — and each rank process keeps its
streams on one hardware queue (GPU_MAX_HW_QUEUES=1, set before its first HIP call),
so 8 ranks plus this process stay within the queues the device schedules at once.

Checked per world size, over 4 fused steps with spread weights (lambda = 1e7, every
shard's row carries weight):
  * every rank's w_eps and nominal are bit-equal (same rows, same rank-order merge);
  * they equal the unsharded engine's (1e-10: only the summation order differs);
  * step 0's w_eps equals the C fp64 oracle's on the same noise (U_TOL, BASELINE.json's 1e-4);
and the same for the 7-link chain (a quad per sample and one lane per sample), plus a
late rank at world 4 through the drop-in controller (every rank falls back to the
all-gather in that tick and stays there; results equal the single-process controller).
Reference: /root/reference/control.py:112-118 (the soft-min merge the exchange splits).
"""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from conftest import ROOT  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import coracle  # noqa: E402  (checker only)

K, T, STEPS, LAM = 8 * 1536, 24, 4, 1.0e7
U_TOL = 1e-4
X_TOL = 1e-10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs():
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    from mppi_robotarm_amd.params import X0_RUNPY
    return X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T)


def _engine(K_local, K_total, k_offset, lps):
    from mppi_robotarm_amd.engine import RolloutEngine
    from mppi_robotarm_amd.params import ArmParams
    return RolloutEngine(K_local, T, 0.006, LAM, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                         ArmParams(), K_total=K_total, k_offset=k_offset, device=0, lanes_per_sample=lps)


def _init(rank, world, port):
    os.environ["GPU_MAX_HW_QUEUES"] = "1"          # read at this process's first HIP call (below)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    return dist


def _rank(rank, world, port, out):
    dist = _init(rank, world, port)
    try:
        from mppi_robotarm_amd.distributed import attach_exchange, shard_geometry
        n, off = shard_geometry(K, world, rank)
        eng = _engine(n, K, off, 1)
        x0, win, u = _inputs()
        eng.set_step_inputs(x0, win, u)
        assert attach_exchange(eng), "exchange set-up failed"
        res = []
        for s in range(STEPS):
            eng.rollout(eng.philox_noise(9, s), fused_update=True, exchange=True)
            res.append((eng.weighted_noise(), eng.nominal()))
        eng.synchronize()
        np.save(f"{out}.{rank}.npy", np.array([[w, v] for w, v in res]))
        np.save(f"{out}.{rank}.geo.npy", np.array([eng.blocks, eng.lanes_per_sample, int(eng.handoff == "poll")]))
        eng.close()
    finally:
        dist.destroy_process_group()


def _spawn(fn, world, *args):
    import torch.multiprocessing as mp
    mp.start_processes(fn, args=(world, _free_port()) + args, nprocs=world, join=True, start_method="spawn")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_exchange_world_matches_unsharded_and_oracle(world, tmp_path):
    torch.cuda.set_device(0)
    out = str(tmp_path / "x")
    _spawn(_rank, world, out)
    r = [np.load(f"{out}.{k}.npy") for k in range(world)]
    geo = [np.load(f"{out}.{k}.geo.npy") for k in range(world)]
    assert sum(int(g[0]) for g in geo) <= torch.cuda.get_device_properties(0).multi_processor_count
    for k in range(1, world):
        assert np.array_equal(r[k], r[0]), f"rank {k} merged differently from rank 0"
    full = _engine(K, K, 0, 0)
    x0, win, u = _inputs()
    full.set_step_inputs(x0, win, u)
    for s in range(STEPS):
        noise = full.philox_noise(9, s)
        full.rollout(noise, fused_update=True)
        np.testing.assert_allclose(r[0][s, 0], full.weighted_noise(), rtol=X_TOL, atol=1e-12)
        np.testing.assert_allclose(r[0][s, 1], full.nominal(), rtol=X_TOL, atol=1e-12)
        if s == 0:
            eps_tk = noise.cpu().numpy()
            from mppi_robotarm_amd.params import ArmParams
            S = coracle.rollout_costs(x0, u, eps_tk, win, 0.006, LAM, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5],
                                      [5, 5, 50, 50], ArmParams(), layout="TK")
            w, ref = coracle.weighted_noise(S, eps_tk, LAM, layout="TK")
            assert np.sort(w)[-2] > 1e-6   # spread weights: more than one sample carries weight
            err = float(np.max(np.abs(r[0][0, 0] - ref)) / max(1.0, float(np.max(np.abs(ref)))))
            assert err < U_TOL, err
    full.close()


CK, CT = 6144, 16


def _chain_rank(rank, world, port, out, lps):
    dist = _init(rank, world, port)
    try:
        from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
        from mppi_robotarm_amd.distributed import attach_exchange, shard_geometry
        n, off = shard_geometry(CK, world, rank)
        eng = ChainEngine(n, CT, 0.006, 1.0e5, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50],
                          K_total=CK, k_offset=off, device=0, lanes_per_sample=lps)
        _, win, _ = _inputs()
        eng.set_step_inputs(CHAIN7_X0, win, np.tile(gravity_torque(CHAIN7_X0[:7]), (CT, 1)))
        assert attach_exchange(eng), "exchange set-up failed"
        res = []
        for s in range(STEPS):
            eng.rollout(eng.philox_noise(4, s), fused_update=True, exchange=True)
            res.append((eng.weighted_noise(), eng.nominal()))
        np.save(f"{out}.{rank}.npy", np.array([[w, v] for w, v in res]))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lps", [(4, 4), (8, 4), (8, 1)])
def test_chain_exchange_world_matches_unsharded(world, lps, tmp_path):
    """Config 5's multi-GPU step ((2 + 7T)-value rows) at world 4 and 8, a quad and one lane per sample."""
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
    torch.cuda.set_device(0)
    out = str(tmp_path / "c")
    _spawn(_chain_rank, world, out, lps)
    r = [np.load(f"{out}.{k}.npy") for k in range(world)]
    for k in range(1, world):
        assert np.array_equal(r[k], r[0]), f"rank {k} merged differently from rank 0"
    full = ChainEngine(CK, CT, 0.006, 1.0e5, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], device=0,
                       lanes_per_sample=lps)
    _, win, _ = _inputs()
    full.set_step_inputs(CHAIN7_X0, win, np.tile(gravity_torque(CHAIN7_X0[:7]), (CT, 1)))
    for s in range(STEPS):
        full.rollout(full.philox_noise(4, s), fused_update=True)
        np.testing.assert_allclose(r[0][s, 0], full.weighted_noise(), rtol=X_TOL, atol=1e-12)
        np.testing.assert_allclose(r[0][s, 1], full.nominal(), rtol=X_TOL, atol=1e-12)
    full.close()


LATE_WORLD, LATE_RANK, LATE_TICK, LATE_SLEEP_S, TICKS = 4, 2, 2, 0.5, 5
DEV_K, DEV_T = 8192, 32


def _late_ticks(pg):
    """The drop-in with device noise, one lane per sample (small grids: world 4 shares one GPU); rank LATE_RANK
    starts tick LATE_TICK LATE_SLEEP_S late, past the 30 ms poll bound."""
    import time
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.params import runpy_config
    path = np.load(os.path.join(ROOT, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    kw = runpy_config()
    kw.update(number_of_samples_K=DEV_K, horizon_step_T=DEV_T, visualze_sampled_trajs=False)
    rank = pg.rank() if pg is not None else 0
    os.environ["MPPI_EXCHANGE_TIMEOUT_US"] = "30000"
    try:
        c = MPPIControllerForPathTracking(ref_path=path, verbose=False, noise="device", seed=11, process_group=pg,
                                          lanes_per_sample=1, **kw)
        from mppi_robotarm_amd.params import X0_RUNPY
        x = X0_RUNPY.copy()
        useq, modes = [], []
        for i in range(TICKS):
            if i == LATE_TICK and rank == LATE_RANK:
                time.sleep(LATE_SLEEP_S)
            _, u_seq, _, _ = c.calc_control_input(x)
            useq.append(u_seq.copy())
            modes.append(str(c._xmode))
            x = x + 0.001 * (i + 1)
        c.close()
    finally:
        del os.environ["MPPI_EXCHANGE_TIMEOUT_US"]
    return np.array(useq), modes


def _late_rank(rank, world, port, out):
    dist = _init(rank, world, port)
    try:
        useq, modes = _late_ticks(dist.group.WORLD)
        np.save(f"{out}.{rank}.npy", useq)
        np.save(f"{out}.{rank}.modes.npy", np.array(modes))
    finally:
        dist.destroy_process_group()


def test_late_rank_world4_falls_back_on_every_rank(tmp_path):
    torch.cuda.set_device(0)
    out = str(tmp_path / "late")
    _spawn(_late_rank, LATE_WORLD, out)
    single, _ = _late_ticks(None)
    for k in range(LATE_WORLD):
        modes = list(np.load(f"{out}.{k}.modes.npy"))
        assert modes[:LATE_TICK] == ["launch"] * LATE_TICK, (k, modes)
        assert all(m == "rccl" for m in modes[LATE_TICK:]), (k, modes)
        u = np.load(f"{out}.{k}.npy")
        np.testing.assert_allclose(u, single, rtol=X_TOL, atol=X_TOL)
