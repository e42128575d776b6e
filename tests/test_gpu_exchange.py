"""GPU: the in-launch multi-GPU exchange (include/mppi_rocm.h mppi_exchange_*),
rehearsed with 2 ranks on ONE GPU (the inboxes are IPC-mapped device memory on
the same device; on a node each rank maps its peers' memory over xGMI).

Each rank simulates its contiguous shard of K samples with Philox noise (an
exact slice of the unsharded draw), and every launch exchanges the ranks'
partial rows and merges them itself (one launch per step, no collective call).
The weighted noise and the nominal after each fused step must equal the
unsharded engine's (1e-10: merge order differs, the rows are the same).
gloo carries only the one-time handle exchange.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

K, T, STEPS = 12288, 24, 4
LAM = 1.0e7   # spread weights: every shard's row matters


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(K_local, K_total, k_offset, lps=0):
    from mppi_robotarm_amd.engine import RolloutEngine
    from mppi_robotarm_amd.params import ArmParams
    return RolloutEngine(K_local, T, 0.006, LAM, 0.98, np.eye(2) * 20.0, [0.5, 0.5, 5, 5], [5, 5, 50, 50], 0.0,
                         ArmParams(), K_total=K_total, k_offset=k_offset, device=0, lanes_per_sample=lps)


def _inputs():
    from mppi_robotarm_amd.params import X0_RUNPY
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = np.load(os.path.join(root, "tests", "golden", "paths.npz"))["xydq_circle"][:, :4]
    return X0_RUNPY, path[:30], np.array([[10.0, -2.0]] * T)


def _rank(rank, world, port, out):
    import torch.distributed as dist
    from mppi_robotarm_amd.distributed import attach_exchange, shard_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        n, off = shard_geometry(K, world, rank)
        eng = _engine(n, K, off)
        x0, win, u = _inputs()
        eng.set_step_inputs(x0, win, u)
        attach_exchange(eng)
        res = []
        for s in range(STEPS):
            eng.rollout(eng.philox_noise(9, s), fused_update=True, exchange=True)
            res.append((eng.weighted_noise(), eng.nominal()))
        eng.synchronize()
        np.save(f"{out}.{rank}.npy", np.array([[w, u] for w, u in res]))
        eng.close()
    finally:
        dist.destroy_process_group()


def test_exchange_two_ranks_match_unsharded(tmp_path):
    import torch.multiprocessing as mp
    torch.cuda.set_device(0)
    out = str(tmp_path / "x")
    mp.start_processes(_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert np.array_equal(r0, r1)          # every rank merged the same rows in the same order
    full = _engine(K, K, 0)
    x0, win, u = _inputs()
    full.set_step_inputs(x0, win, u)
    for s in range(STEPS):
        full.rollout(full.philox_noise(9, s), fused_update=True)
        np.testing.assert_allclose(r0[s, 0], full.weighted_noise(), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(r0[s, 1], full.nominal(), rtol=1e-10, atol=1e-12)
    full.close()


def test_exchange_flag_needs_attach():
    eng = _engine(1024, 1024, 0)
    x0, win, u = _inputs()
    eng.set_step_inputs(x0, win, u)
    with pytest.raises(Exception):
        eng.rollout(eng.philox_noise(1, 0), exchange=True)
    with pytest.raises(Exception):
        eng.exchange_attach(0, 2, [b"\0" * 64] * 2)   # before exchange_handle
    eng.close()


CK, CT = 6144, 16


def _chain_rank(rank, world, port, out, precision="f32", lps=0):
    import torch.distributed as dist
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
    from mppi_robotarm_amd.distributed import attach_exchange, shard_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        n, off = shard_geometry(CK, world, rank)
        eng = ChainEngine(n, CT, 0.006, 1.0e5, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50],
                          K_total=CK, k_offset=off, device=0, precision=precision, lanes_per_sample=lps)
        _, win, _ = _inputs()
        eng.set_step_inputs(CHAIN7_X0, win, np.tile(gravity_torque(CHAIN7_X0[:7]), (CT, 1)))
        attach_exchange(eng)
        res = []
        for s in range(STEPS):
            eng.rollout(eng.philox_noise(4, s), fused_update=True, exchange=True)
            res.append((eng.weighted_noise(), eng.nominal()))
        np.save(f"{out}.{rank}.npy", np.array([[w, u] for w, u in res]))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("precision,lps", [("f32", 1), ("f32", 4), ("f64", 1)])
def test_chain_exchange_two_ranks_match_unsharded(precision, lps, tmp_path):
    """Config 5's multi-GPU step: (2 + 7T) rows exchanged inside the launch, for one lane and a quad per sample
    and for the fp64 rollout."""
    import torch.multiprocessing as mp
    from mppi_robotarm_amd.chain import CHAIN7_SIGMA, CHAIN7_X0, ChainEngine, gravity_torque
    torch.cuda.set_device(0)
    out = str(tmp_path / "c")
    mp.start_processes(_chain_rank, args=(2, _free_port(), out, precision, lps), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert np.array_equal(r0, r1)
    full = ChainEngine(CK, CT, 0.006, 1.0e5, 0.98, CHAIN7_SIGMA, [0.5, 0.5, 5, 5], [5, 5, 50, 50], device=0,
                       precision=precision, lanes_per_sample=lps)
    _, win, _ = _inputs()
    full.set_step_inputs(CHAIN7_X0, win, np.tile(gravity_torque(CHAIN7_X0[:7]), (CT, 1)))
    for s in range(STEPS):
        full.rollout(full.philox_noise(4, s), fused_update=True)
        np.testing.assert_allclose(r0[s, 0], full.weighted_noise(), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(r0[s, 1], full.nominal(), rtol=1e-10, atol=1e-12)
    full.close()
