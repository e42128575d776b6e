"""CPU, world_size 2 over gloo: the multi-GPU exchange of the drop-in
(mppi_robotarm_amd.distributed) — sharding, the one all-gather of per-rank
partial rows, and that merging the gathered rows in rank order reproduces the
unsharded weighted noise (control.py:112-118).  Each rank's partial row is
computed from the C fp64 oracle's per-sample costs of its shard with the same
{rho, eta, N} definition the device uses (include/mppi_rocm.h)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT  # noqa: F401

LAM = 3.0e6  # spread weights so every shard contributes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _partial_row(S, eps_kt, lam):
    rho = S.min()
    e = np.exp((rho - S) / lam)
    N = np.einsum("k,ktd->td", e, eps_kt.astype(np.float64))
    return np.concatenate([[rho, e.sum()], N.ravel()])


def _merge_rows(rows, lam):
    rho = rows[:, 0].min()
    s = np.exp((rho - rows[:, 0]) / lam)
    eta = (s * rows[:, 1]).sum()
    N = (s[:, None] * rows[:, 2:]).sum(0)
    return N.reshape(-1, 2) / eta


def _worker(rank, world, port, K, T, out_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    import mppi_oracle as O
    from mppi_robotarm_amd.distributed import exchange_partials, shard_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        path = np.load(os.path.join(GOLDEN, "paths.npz"))["xydq_circle"][:, :4]
        rng = np.random.default_rng(5)  # same draw on every rank (same seed, like np.random in the drop-in)
        eps = (rng.standard_normal((K, T, 2)) * np.sqrt(20.0)).astype(np.float32)
        u = np.array([[10.0, -2.0]] * T)
        x0 = np.array([1.152198236517471885, -1.266101672070702344, 0.0, 0.0])
        n, off = shard_geometry(K, world, rank)
        S = coracle.rollout_costs(x0, u, eps, path[:30], 0.006, LAM, 0.9, np.eye(2) * 20.0,
                                  [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0], O.ArmParams(),
                                  k_range=(off, off + n), k_exploit=K)
        partial = torch.from_numpy(_partial_row(S, eps[off:off + n], LAM))
        gathered = torch.empty(world * partial.numel(), dtype=torch.float64)
        exchange_partials(partial, gathered)
        w_eps = _merge_rows(gathered.numpy().reshape(world, -1), LAM)
        np.save(f"{out_path}.{rank}.npy", w_eps)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("K,T", [(600, 16), (257, 9)])
def test_sharded_exchange_matches_unsharded(tmp_path, K, T):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import coracle
    import mppi_oracle as O
    world = 2
    out = str(tmp_path / "weps")
    mp.start_processes(_worker, args=(world, _free_port(), K, T, out), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert np.array_equal(r0, r1)  # every rank continues with identical w_eps
    path = np.load(os.path.join(GOLDEN, "paths.npz"))["xydq_circle"][:, :4]
    rng = np.random.default_rng(5)
    eps = (rng.standard_normal((K, T, 2)) * np.sqrt(20.0)).astype(np.float32)
    S = coracle.rollout_costs(np.array([1.152198236517471885, -1.266101672070702344, 0.0, 0.0]),
                              np.array([[10.0, -2.0]] * T), eps, path[:30], 0.006, LAM, 0.9,
                              np.eye(2) * 20.0, [0.5, 0.5, 5.0, 5.0], [5.0, 5.0, 50.0, 50.0], O.ArmParams())
    w, ref = coracle.weighted_noise(S, eps, LAM)
    assert 1.0 / np.sum(w ** 2) > 5            # weights really are spread over samples
    np.testing.assert_allclose(r0, ref, rtol=1e-10, atol=1e-12)


def test_exchange_rejects_bad_shapes(tmp_path):
    from mppi_robotarm_amd.distributed import exchange_partials
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        with pytest.raises(ValueError):
            exchange_partials(torch.zeros(10, dtype=torch.float64), torch.zeros(11, dtype=torch.float64))
        with pytest.raises(TypeError):
            exchange_partials(torch.zeros(10), torch.zeros(10))
        g = exchange_partials(torch.arange(4, dtype=torch.float64), torch.zeros(4, dtype=torch.float64))
        assert g.tolist() == [0.0, 1.0, 2.0, 3.0]
    finally:
        dist.destroy_process_group()
