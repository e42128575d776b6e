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


def _chain_inputs(K, T):
    import chain_oracle as CO
    rng = np.random.default_rng(8)
    x0 = np.concatenate([[1.481492] + [-0.320757] * 6, [0.0] * 7])
    sig = np.diag([20.0, 16.0, 12.0, 8.0, 4.0, 2.0, 1.0])
    u = np.tile(CO.gravity_torque(x0[:7], CO.ChainParams()), (T, 1))
    eps = (rng.standard_normal((K, T, 7)) * np.sqrt(np.diag(sig))).astype(np.float32)
    return x0, u, sig, eps


def _chain_worker(rank, world, port, K, T, out_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import chain_oracle as CO
    import coracle
    from mppi_robotarm_amd.distributed import exchange_partials, shard_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        path = np.load(os.path.join(GOLDEN, "paths.npz"))["xydq_circle"][:, :4]
        x0, u, sig, eps = _chain_inputs(K, T)
        n, off = shard_geometry(K, world, rank)
        S = coracle.chain_rollout_costs(x0, u, eps, path[:30], 0.006, CHAIN_LAM, 0.98, sig, [0.5, 0.5, 5.0, 5.0],
                                        [5.0, 5.0, 50.0, 50.0], CO.ChainParams(), k_range=(off, off + n))
        partial = torch.from_numpy(_partial_row(S, eps[off:off + n], CHAIN_LAM))   # 2 + 7 T values
        gathered = torch.empty(world * partial.numel(), dtype=torch.float64)
        exchange_partials(partial, gathered)
        rows = gathered.numpy().reshape(world, -1)
        rho = rows[:, 0].min()
        s = np.exp((rho - rows[:, 0]) / CHAIN_LAM)
        w_eps = ((s[:, None] * rows[:, 2:]).sum(0) / (s * rows[:, 1]).sum()).reshape(T, 7)
        np.save(f"{out_path}.{rank}.npy", w_eps)
    finally:
        dist.destroy_process_group()


CHAIN_LAM = 1.0e4


@pytest.mark.parametrize("K,T", [(300, 12), (131, 5)])
def test_chain_sharded_exchange_matches_unsharded(tmp_path, K, T):
    """Config 5's exchange: the 7-link chain's (2 + 7T) partial rows over 2 ranks."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import chain_oracle as CO
    import coracle
    world = 2
    out = str(tmp_path / "weps")
    mp.start_processes(_chain_worker, args=(world, _free_port(), K, T, out), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    assert np.array_equal(r0, r1)
    path = np.load(os.path.join(GOLDEN, "paths.npz"))["xydq_circle"][:, :4]
    x0, u, sig, eps = _chain_inputs(K, T)
    S = coracle.chain_rollout_costs(x0, u, eps, path[:30], 0.006, CHAIN_LAM, 0.98, sig, [0.5, 0.5, 5.0, 5.0],
                                    [5.0, 5.0, 50.0, 50.0], CO.ChainParams())
    w, ref = coracle.chain_weighted_noise(S, eps, CHAIN_LAM)
    assert 1.0 / np.sum(w ** 2) > 3            # several samples carry weight
    np.testing.assert_allclose(r0, ref, rtol=1e-10, atol=1e-12)


class _FakeEngine:
    """Stands in for an engine in the exchange set-up (no GPU): rank `bad` fails at `where`."""

    def __init__(self, rank, bad, where):
        self.rank, self.bad, self.where, self.attached = rank, bad, where, None

    def exchange_handle(self, world):
        if self.rank == self.bad and self.where == "handle":
            raise RuntimeError("no inbox")
        return bytes([self.rank]) * 64

    def exchange_attach(self, rank, world, handles):
        if self.rank == self.bad and self.where == "attach":
            raise RuntimeError("cannot map")
        self.attached = [h[0] for h in handles]


def _attach_worker(rank, world, port, bad, where, out_path):
    import sys
    sys.path.insert(0, ROOT)
    from mppi_robotarm_amd.distributed import attach_exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _FakeEngine(rank, bad, where)
        ok = attach_exchange(eng)
        np.save(f"{out_path}.{rank}.npy", np.array([int(ok)] + (eng.attached or [-1] * world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad,where", [(-1, ""), (1, "handle"), (0, "attach")])
def test_attach_exchange_is_collective_safe(tmp_path, bad, where):
    """A rank that cannot export or map inboxes makes EVERY rank fall back (same
    verdict everywhere, no rank left waiting in a collective)."""
    world = 2
    out = str(tmp_path / "att")
    mp.start_processes(_attach_worker, args=(world, _free_port(), bad, where, out), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(f"{out}.{k}.npy") for k in range(world)]
    assert r[0][0] == r[1][0] == (1 if bad < 0 else 0)
    if bad < 0:
        assert r[0][1:].tolist() == r[1][1:].tolist() == [0, 1]   # handles in rank order


def _traj_worker(rank, world, port, K, T, out_path):
    import sys
    sys.path.insert(0, ROOT)
    from mppi_robotarm_amd.distributed import gather_trajectories, shard_geometry
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, off = shard_geometry(K, world, rank)
        # this rank's shard of a known (K, T, 4) array, fp32 like the device re-roll
        full = np.arange(K * T * 4, dtype=np.float32).reshape(K, T, 4)
        out = np.zeros((K, T, 4))
        gather_trajectories(torch.from_numpy(full[off:off + n].copy()), K, out)
        np.save(f"{out_path}.{rank}.npy", out)
        with pytest.raises(ValueError):
            gather_trajectories(torch.zeros((n + 1, T, 4)), K, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("K,world", [(10, 3), (12, 2)])
def test_gather_trajectories_uneven_shards(tmp_path, K, world):
    """Sampled trajectories (control.py:136-145, run.py:36) of uneven shards come
    back in sample order on every rank (tensor all-gather, padded shards)."""
    T = 5
    out = str(tmp_path / "traj")
    mp.start_processes(_traj_worker, args=(world, _free_port(), K, T, out), nprocs=world, join=True,
                       start_method="spawn")
    ref = np.arange(K * T * 4, dtype=np.float32).reshape(K, T, 4).astype(np.float64)
    for r in range(world):
        assert np.array_equal(np.load(f"{out}.{r}.npy"), ref)


def _setup_worker(rank, world, port, seeds_differ, out_path):
    import sys
    sys.path.insert(0, ROOT)
    from mppi_robotarm_amd.controller import MPPIControllerForPathTracking
    from mppi_robotarm_amd.distributed import same_on_all_ranks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = [int(same_on_all_ranks(("k", 3), None)), int(same_on_all_ranks(("k", rank), None))]
        c = MPPIControllerForPathTracking(ref_path=np.zeros((40, 4)), verbose=False, noise="device",
                                          seed=rank if seeds_differ else 7, process_group=dist.group.WORLD,
                                          exchange="rccl")
        try:
            c._multi_setup(None, None)          # the engine is not touched on the RCCL path
            res.append(1 if c._xmode == "rccl" else -1)
        except RuntimeError:
            res.append(0)
        np.save(f"{out_path}.{rank}.npy", np.array(res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("seeds_differ", [False, True])
def test_multi_gpu_controller_checks_the_noise_stream(tmp_path, seeds_differ):
    """The multi-GPU drop-in's first step: ranks that would draw different noise
    streams stop on every rank (RuntimeError), instead of merging inconsistent shards."""
    world = 2
    out = str(tmp_path / "setup")
    mp.start_processes(_setup_worker, args=(world, _free_port(), seeds_differ, out), nprocs=world, join=True,
                       start_method="spawn")
    for r in range(world):
        assert np.load(f"{out}.{r}.npy").tolist() == [1, 0, 0 if seeds_differ else 1]


def _report_worker(rank, world, port, bad, where, out_path):
    import json
    import sys
    sys.path.insert(0, ROOT)
    from mppi_robotarm_amd.distributed import attach_exchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if rank == 1 and where == "handle":
        os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)   # the env the driver's IPC needs, missing on one rank
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rep = {}
        ok = attach_exchange(_FakeEngine(rank, bad, where), report=rep)
        json.dump({"ok": ok, "report": rep}, open(f"{out_path}.{rank}.json", "w"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad,where", [(-1, ""), (1, "handle"), (0, "attach")])
def test_attach_exchange_reports_why(tmp_path, bad, where):
    """bench.py --gpus N records the step-1 self-check (exchange_selfcheck): every rank gets the same report of
    the failing ranks, their errors (a failed handle export names the missing HSA_ENABLE_IPC_MODE_LEGACY=0) and
    each rank's IPC environment."""
    import json
    world = 2
    out = str(tmp_path / "rep")
    env = dict(os.environ)
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    try:
        mp.start_processes(_report_worker, args=(world, _free_port(), bad, where, out), nprocs=world, join=True,
                           start_method="spawn")
    finally:
        os.environ.clear()
        os.environ.update(env)
    r = [json.load(open(f"{out}.{k}.json")) for k in range(world)]
    assert r[0] == r[1]
    a = r[0]["report"]["attach"]
    assert r[0]["ok"] is a["ok"] is (bad < 0)
    if bad < 0:
        assert a["failed_ranks"] == [] and a["errors"] == {} and a["ipc_env"] == ["0", "0"]
    elif where == "handle":
        assert 1 in a["failed_ranks"] and "no inbox" in a["errors"]["1"]
        assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in a["errors"]["1"] and a["ipc_env"] == ["0", None]
    else:
        assert a["failed_ranks"] == [0] and "cannot map" in a["errors"]["0"]


class _CostEngine:
    device = "cpu"

    def __init__(self):
        self.calls = []

    def rollout(self, noise, partial_out=None, fused_update=False, exchange=False):
        self.calls.append(("rollout", exchange, partial_out is not None))

    def merge(self, gathered, n, fused_update=False):
        self.calls.append(("merge", n))

    def synchronize(self):
        pass


def _cost_worker(rank, world, port, xmode, out_path):
    import json
    import sys
    sys.path.insert(0, ROOT)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _CostEngine()
        partial, gathered = torch.zeros(6, dtype=torch.float64), torch.zeros(12, dtype=torch.float64)

        class A:
            backend = "gloo"
        out = bench.exchange_costs(eng, [None, None], partial, gathered, world, xmode, A(), steps=5)
        json.dump({"costs": out, "calls": eng.calls}, open(f"{out_path}.{rank}.json", "w"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("xmode", ["launch", "rccl"])
def test_bench_exchange_costs_fields(tmp_path, xmode):
    """bench.py's exchange_costs (the N > 1 JSON line's per-step cost of each exchange on the node): the fields,
    each leg's launches, and the in-launch leg only when that exchange was attached."""
    import json
    world = 2
    out = str(tmp_path / "cost")
    mp.start_processes(_cost_worker, args=(world, _free_port(), xmode, out), nprocs=world, join=True,
                       start_method="spawn")
    for k in range(world):
        r = json.load(open(f"{out}.{k}.json"))
        c = r["costs"]
        assert set(c) == {"steps", "no_exchange_ms_per_step", "rccl_allgather_merge_ms_per_step", "in_launch_ms_per_step"}
        assert c["steps"] == 5 and c["no_exchange_ms_per_step"] > 0 and c["rccl_allgather_merge_ms_per_step"] > 0
        assert (c["in_launch_ms_per_step"] is None) == (xmode != "launch")
        n_ex = sum(1 for x in r["calls"] if x[0] == "rollout" and x[1])
        assert n_ex == (5 if xmode == "launch" else 0)
        assert sum(1 for x in r["calls"] if x[0] == "merge") == 5


def test_bench_launcher_env_and_command():
    """bench.py --gpus N without a launcher: the ranks get HSA_ENABLE_IPC_MODE_LEGACY=0 and a 127.0.0.1
    rendezvous."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    env = bench.launcher_env()
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    cmd = bench.launcher_cmd(8, 29500, ["--gpus", "8"])
    assert "--master-addr" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert "--nproc-per-node=8" in cmd and cmd[-2:] == ["--gpus", "8"]
