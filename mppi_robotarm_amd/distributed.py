"""Multi-GPU sharding of the MPPI samples (one process per GPU, RCCL over xGMI).

Samples are independent, so each rank simulates a contiguous slice of the K
samples (control.py:91-109 restricted to k in [k_offset, k_offset + K_local))
and reduces it on device to one partial row {rho, eta, N[T][2]}
(log-sum-exp form of control.py:112-118).  The only exchange of a control step
is ONE all-gather of those 2 + 2T doubles (1 KB at T = 64) over the process
group; every rank then merges the gathered rows on device in rank order
(deterministic, identical on all ranks) and continues with the same w_eps.
An all-gather (not an all-reduce) keeps the merge exact: rows carry their own
rho, so no prior MIN collective is needed.  The preferred form does without
the collective call: attach_exchange maps every rank's inbox once, and each
launch then trades the rows itself (include/mppi_rocm.h mppi_exchange_*);
check_exchange is its one-step self-check against the all-gather.
"""
from __future__ import annotations

import os
import sys

import torch
import torch.distributed as dist

# The in-launch exchange maps every rank's inbox through hipIpcGetMemHandle / hipIpcOpenMemHandle.  On this
# pool's host driver only the dmabuf form of HIP IPC exists; ROCm picks it when HSA_ENABLE_IPC_MODE_LEGACY=0,
# and without it the export fails with "hipIpcGetMemHandle: invalid argument" (RCCL's own intra-node transport
# uses the same IPC and fails the same way).  bench.py's self-launch sets it for its ranks; an external launcher
# must export it (the driver's and the GPU box's environment already does).
IPC_ENV = "HSA_ENABLE_IPC_MODE_LEGACY"


def ipc_env_ok() -> bool:
    """Whether this process has the dmabuf IPC mode the in-launch exchange needs (IPC_ENV=0)."""
    return os.environ.get(IPC_ENV) == "0"


def shard_geometry(K: int, world: int, rank: int) -> tuple[int, int]:
    """(K_local, k_offset) of `rank`: contiguous slices, the first K % world ranks one larger."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank / world size")
    if K < world:
        raise ValueError("number_of_samples_K must be >= the number of ranks")
    base, rem = divmod(K, world)
    return base + (1 if rank < rem else 0), rank * base + min(rank, rem)


def exchange_partials(partial: torch.Tensor, gathered: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather every rank's partial row into `gathered` ([world * len] fp64, rank order).

    With the "nccl" backend (RCCL on ROCm) both tensors live on the rank's GPU
    and the collective is ordered on the current stream; with "gloo" (CPU
    tests) they live on the host.
    """
    if partial.dtype != torch.float64 or gathered.dtype != torch.float64:
        raise TypeError("partials are fp64")
    world = dist.get_world_size(group)
    if gathered.numel() != world * partial.numel():
        raise ValueError("gathered must hold world_size partial rows")
    if partial.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device all-gather: stage the 1 KB rows through the host
        host = torch.empty(gathered.numel(), dtype=torch.float64)
        dist.all_gather_into_tensor(host, partial.cpu(), group=group)
        gathered.copy_(host)
        return gathered
    dist.all_gather_into_tensor(gathered, partial, group=group)
    return gathered


def gather_trajectories(tr: torch.Tensor, K_total: int, out, group=None):
    """Sampled trajectories of every rank's shard into `out` ((K_total, T, 4) fp64
    host array, rows in sample order): one all_gather_into_tensor of the fp32
    shards, each padded to the largest shard (shard_geometry), on the rank's GPU
    under "nccl" (RCCL over xGMI) or through the host under "gloo".  Replaces a
    pickled all_gather_object of ~67 MB per rank at K = 65536 per rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    K_local, _ = shard_geometry(K_total, world, rank)
    if tr.shape[0] != K_local:
        raise ValueError("trajectory shard does not match shard_geometry")
    K_max = shard_geometry(K_total, world, 0)[0]
    on_dev = tr.is_cuda and dist.get_backend(group) != "gloo"
    src = tr if on_dev else tr.cpu()
    if K_local < K_max:
        pad = torch.zeros((K_max - K_local,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
        src = torch.cat([src, pad])
    buf = torch.empty((world * K_max,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(buf, src.contiguous(), group=group)
    host = buf.cpu().numpy()
    for r in range(world):
        n, off = shard_geometry(K_total, world, r)
        out[off:off + n] = host[r * K_max:r * K_max + n]
    return out


def attach_exchange(engine, group=None, report: dict | None = None) -> bool:
    """Set up the in-launch exchange (include/mppi_rocm.h mppi_exchange_*): every
    rank exports its inbox's IPC handle, the handles are all-gathered over the
    group once, and every rank maps its peers' inboxes.  Afterwards
    ``engine.rollout(noise, exchange=True, fused_update=True)`` finishes a whole
    multi-GPU control step in one launch per rank.

    Collective-safe: every rank joins every collective whatever fails locally,
    and all ranks return the same answer (False: use exchange_partials).
    `report` (a dict) receives report["attach"]: the verdict, the failing ranks
    and their errors, and each rank's IPC_ENV (the same on every rank); a failure
    is also printed to stderr."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    env = os.environ.get(IPC_ENV)
    err = None
    try:
        h = engine.exchange_handle(world)
    except Exception as e:  # noqa: BLE001 - reported to every rank below
        h, err = None, f"handle: {e}"
        if env != "0":
            err += f" ({IPC_ENV}={env!r}: this driver's IPC needs {IPC_ENV}=0)"
    handles = [None] * world
    dist.all_gather_object(handles, h, group=group)
    if err is None and all(x is not None for x in handles):
        try:
            engine.exchange_attach(rank, world, handles)
        except Exception as e:  # noqa: BLE001
            err = f"attach: {e}"
    elif err is None:
        err = "a peer failed to export its handle"
    infos = [None] * world
    dist.all_gather_object(infos, (err, env), group=group)
    ok = all(i[0] is None for i in infos)
    if report is not None:
        report["attach"] = {"ok": ok, "failed_ranks": [r for r, i in enumerate(infos) if i[0] is not None],
                            "errors": {str(r): i[0] for r, i in enumerate(infos) if i[0] is not None},
                            "ipc_env": [i[1] for i in infos]}
    if not ok and rank == 0:
        first = next(i[0] for i in infos if i[0] is not None)
        print(f"mppi multi-GPU: in-launch exchange unavailable ({first}); the RCCL all-gather is used",
              file=sys.stderr, flush=True)
    return ok


def check_exchange(engine, noise, partial, gathered, group=None, report: dict | None = None) -> bool:
    """One step both ways from the same state (no update): the in-launch exchange
    must reproduce all-gather + device merge (1e-9) without a hand-off timeout.
    Every rank gets the same verdict; `report` receives report["check"] (the
    verdict, the failing ranks and why, each rank's largest w_eps difference)."""
    import numpy as np
    engine.rollout(noise, partial_out=partial)
    exchange_partials(partial, gathered, group)
    engine.merge(gathered, dist.get_world_size(group))
    w_ref = engine.weighted_noise()
    err, diff = None, None
    try:
        engine.rollout(noise, exchange=True)
        engine.synchronize()          # raises on a hand-off timeout
        w = engine.weighted_noise()
        diff = float(np.max(np.abs(w - w_ref)))
        if not np.allclose(w, w_ref, rtol=1e-9, atol=1e-12):
            err = f"w_eps differs from the all-gather's by {diff:.3g}"
    except Exception as e:  # noqa: BLE001
        err = f"in-launch step: {e}"
    infos = [None] * dist.get_world_size(group)
    dist.all_gather_object(infos, (err, diff), group=group)
    ok = all(i[0] is None for i in infos)
    if report is not None:
        report["check"] = {"ok": ok, "failed_ranks": [r for r, i in enumerate(infos) if i[0] is not None],
                           "errors": {str(r): i[0] for r, i in enumerate(infos) if i[0] is not None},
                           "max_abs_diff": [i[1] for i in infos]}
    if not ok and dist.get_rank(group) == 0:
        first = next(i[0] for i in infos if i[0] is not None)
        print(f"mppi multi-GPU: the in-launch exchange failed its self-check ({first}); the RCCL all-gather is used",
              file=sys.stderr, flush=True)
    return ok


def same_on_all_ranks(obj, group=None) -> bool:
    """True on every rank iff every rank passed an equal (picklable) `obj`."""
    objs = [None] * dist.get_world_size(group)
    dist.all_gather_object(objs, obj, group=group)
    return all(o == objs[0] for o in objs)

