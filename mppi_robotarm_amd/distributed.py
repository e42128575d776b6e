"""Multi-GPU sharding of the MPPI samples (one process per GPU, RCCL over xGMI).

Samples are independent, so each rank simulates a contiguous slice of the K
samples (control.py:91-109 restricted to k in [k_offset, k_offset + K_local))
and reduces it on device to one partial row {rho, eta, N[T][2]}
(log-sum-exp form of control.py:112-118).  The only exchange of a control step
is ONE all-gather of those 2 + 2T doubles (1 KB at T = 64) over the process
group; every rank then merges the gathered rows on device in rank order
(deterministic, identical on all ranks) and continues with the same w_eps.
An all-gather (not an all-reduce) keeps the merge exact: rows carry their own
rho, so no prior MIN collective is needed.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


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
