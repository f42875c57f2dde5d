"""Multi-GPU plumbing: one process per GPU, lanes sharded across ranks, and the ONE
collective of the hot path — the all-reduce of the fp64 RFF feature sum and the sample
count before the MMD witness (RBFLinearCost.fit_cost's global mean,
milo/milo/linear_cost.py:84-94).  Everything per-sample stays rank-local.

On ROCm the "nccl" backend of torch.distributed is RCCL (xGMI inside a node); the same
code runs on "gloo" with CPU tensors for the CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def allreduce_sum(t: torch.Tensor) -> torch.Tensor:
    """In-place SUM over ranks (no-op without an initialised process group)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def allreduce_max(t: torch.Tensor) -> torch.Tensor:
    """In-place MAX over ranks: the ensemble threshold when the offline set is sharded
    (compute_threshold's global max, milo/milo/dynamics.py:145-152)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t


def feature_mean(phi_sum: torch.Tensor, count: float | torch.Tensor, allreduce=allreduce_sum) -> torch.Tensor:
    """Global mean of the RFF features from per-rank fp64 sums: ONE fused all-reduce of
    [phi_sum (F), count] (a 4 KB message: latency-bound, a single RCCL call)."""
    F = phi_sum.numel()
    buf = torch.empty(F + 1, dtype=torch.float64, device=phi_sum.device)
    buf[:F] = phi_sum
    buf[F] = count if not isinstance(count, torch.Tensor) else count.reshape(())
    allreduce(buf)
    return buf[:F] / buf[F]


def shard(total: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous [start, end) of `total` units for `rank` (strong-scaling lane split)."""
    base, rem = divmod(total, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def rank_seed(seed: int, rank: int) -> int:
    """Independent Philox key per rank (the lane counter restarts at 0 on every rank)."""
    return (int(seed) + (int(rank) << 40)) & 0xFFFFFFFFFFFFFFFF
