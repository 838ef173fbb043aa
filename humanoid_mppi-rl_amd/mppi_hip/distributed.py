"""Multi-GPU MPPI: independent solves sharded over ranks, RCCL all-gather of the reduced controls only.

SURVEY 8(e): B initial states (config #4: 64) are split into contiguous shards of ceil(B/world) solves, one
process per GPU; each rank runs its shard through its own engine (no data-path collective), then one
all_gather of U* [B_local, nu, H] and u0 [B_local, nu] gives every rank the full controls. With the nccl
backend this is RCCL over xGMI (~43 KB per rank for the humanoid config: latency-bound, not bandwidth-bound).
The gather is the only collective; the reference has none (it solves one state at a time on host threads).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int, int]:
    """(start, stop, per_rank): rank r owns solves [start, stop); per_rank = ceil(n_total / world)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    per = -(-n_total // world)
    start = min(n_total, rank * per)
    stop = min(n_total, start + per)
    return start, stop, per


def pad_shard(x: np.ndarray, per: int) -> np.ndarray:
    """Pad a shard to `per` rows by repeating its last row (fixed-size all_gather); empty shards get zeros."""
    if x.shape[0] == per:
        return x
    if x.shape[0] == 0:
        return np.zeros((per,) + x.shape[1:], x.dtype)
    return np.concatenate([x, np.repeat(x[-1:], per - x.shape[0], axis=0)], axis=0)


@dataclass
class GatherResult:
    U: "object"   # [n_total, nu, H] (torch tensor on the rank's device)
    u0: "object"  # [n_total, nu]


def all_gather_controls(U_local, u0_local, n_total: int, group=None) -> GatherResult:
    """Gather every rank's reduced controls (torch tensors [per, nu, H], [per, nu]) and trim the padding."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    per = U_local.shape[0]
    U_all = torch.empty((world * per,) + tuple(U_local.shape[1:]), dtype=U_local.dtype, device=U_local.device)
    u0_all = torch.empty((world * per,) + tuple(u0_local.shape[1:]), dtype=u0_local.dtype, device=u0_local.device)
    if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
        dist.all_gather(list(U_all.chunk(world)), U_local.contiguous(), group=group)
        dist.all_gather(list(u0_all.chunk(world)), u0_local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(U_all, U_local.contiguous(), group=group)
        dist.all_gather_into_tensor(u0_all, u0_local.contiguous(), group=group)
    return GatherResult(U=U_all[:n_total], u0=u0_all[:n_total])


def solve_sharded(x0_all: np.ndarray, U_all: np.ndarray, solve_local: Callable, rank: int, world: int, group=None,
                  device=None) -> GatherResult:
    """One distributed MPPI step: rank-local solves of its shard, then the controls all-gather.

    solve_local(x0 [per, nx], U [per, nu, H]) -> (U_new [per, nu, H], u0 [per, nu]) as numpy arrays; on a GPU
    rank it wraps Engine.solve(..., shift=True), in the CPU tests an oracle-backed stand-in.
    """
    import torch

    n_total = x0_all.shape[0]
    start, stop, per = shard_bounds(n_total, rank, world)
    x0 = pad_shard(np.asarray(x0_all[start:stop]), per)
    U = pad_shard(np.asarray(U_all[start:stop]), per)
    U_new, u0 = solve_local(x0, U)
    dev = torch.device("cpu") if device is None else device
    return all_gather_controls(torch.as_tensor(np.asarray(U_new, np.float32), device=dev),
                               torch.as_tensor(np.asarray(u0, np.float32), device=dev), n_total, group)


class ControlGatherer:
    """Pipelined all-gather of each step's reduced controls for a stream of solves (bench.py's timed loop).

    submit(U, u0) snapshots the rank's controls on the current (compute) stream and starts the collective
    asynchronously (RCCL runs it on its own stream), so step i's gather overlaps step i+1's solve, which updates
    U in place. Snapshots and outputs rotate over `depth` slots; a slot is reused only after its gather has
    completed (work.wait() orders the compute stream behind it without blocking the host). drain() waits for all.
    result(slot) is the gathered (U_all [world*per, nu, H], u0_all [world*per, nu]) of that submit.
    """

    def __init__(self, U, u0, group=None, depth: int = 2):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.nccl = dist.get_backend(group) != "gloo"
        self.depth = depth
        self.snap = [(torch.empty_like(U), torch.empty_like(u0)) for _ in range(depth)]
        self.out = [(U.new_empty((self.world * U.shape[0],) + tuple(U.shape[1:])),
                     u0.new_empty((self.world * u0.shape[0],) + tuple(u0.shape[1:]))) for _ in range(depth)]
        self.work = [None] * depth
        self.n = 0

    def submit(self, U, u0) -> int:
        k = self.n % self.depth
        self._wait(k)
        sU, su0 = self.snap[k]
        sU.copy_(U)
        su0.copy_(u0)
        oU, ou0 = self.out[k]
        d = self.dist
        if self.nccl:
            self.work[k] = (d.all_gather_into_tensor(oU, sU, group=self.group, async_op=True),
                            d.all_gather_into_tensor(ou0, su0, group=self.group, async_op=True))
        else:  # gloo has no all_gather_into_tensor
            self.work[k] = (d.all_gather(list(oU.chunk(self.world)), sU, group=self.group, async_op=True),
                            d.all_gather(list(ou0.chunk(self.world)), su0, group=self.group, async_op=True))
        self.n += 1
        return k

    def _wait(self, k: int) -> None:
        if self.work[k] is not None:
            for w in self.work[k]:
                w.wait()
            self.work[k] = None

    def drain(self) -> None:
        for k in range(self.depth):
            self._wait(k)

    def result(self, k: int):
        self._wait(k)
        return self.out[k]
