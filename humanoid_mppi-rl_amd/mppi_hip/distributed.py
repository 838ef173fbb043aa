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


def control_buffers(B: int, nu: int, H: int, device=None):
    """(flat, U, u0): the nominal sequences U [B, nu, H] and the applied controls u0 [B, nu] as contiguous views of
    ONE flat fp32 buffer, so a step's controls are snapshotted with one copy and gathered with one collective."""
    import torch

    flat = torch.zeros(B * nu * H + B * nu, dtype=torch.float32, device=device)
    return flat, flat[:B * nu * H].view(B, nu, H), flat[B * nu * H:].view(B, nu)


def _flat_parent(U, u0):
    """The flat buffer U and u0 were cut from by control_buffers(), or None if they are separate tensors."""
    if U.dtype != u0.dtype or not (U.is_contiguous() and u0.is_contiguous()):
        return None
    if U.untyped_storage().data_ptr() != u0.untyped_storage().data_ptr():
        return None
    if u0.data_ptr() != U.data_ptr() + U.numel() * U.element_size():
        return None
    return U.as_strided((U.numel() + u0.numel(),), (1,), U.storage_offset())


class ControlGatherer:
    """Pipelined all-gather of each step's reduced controls for a stream of solves (bench.py's timed loop).

    submit(U, u0) snapshots the rank's controls on the current (compute) stream; the collective runs asynchronously
    (RCCL runs it on its own stream), so it overlaps the following solves, which update U in place. When U and u0 are
    views of one flat buffer (control_buffers) a step costs one copy; otherwise two.
    every = m batches the collective: the snapshots of m consecutive steps go side by side into one slot and ONE
    all-gather moves them (each step's controls are still snapshotted at its own step and gathered, up to m - 1
    steps later). Each all-gather carries a fixed GPU cost beside the solves, ~6 us at world 1 on config #4
    (scripts/gather_probe.py), which m amortises.
    Slots rotate over `depth`; a slot is reused only after its gather has completed: every `depth` collectives the
    compute stream is ordered behind the NEWEST gather (work.wait(), a stream-level wait), and collectives complete
    in order on RCCL's stream, so every slot's previous gather is complete before its snapshots are overwritten.
    Per-submit completion queries (is_completed) cost the host ~40 us each on ROCm and a stream-level wait per submit
    ~6 us of GPU time (scripts/gather_probe.py); one wait per ring turn costs neither.
    drain() launches a partly filled batch (a collective: every rank calls it at the same point) and waits for all.
    result(h) is the gathered (U_all [world*per, nu, H], u0_all [world*per, nu]) of the submit that returned h.
    reserve() / commit() split submit for producers that write the snapshot place themselves (no copy).
    """

    def __init__(self, U, u0, group=None, depth: int = 8, flat=None, every: int = 1):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.nccl = dist.get_backend(group) != "gloo"
        self.depth = depth
        self.every = max(1, int(every))
        self.shapeU, self.shapeu0 = tuple(U.shape), tuple(u0.shape)
        # flat: the buffer control_buffers() cut U and u0 from (its plain contiguous form copies fastest)
        self.flat = flat if flat is not None else _flat_parent(U, u0)
        self.fused = self.flat is not None
        self.parts = [U.numel() + u0.numel()] if self.fused else [U.numel(), u0.numel()]
        self.snap = [[U.new_empty(self.every * n) for n in self.parts] for _ in range(depth)]
        self.out = [[U.new_empty(self.world * self.every * n) for n in self.parts] for _ in range(depth)]
        self.work = [None] * depth
        self.last = None  # the newest collective's works
        self.nb = 0       # batches launched
        self.fill = 0     # snapshots in the current (unlaunched) batch

    def _launch(self) -> None:
        k = self.nb % self.depth
        d = self.dist
        works = []
        for snap, out in zip(self.snap[k], self.out[k]):
            if self.nccl:
                works.append(d.all_gather_into_tensor(out, snap, group=self.group, async_op=True))
            else:  # gloo has no all_gather_into_tensor
                works.append(d.all_gather(list(out.chunk(self.world)), snap, group=self.group, async_op=True))
        self.work[k] = works
        self.last = works
        self.nb += 1
        self.fill = 0

    def _slot(self):
        k, j = self.nb % self.depth, self.fill
        if j == 0 and not self.nccl:
            # gloo runs async work on a pool of threads, so collectives may complete out of order: wait for the
            # one that last read THIS slot before overwriting its snapshot (a host wait; costs nothing extra there)
            self._wait(k)
        elif k == 0 and j == 0 and self.last is not None:  # NCCL/RCCL: once per ring turn (see the class doc)
            for w in self.last:
                w.wait()
        return k, j

    def submit(self, U, u0) -> int:
        k, j = self._slot()
        srcs = [self.flat] if self.fused else [U.reshape(-1), u0.reshape(-1)]
        for src, snap, n in zip(srcs, self.snap[k], self.parts):
            snap[j * n:(j + 1) * n].copy_(src)
        return self.commit()

    def reserve(self):
        """(handle, U_view, u0_view): this step's snapshot place in the current slot, for a producer that writes it
        itself (an Engine solve with MPPI_FLAG_RESIDENT_U writes the updated U and u0 there from its update kernel,
        so the step needs no copy launch).  Enqueue the producer on the current stream, then call commit().
        Fused layout only (control_buffers)."""
        if not self.fused:
            raise ValueError("ControlGatherer.reserve needs U and u0 cut from one flat buffer (control_buffers)")
        k, j = self._slot()
        n = self.parts[0]
        view = self.snap[k][0][j * n:(j + 1) * n]
        nU = 1
        for d in self.shapeU:
            nU *= d
        return k * self.every + j, view[:nU].view(self.shapeU), view[nU:].view(self.shapeu0)

    def commit(self) -> int:
        """Close this step's snapshot (after submit's copy or a reserve()d producer); launches the batch when full."""
        h = (self.nb % self.depth) * self.every + self.fill
        self.fill += 1
        if self.fill == self.every:
            self._launch()
        return h

    def _wait(self, k: int) -> None:
        if self.work[k] is not None:
            for w in self.work[k]:
                w.wait()
            self.work[k] = None

    def drain(self) -> None:
        if self.fill:
            self._launch()
        for k in range(self.depth):
            self._wait(k)

    def result(self, h: int):
        """The gathered controls of step handle h (every rank's rows).  A local read: h's batch must have been
        launched (a full batch launches itself; drain(), a collective every rank calls at the same point, launches a
        partial one) -- launching it here would hide a collective inside a read that ranks may reach at different
        points."""
        k, j = divmod(h, self.every)
        if self.fill and k == self.nb % self.depth:  # its batch is still being filled
            raise RuntimeError("ControlGatherer.result: the batch of this step is not launched yet; call drain() "
                               "(collective) on every rank first")
        self._wait(k)
        nU = 1
        for s in self.shapeU:
            nU *= s
        rowsU = (self.world * self.shapeU[0],) + self.shapeU[1:]
        rowsu0 = (self.world * self.shapeu0[0],) + self.shapeu0[1:]
        if self.fused:
            per = self.out[k][0].view(self.world, self.every, -1)[:, j]
            return per[:, :nU].reshape(rowsU), per[:, nU:].reshape(rowsu0)
        oU = self.out[k][0].view(self.world, self.every, -1)[:, j]
        ou0 = self.out[k][1].view(self.world, self.every, -1)[:, j]
        return oU.reshape(rowsU), ou0.reshape(rowsu0)


# ---------------------------------------------------------------------------------------------- K-sharded solve
def combine_k_shards(costs: np.ndarray, dU_r: np.ndarray, lam: float, norm_eps: float = 0.0, group=None) -> np.ndarray:
    """The second mode of SURVEY 8e: ONE solve's K samples split over ranks.  Each rank's shard gives its costs and
    dU_r, its own softmin-weighted noise sum normalised by its own weights (an engine with a replace-mode update and
    no clamp or shift returns exactly that as U).  Two collectives combine the shards exactly (online softmin):
    allreduce(MIN) of beta_r = min_k c_k, then allreduce(SUM) of [f_r S_r, f_r P_r] with S_r = sum_k
    exp(-(c_k - beta_r)/lam), P_r = dU_r (S_r + eps) and f_r = exp(-(beta_r - beta)/lam), so that
    dU = sum_r f_r P_r / (sum_r f_r S_r + eps) = sum_k w_k eps_k / (sum_k w_k + eps) over all K
    (src/cartpole_mppi.py:92-98, src/mppi.jl:87-94).  Returns dU [nu, H] (float64), identical on every rank.

    Non-finite costs get weight 0, as in the engine.  A shard with no finite cost contributes
    S_r = 0 and P_r = 0 without reading its dU_r (an engine reports such a solve as MPPI_E_NONFINITE and its dU_r
    is undefined, e.g. NaN), so the combine equals the unsharded solve over the finite samples.  If no rank has a
    finite cost every rank raises ValueError after the MIN allreduce (collectively, so no rank is left waiting)."""
    import torch
    import torch.distributed as dist

    c = np.asarray(costs, np.float64)
    fin = np.isfinite(c)
    shape = np.shape(dU_r)
    if fin.any():
        beta_r = float(c[fin].min())
        S_r = float(np.exp(-(c[fin] - beta_r) / lam).sum())
        P_r = np.asarray(dU_r, np.float64) * (S_r + norm_eps)
    else:
        beta_r, S_r, P_r = float("inf"), 0.0, np.zeros(shape, np.float64)
    b = torch.tensor([beta_r], dtype=torch.float64)
    dist.all_reduce(b, op=dist.ReduceOp.MIN, group=group)
    beta = float(b.item())
    if not np.isfinite(beta):
        raise ValueError("combine_k_shards: no shard has a finite cost (MPPI_E_NONFINITE on every rank)")
    f_r = float(np.exp(-(beta_r - beta) / lam)) if np.isfinite(beta_r) else 0.0
    buf = torch.from_numpy(np.concatenate([[f_r * S_r], f_r * P_r.ravel()]))
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    buf = buf.numpy()
    return buf[1:].reshape(P_r.shape) / (buf[0] + norm_eps)


def solve_k_sharded(solve_shard: Callable, x0: np.ndarray, U: np.ndarray, lam: float, update: str = "add",
                    U_clamp: float = 0.0, norm_eps: float = 0.0, shift_fill: float | None = None, group=None):
    """One MPPI solve whose K samples are spread over the ranks (each rank draws its own K/world samples).

    solve_shard(x0, U) -> (costs [K_r], dU_r [nu, H]) runs this rank's shard (e.g. Engine.solve on an engine created
    with update_mode = replace, no U clamp, no shift, and a rank-specific seed).  Then the exact combine above, and
    the update of the reference controller on the combined dU: add or replace, clamp, u0 = U[:, 0], and the shift
    when shift_fill is given (src/cartpole_mppi.py:96-106, src/mppi.jl:91-98).  Returns (U_new, u0)."""
    costs, dU_r = solve_shard(x0, U)
    dU = combine_k_shards(costs, dU_r, lam, norm_eps, group)
    Un = dU if update == "replace" else np.asarray(U, np.float64) + dU
    if U_clamp > 0:
        Un = np.clip(Un, -U_clamp, U_clamp)
    u0 = Un[:, 0].copy()
    if shift_fill is not None:
        Us = Un.copy()
        Us[:, :-1] = Un[:, 1:]
        Us[:, -1] = shift_fill * Us[:, -2]
        Un = Us
    return Un, u0
