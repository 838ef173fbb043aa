"""Multi-rank path on CPU: world_size 2 (and 3, uneven) over gloo, 127.0.0.1.

The ranks shard the initial states, solve their shard with an oracle-backed stand-in for the engine (the
engine itself needs a GPU; its per-solve results are covered by the -m gpu parity tests) and all-gather the
reduced controls. The gathered result must equal the single-process solve of all states, bitwise."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mppi_hip.distributed import pad_shard, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_solve_local(x0, U):
    """Stand-in for Engine.solve(shift=True): oracle cartpole solve with per-state seeded reference noise."""
    from oracle import mppi_ref as R
    pre = R.Preset("t", K=32, H=U.shape[2], lam=1.0, sigma=1.0)
    U_new, u0 = np.empty_like(U), np.empty((U.shape[0], U.shape[1]))
    for i in range(x0.shape[0]):
        seed = int(abs(x0[i, 1]) * 1000) % 1000  # noise keyed by the state, not by the rank
        noise = R.reference_noise(seed, 1, U.shape[2], 32, 1.0)
        out = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0[i], U[i], noise)
        u0[i], U_new[i] = out["u0"], out["U_shifted"]
    return U_new, u0


def _worker(rank, world, port, x0_all, U_all, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "humanoid_mppi-rl_amd")]
    import torch.distributed as dist
    from mppi_hip.distributed import solve_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = solve_sharded(x0_all, U_all, _oracle_solve_local, rank, world)
        q.put((rank, res.U.numpy(), res.u0.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 8), (3, 7)])
def test_sharded_solve_gathers_full_controls(world, n):
    rs = np.random.RandomState(0)
    x0_all = np.stack([[0.0, 0.1 * i + 0.05, 0.0, 0.0] for i in range(n)])
    U_all = 0.1 * rs.randn(n, 1, 12)
    ref_U, ref_u0 = _oracle_solve_local(x0_all, U_all)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, x0_all, U_all, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, U, u0 in outs:
        np.testing.assert_array_equal(U, ref_U.astype(np.float32))
        np.testing.assert_array_equal(u0, ref_u0.astype(np.float32))


def test_shard_bounds_cover_everything_once():
    for n in (1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                a, b, per = shard_bounds(n, r, world)
                assert b - a <= per
                seen += list(range(a, b))
            assert seen == list(range(n))
    x = np.arange(6).reshape(3, 2)
    assert pad_shard(x, 5).shape == (5, 2) and (pad_shard(x, 5)[-1] == x[-1]).all()
    assert pad_shard(x[:0], 2).shape == (2, 2)


def _gather_worker(rank, world, port, q, fused, every=1, reserve=False):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "humanoid_mppi-rl_amd")]
    import torch
    import torch.distributed as dist
    from mppi_hip.distributed import ControlGatherer, control_buffers
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if fused:  # U, u0 views of one flat buffer: one copy + one collective per step
            _, U, u0 = control_buffers(3, 2, 5)
        else:
            U, u0 = torch.zeros(3, 2, 5), torch.zeros(3, 2)
        g = ControlGatherer(U, u0, depth=2, every=every)
        assert g.fused == fused
        slots = []
        for step in range(4):  # the "solve" updates U in place right after each submit
            if reserve:  # the producer writes its snapshot place itself, then commits
                h, Us, u0s = g.reserve()
                Us.fill_(100 * step + rank)
                u0s.fill_(-(100 * step + rank))
                assert g.commit() == h
                slots.append(h)
            else:
                U.fill_(100 * step + rank)
                u0.fill_(-(100 * step + rank))
                slots.append(g.submit(U, u0))
            U.fill_(-1.0)  # next step's in-place update must not leak into the gathered snapshot
        g.drain()
        # the last depth submits are still readable from their slots
        out = [tuple(t.clone().numpy() for t in g.result(k)) for k in slots[-2:]]
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fused,every,reserve", [(False, 1, False), (True, 1, False), (False, 3, False),
                                                 (True, 3, False), (True, 1, True), (True, 3, True)])
def test_pipelined_control_gather(fused, every, reserve):
    """ControlGatherer (bench.py's overlapped all-gather): each step's snapshot is gathered intact although U is
    overwritten right after submit; results rotate over 2 slots.  every = 3: the 4 steps' snapshots go out as one
    full batch of 3 and a partial batch of 1 (launched by drain), and each step's result is still its own.
    reserve: the step's snapshot place is written directly (the engine's RESIDENT_U mirror), then committed."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q, fused, every, reserve)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        for step, (Ug, u0g) in zip((2, 3), res[r]):
            want = np.concatenate([np.full((3, 2, 5), 100 * step + k, np.float32) for k in range(world)])
            np.testing.assert_array_equal(Ug, want)
            np.testing.assert_array_equal(u0g, -want[:, :, 0])


def _kshard_worker(rank, world, port, x0, U0, noise, q, dead=()):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "humanoid_mppi-rl_amd")]
    import torch.distributed as dist
    from mppi_hip.distributed import solve_k_sharded
    from oracle import mppi_ref as R
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        K = noise.shape[2]
        lo, hi = rank * K // world, (rank + 1) * K // world  # this rank's samples

        def shard(x, U):  # oracle stand-in for a replace-mode, unclamped, unshifted engine solve of the shard
            if rank in dead:  # every cost non-finite: the engine reports MPPI_E_NONFINITE, its dU_r is undefined
                return np.full(hi - lo, np.inf), np.full(U.shape, np.nan)
            pre = R.Preset("s", K=hi - lo, H=U.shape[1], lam=0.5, sigma=1.0, update="replace")
            out = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x, U, noise[:, :, lo:hi])
            return out["costs"], out["U_new"]
        try:
            Un, u0 = solve_k_sharded(shard, x0, U0, lam=0.5, U_clamp=0.45, norm_eps=1e-10, shift_fill=0.1)
        except ValueError as e:
            q.put((rank, "ValueError", str(e)))
        else:
            q.put((rank, Un, u0))
    finally:
        dist.destroy_process_group()


def _run_kshard(world, x0, U0, noise, dead=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kshard_worker, args=(r, world, port, x0, U0, noise, q, dead)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return outs


@pytest.mark.parametrize("world,dead", [(2, ()), (3, ()), (2, (1,)), (3, (0, 2))])
def test_k_sharded_solve_equals_the_whole_solve(world, dead):
    """SURVEY 8e second mode: one solve's K samples over ranks; the two-collective online-softmin combine equals
    the single-process solve over all K samples (add update, clamp, eps normaliser, shift) to fp64 rounding.
    With `dead` ranks every cost of those shards is inf and their dU_r is NaN (an engine's MPPI_E_NONFINITE shard):
    those samples get weight 0, so the result equals the whole solve over the live shards' samples only."""
    from oracle import mppi_ref as R
    K, H = 90, 10
    noise = R.reference_noise(3, 1, H, K, 1.0)
    x0 = np.array([0.0, 0.3, 0.0, 0.0])
    U0 = 0.2 * np.sin(np.arange(H))[None, :]
    live = [k for r in range(world) if r not in dead for k in range(r * K // world, (r + 1) * K // world)]
    pre = R.Preset("w", K=len(live), H=H, lam=0.5, sigma=1.0, U_clamp=0.45, norm_eps=1e-10, shift_fill=0.1)
    ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0, U0, noise[:, :, live])
    for rank, Un, u0 in _run_kshard(world, x0, U0, noise, dead):
        assert np.isfinite(Un).all()
        np.testing.assert_allclose(u0, ref["u0"], rtol=0, atol=1e-10)
        np.testing.assert_allclose(Un, ref["U_shifted"], rtol=0, atol=1e-10)


def test_k_sharded_solve_without_any_finite_cost_raises_on_every_rank():
    """No shard has a finite cost: every rank raises ValueError (none is left waiting in a collective)."""
    from oracle import mppi_ref as R
    K, H = 40, 6
    noise = R.reference_noise(1, 1, H, K, 1.0)
    outs = _run_kshard(2, np.zeros(4), np.zeros((1, H)), noise, dead=(0, 1))
    assert sorted(r for r, kind, _ in outs) == [0, 1]
    assert all(kind == "ValueError" for _, kind, _ in outs)


def test_gather_result_of_an_unlaunched_batch_raises():
    """result() is a local read: on a batch still being filled it raises (the launch is a collective that every rank
    must reach at the same point: drain()), and after drain() it returns the step's controls."""
    import socket
    import torch
    import torch.distributed as dist
    from mppi_hip.distributed import ControlGatherer, control_buffers
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        _, U, u0 = control_buffers(2, 2, 3)
        g = ControlGatherer(U, u0, depth=2, every=3)
        U.fill_(7.0)
        u0.fill_(-7.0)
        h = g.submit(U, u0)
        with pytest.raises(RuntimeError):
            g.result(h)
        g.drain()
        Ug, u0g = g.result(h)
        assert torch.all(Ug == 7.0) and torch.all(u0g == -7.0)
    finally:
        dist.destroy_process_group()
