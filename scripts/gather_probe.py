"""Diagnostic: what the per-step RCCL control gather costs on top of the captured solve (config #4), at world 1.

    python scripts/gather_probe.py [--chain]   (one GPU; RCCL process group of size 1; --chain: chained solves)

Variants (each 300 steps after 20 warm-ups): plain graph replay; + snapshot copy; + all-gather of the live buffer
(no snapshot; timing only); full ControlGatherer, also batched (every = 2, 4, 8 steps per collective).  Prints wall ms/step and the host's enqueue time per step.
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "humanoid_mppi-rl_amd")]


def main():
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    import mppi_hip
    from mppi_hip.distributed import ControlGatherer, control_buffers

    spec = bench.workload_spec("humanoid_ca", "bf16")
    cfg, B = spec["cfg"], spec["B"]
    eng = mppi_hip.Engine(cfg, device=0)
    eng.load_dynamics(*spec["dyn"]).set_cost(spec["cost"])
    stream = torch.cuda.current_stream(dev)
    eng.set_stream(stream.cuda_stream)
    x0 = torch.from_numpy(np.ascontiguousarray(spec["x0_all"][:B], np.float32)).to(dev)
    flat, U, u0 = control_buffers(B, cfg.nu, cfg.H, device=dev)
    chain = "--chain" in sys.argv  # bench.py's one-solve steps: chained stream launches instead of graph replays
    if not chain:
        eng.graph_capture(B, 1, x0.data_ptr(), U.data_ptr(), u0.data_ptr(), seed=0, env_step=False)

    def launch():
        if chain:
            eng.solve_device(B, x0.data_ptr(), U.data_ptr(), None, seed=0, u0_ptr=u0.data_ptr(), shift=True,
                             seed_counter=True, chain=True)
        else:
            eng.graph_launch(sync=False)
    snap = torch.empty_like(flat)
    out = torch.empty_like(flat)
    g = ControlGatherer(U, u0, flat=flat)
    g2 = ControlGatherer(U, u0, depth=2, flat=flat)
    gb = {m: ControlGatherer(U, u0, flat=flat, every=m) for m in (2, 4, 8)}
    snaps = [torch.empty_like(flat) for _ in range(8)]
    outs = [torch.empty_like(flat) for _ in range(8)]
    ctr = [0]

    def copy_gather(ring: int):
        k = ctr[0] % ring
        ctr[0] += 1
        snaps[k].copy_(flat)
        dist.all_gather_into_tensor(outs[k], snaps[k], async_op=True)

    works = [None] * 8

    def copy_gather_keep(check: bool):  # ControlGatherer's steps inline: keep the work, query it before reuse
        k = ctr[0] % 8
        ctr[0] += 1
        if check and works[k] is not None and not works[k].is_completed():
            works[k].wait()
        snaps[k].copy_(flat)
        works[k] = dist.all_gather_into_tensor(outs[k], snaps[k], async_op=True)

    variants = {
        "solve only": lambda: None,
        "+ snapshot copy": lambda: snap.copy_(flat),
        "+ all-gather (no snapshot)": lambda: dist.all_gather_into_tensor(out, flat, async_op=True),
        "+ all-gather sync (no snapshot)": lambda: dist.all_gather_into_tensor(out, flat),
        "+ copy + all-gather, 1 slot": lambda: copy_gather(1),
        "+ copy + all-gather, 8 slots": lambda: copy_gather(8),
        "+ copy + all-gather, keep works": lambda: copy_gather_keep(False),
        "+ copy + all-gather, keep + query": lambda: copy_gather_keep(True),
        "ControlGatherer depth 2": lambda: g2.submit(U, u0),
        "ControlGatherer depth 8": lambda: g.submit(U, u0),
        "ControlGatherer every 2": lambda: gb[2].submit(U, u0),
        "ControlGatherer every 4": lambda: gb[4].submit(U, u0),
        "ControlGatherer every 8": lambda: gb[8].submit(U, u0),
    }
    for name, extra in list(variants.items()) * 2:  # twice: run-to-run spread
        for _ in range(20):
            launch()
            extra()
        g.drain()
        g2.drain()
        for x in gb.values():
            x.drain()
        torch.cuda.synchronize()
        n = 300
        t0 = time.perf_counter()
        for _ in range(n):
            launch()
            extra()
        t_host = time.perf_counter() - t0
        g.drain()
        g2.drain()
        for x in gb.values():
            x.drain()
        torch.cuda.synchronize()
        t1 = time.perf_counter() - t0
        print(f"{name:34s} wall {t1 / n * 1e3:.4f} ms/step   host enqueue {t_host / n * 1e3:.4f} ms/step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
