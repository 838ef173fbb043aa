"""Probe: does splitting the 64 config-#4 solves over independent engines on separate HIP streams ("lanes") overlap one
lane's HBM-bound reduce_kernel<GEN> with another lane's latency-bound rollout?  Each lane is its own mppi_hip.Engine
(own device buffers, own stream) with 64/lanes solves, chained solves as in bench.py; a step = one solve of every lane.
Prints ms per step for lanes = 1, 2, 4 (same process, same box).  usage: python tools/lanes_probe.py [steps] [--offset]
--offset: lane j's stream starts with a spin of j / lanes of a step (torch.cuda._sleep), so the lanes' reduces fall
inside the other lanes' rollouts instead of all lanes running in phase.
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "humanoid_mppi-rl_amd"))
import bench  # noqa: E402  (workload_spec)
import mppi_hip  # noqa: E402


def run(lanes: int, steps: int, total: int = 64, prec: str = "bf16", offset: bool = False) -> float:
    dev = torch.device("cuda", 0)
    B = total // lanes
    engs, bufs, streams = [], [], []
    for j in range(lanes):
        spec = bench.workload_spec("humanoid_ca", prec, solves=B)
        e = mppi_hip.Engine(spec["cfg"], device=0)
        e.load_dynamics(*spec["dyn"]).set_cost(spec["cost"])
        s = torch.cuda.Stream(dev)
        e.set_stream(s.cuda_stream)
        rows = np.arange(j * B, (j + 1) * B) % spec["x0_all"].shape[0]
        x0 = torch.from_numpy(np.ascontiguousarray(spec["x0_all"][rows], np.float32)).to(dev)
        cfg = spec["cfg"]
        U = torch.zeros(B, cfg.nu, cfg.H, device=dev)
        u0 = torch.zeros(B, cfg.nu, device=dev)
        engs.append(e)
        bufs.append((x0, U, u0))
        streams.append(s)

    def step():
        for j, e in enumerate(engs):
            x0, U, u0 = bufs[j]
            e.solve_device(B, x0.data_ptr(), U.data_ptr(), None, seed=j << 40, u0_ptr=u0.data_ptr(), shift=True,
                           seed_counter=True, chain=True)

    if offset:  # one-time phase offset of lane j by j / lanes of a (~0.48 ms) step, on its own stream
        for j in range(1, lanes):
            with torch.cuda.stream(streams[j]):
                torch.cuda._sleep(int(2.4e9 * 0.48e-3 * j / lanes))
    for _ in range(200):  # clock ramp + warm-up
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    for e in engs:
        e.close() if hasattr(e, "close") else None
    return ms


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 100
    off = "--offset" in sys.argv
    only = [int(a.split("=")[1]) for a in sys.argv if a.startswith("--lanes=")]
    for prec in ("bf16",):
        for lanes in only or (1, 2, 4, 1, 2, 4):
            ms = run(lanes, steps, prec=prec, offset=off)
            print(f"{prec} lanes={lanes} solves/lane={64 // lanes} offset={off}: {ms:.4f} ms/step "
                  f"({64 * 1024 * 64 / ms * 1e3:.4g} trajectory-steps/s)", flush=True)
