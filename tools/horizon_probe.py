"""Diagnostic: rollout time per launch vs the horizon H, to split a launch into its fixed cost (start-up, epilogue)
and its per-step cost.  python tools/horizon_probe.py [--B=8] [--cartpole | --quad] [--ramp]
  default: config #4's shape (B solves x K=1024, CA, bf16); --cartpole: config #2 (K=4096, analytic, fused epilogue);
  --quad: config #3's shape (K=2048, the quadruped MLPStatePredictor(37, 12, 128, 2), seeded weights, quad_est cost);
  --ramp: 150 ms of untimed solves before each horizon's measured ones (the GPU clock ramp, as bench.py)"""
import time
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "humanoid_mppi-rl_amd")]
import mppi_hip  # noqa: E402

sd = mppi_hip.load_npz(os.path.join(REPO, "tests", "golden", "ca_humanoid_weights.npz"))
x0_all = np.load(os.path.join(REPO, "tests", "golden", "g5_ca_humanoid_fwd.npz"))["x0_stride20"]
dev = torch.device("cuda", 0)
B = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--B=")), 8))
rows = []
for H in (1, 2, 4, 8, 16, 32, 64, 128):
    if "--quad" in sys.argv:
        from mppi_hip.nets import mlp_blob, synthetic_mlp
        cfg = mppi_hip.Config.preset("quad_est", K=2048, H=H, precision=1, max_batch=B)
        eng = mppi_hip.Engine(cfg, device=0).load_dynamics(*mlp_blob(synthetic_mlp(37, 12, seed=0), 37, 12))
        eng.set_cost("quad_est")
        x0 = torch.zeros(B, 37, dtype=torch.float32, device=dev)
        U = torch.zeros(B, 12, H, device=dev)
    elif "--cartpole" in sys.argv:
        cfg = mppi_hip.Config.preset("cartpole_py", K=4096, H=H, precision=0, max_batch=B)
        eng = mppi_hip.Engine(cfg, device=0).load_dynamics(1).set_cost("cartpole")
        x0 = torch.tensor([[0.0, np.pi, 0.0, 0.0]] * B, dtype=torch.float32, device=dev)
        U = torch.zeros(B, 1, H, device=dev)
    else:
        cfg = mppi_hip.Config.preset("humanoid_v3", K=1024, H=H, precision=1, max_batch=B)
        eng = mppi_hip.Engine(cfg, device=0).load_dynamics(*mppi_hip.cross_attention_blob(sd)).set_cost("humanoid_v3")
        x0 = torch.from_numpy(np.ascontiguousarray(x0_all[np.arange(B) % len(x0_all)], np.float32)).to(dev)
        U = torch.zeros(B, 21, H, device=dev)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    if "--ramp" in sys.argv:
        t_end = time.perf_counter() + 0.15
        while time.perf_counter() < t_end:
            for _ in range(8):
                eng.solve_device(B, x0.data_ptr(), U.data_ptr(), None, seed=1, shift=True, seed_counter=True)
            torch.cuda.synchronize()
    for i in range(24):
        if i == 4:
            torch.cuda.synchronize()
            eng.profile(True)
            eng.kernel_clock(True)
        eng.solve_device(B, x0.data_ptr(), U.data_ptr(), None, seed=1, shift=True, seed_counter=True)
    torch.cuda.synchronize()
    eng.profile(False)
    n, ms = eng.kernel_time("rollout")
    nc, us, _ = eng.kernel_clock_read()
    rows.append((H, us / nc, 1e3 * ms / n))
    print(f"H={H:4d} rollout clock {us / nc:8.1f} us  events {1e3 * ms / n:8.1f} us", flush=True)
    eng.close()
h = np.array([r[0] for r in rows], float)
t = np.array([r[1] for r in rows])
sl, ic = np.polyfit(h[h >= 8], t[h >= 8], 1)
print(f"fit H>=8: {ic:.1f} us + {sl:.3f} us/step")
