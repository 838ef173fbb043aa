"""Diagnostic: fc rollout time per launch vs the number of 16-sample groups per CU (B solves of K=1024, H=64),
to separate the per-group latency chain from shared-SIMD throughput.  python tools/occupancy_probe.py"""
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
for B in (1, 2, 4, 8, 12, 16):
    cfg = mppi_hip.Config.preset("humanoid_v3", K=1024, H=64, precision=1, max_batch=B)
    eng = mppi_hip.Engine(cfg, device=0).load_dynamics(*mppi_hip.cross_attention_blob(sd)).set_cost("humanoid_v3")
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    x0 = torch.from_numpy(np.ascontiguousarray(x0_all[np.arange(B) % len(x0_all)], np.float32)).to(dev)
    U = torch.zeros(B, 21, 64, device=dev)
    for i in range(24):
        if i == 4:
            torch.cuda.synchronize()
            eng.profile(True)
        eng.solve_device(B, x0.data_ptr(), U.data_ptr(), None, seed=1, shift=True)
    torch.cuda.synchronize()
    eng.profile(False)
    n, ms = eng.kernel_time("rollout")
    print(f"B={B:2d} groups/CU={B * 64 / 256:5.2f} rollout {1e3 * ms / n:7.1f} us")
    eng.close()
