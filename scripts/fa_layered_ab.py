"""Config #3's FA hidden-512 solve (K = 2048, H = 40, quad_est, synthetic weights) timed per solve with HIP events
(mppi_profile): the fused fa_rollout_kernel, or with MPPI_FA_LAYERED=1 the layer-by-layer path."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "humanoid_mppi-rl_amd"))
import mppi_hip as M  # noqa: E402
from mppi_hip.nets import feature_attention_blob, synthetic_feature_attention  # noqa: E402

nx, nu, K, H = 37, 12, 2048, 40
sd = synthetic_feature_attention(nx, nu, 512, seed=0)
eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=10.0, sigma=0.4, precision=1, update_mode=1,
                        shift_fill=0.1, terminal_weight=10.0))
eng.load_dynamics(*feature_attention_blob(sd, nx, nu, 512)).set_cost("quad_est")
x0 = np.zeros(nx, np.float32)
x0[2], x0[3] = 0.35, 1.0
U0 = np.zeros((nu, H), np.float32)
eng.solve(x0, U0, seed=1)
eng.profile(True)
eng.kernel_clock(True)
n = int(os.environ.get("N", "5"))
t0 = time.perf_counter()
for i in range(n):
    res = eng.solve(x0, U0, seed=2 + i)
dt = (time.perf_counter() - t0) / n
k = {name: eng.kernel_time(name) for name in ("rollout", "reduce")}
kc = eng.kernel_clock_read()
print(f"layered={os.environ.get('MPPI_FA_LAYERED', '0')} wall {dt * 1e3:.2f} ms/solve; events {k}; rollout clock "
      f"{kc[0]} launches mean {kc[1] / max(kc[0], 1) / 1e3:.3f} ms; "
      f"cost mean {np.mean(res.costs):.4f} std {np.std(res.costs):.4f}", flush=True)
