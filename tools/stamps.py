"""Diagnostic: per-segment cycle shares of the fc rollout horizon loop (diagnostic stamps build only).

    MPPI_STAMPS=1 python humanoid_mppi-rl_amd/build.py && python tools/stamps.py [--mlp] [--fp32 | --x3] [--B=8]
(--x3: split bf16 on the M-split kernel, two 16-sample tiles per wave)
Read SHARES, not absolute time (the stamps' waits forbid overlaps the real kernel has)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MPPI_HIP_LIB"] = os.path.join(REPO, "humanoid_mppi-rl_amd", "lib", "libmppi_hip_stamps.so")
sys.path[:0] = [REPO, os.path.join(REPO, "humanoid_mppi-rl_amd")]
import mppi_hip  # noqa: E402
from mppi_hip import _lib as L  # noqa: E402

prec = 0 if "--fp32" in sys.argv else (2 if "--x3" in sys.argv else 1)
if prec == 2:
    os.environ["MPPI_X3_WAVE"] = "0"  # the M-split kernels (the stamps live in fc_rollout_body)
K, H, runs = 1024, 64, 5
B = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--B=")), 8))
if "--mlp" in sys.argv:
    cfg = mppi_hip.Config.preset("humanoid_v3", K=K, H=H, precision=prec, max_batch=B)
    eng = mppi_hip.Engine(cfg).load_dynamics(*mppi_hip.mlp_blob(mppi_hip.synthetic_mlp(55, 21), 55, 21))
else:
    sd = mppi_hip.load_npz(os.path.join(REPO, "tests", "golden", "ca_humanoid_weights.npz"))
    cfg = mppi_hip.Config.preset("humanoid_v3", K=K, H=H, precision=prec, max_batch=B)
    eng = mppi_hip.Engine(cfg).load_dynamics(*mppi_hip.cross_attention_blob(sd))
eng.set_cost("humanoid_v3")
x0 = np.load(os.path.join(REPO, "tests", "golden", "g5_ca_humanoid_fwd.npz"))["x0_stride20"][:B]
lib = L.load()
lib.mppi_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
st = (ctypes.c_ulonglong * 8)()
eng.solve(x0, np.zeros((B, 21, H)), seed=1)
lib.mppi_debug_stamps(st, 1)
for r in range(runs):
    eng.solve(x0, np.zeros((B, 21, H)), seed=r)
lib.mppi_debug_stamps(st, 1)
waves = 4 * B * ((K + 63) // 64 * 64) // 16 // (2 if prec == 2 else 1)  # 4 waves per 16-sample group (x3: 2 per wave)
names = ["loop top + u loads", "layer0 + LN stats", "LN barrier wait", "LN apply + act0 barrier",
         "layer1 (+layer2) + barriers", "last layer + x barrier", "ring cost (every 16 steps)", "-"]
tot = sum(st[i] for i in range(7))
for i in range(7):
    print(f"{names[i]:24s} {st[i] / (waves * runs * H):9.0f} cyc/step/wave  {100 * st[i] / tot:5.1f}%")
print(f"total {tot / (waves * runs * H):.0f} cycles per step per wave")
