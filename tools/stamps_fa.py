"""Diagnostic: per-phase cycle shares of the FA rollout horizon loop (diagnostic stamps build only).

    MPPI_STAMPS=1 python humanoid_mppi-rl_amd/build.py && python tools/stamps_fa.py [--cartpole]   (cartpole: the small-net kernel unless MPPI_FA_SMALL=0)
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

if "--cartpole" in sys.argv:
    sd = mppi_hip.load_npz(os.path.join(REPO, "tests", "golden", "fa_cartpole_weights.npz"))
    nx, nu, D, K, H, cost = 4, 1, 64, 2048, 20, "cartpole_est"
    cfg = mppi_hip.Config.preset("cartpole_est", K=K, H=H, precision=1)
else:
    sd = mppi_hip.synthetic_feature_attention(37, 12, 512, seed=0)
    nx, nu, D, K, H, cost = 37, 12, 512, 512, 4, "quad_est"
    cfg = mppi_hip.Config.preset("quad_est", K=K, H=H, precision=1)
eng = mppi_hip.Engine(cfg).load_dynamics(*mppi_hip.feature_attention_blob(sd, nx, nu, D)).set_cost(cost)
x0 = np.zeros(nx, np.float32)
lib = L.load()
lib.mppi_debug_fa_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
st = (ctypes.c_ulonglong * 8)()
eng.solve(x0, np.zeros((nu, H)), seed=1)
lib.mppi_debug_fa_stamps(st, 1)
runs = 2
for r in range(runs):
    eng.solve(x0, np.zeros((nu, H)), seed=r)
lib.mppi_debug_fa_stamps(st, 1)
if "--cartpole" in sys.argv and os.environ.get("MPPI_FA_SMALL", "1") != "0":  # fa_small_kernel's segments
    names = ["encoding", "LN1 + QKV + attention + out-proj", "out-proj exchange", "LN2 + FFN1 + FFN2",
             "FFN2 exchange", "output + state + cost", "controls", "(unused)"]
else:
    names = ["controls + encoding", "LayerNorm (x2 per layer)", "Q|K|V GEMM + store", "attention (VALU)",
             "out-proj GEMM", "FFN1 GEMM + ReLU + store", "FFN2 GEMM", "output + state + cost"]
tot = sum(st[i] for i in range(8))
for i in range(8):
    print(f"{names[i]:28s} {100 * st[i] / tot:5.1f}%")
