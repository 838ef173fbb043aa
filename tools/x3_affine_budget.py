"""Error budget of the affine (state-exchange-free) form of the split CA M-split rollout, CPU emulation against the fp32
oracle (test infrastructure, like oracle/: nothing in the product imports it).

The CA surrogate's dynamics ignore the controls (oracle/nets_ref.py ca_fold), and its LayerNorm-folded layer 0 is
linear in the state: g_t = W0 x_t + b0.  With x_{t+1} = x_t + W2 a1_t + b2, the layer-0 pre-activation can be carried
instead of recomputed from the state:  g_{t+1} = g_t + M a1_t + c,  M = W0 W2 (256 x 128),  c = W0 b2,
which removes the state -> layer-0 exchange from the per-step chain.  Schemes (config #4's 64 logged states, H = 64,
K = 1; costs against the fp32 oracle's):
    f16      the fp16 form as the kernels run it: layer 0 fp16 W hi + lo against the state rounded to fp16 every step
    affine1  g carried in fp32, M as ONE fp16 product (g_0 as in f16), layers 1 / 2 as in f16
    affine2  the same with M as fp16 hi + lo
    python tools/x3_affine_budget.py f16 affine1 affine2"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "humanoid_mppi-rl_amd"), os.path.join(REPO, "tests")]
from conftest import golden, golden_sd  # noqa: E402
from oracle import mppi_ref as R, nets_ref as N  # noqa: E402

NX, NU, H = 55, 21, int(os.environ.get("EB_H", "64"))


def f16(a):
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float64)


def split16(W):
    h = f16(W)
    return h, f16(np.asarray(W, np.float64) - h)


def mm(a, W, terms):  # a [n, k] @ W.T, fp16 operands as named, fp32 accumulate emulated by float64 -> fp32
    a16 = f16(a)
    if terms == 1:
        r = a16 @ f16(W).T
    else:
        Wh, Wl = split16(W)
        r = a16 @ (Wh + Wl).T
    return r.astype(np.float32)


stack = N.ln_fold(N.ca_fold(golden_sd("ca_humanoid_weights.npz"), 28, 27, 21))
L0, L1, L2 = stack
W0x = np.asarray(L0["W"], np.float64)[:, :NX]  # control columns are 0 (ca_fold)
assert not np.any(np.asarray(L0["W"])[:, NX:]), "the affine form needs a control-free layer 0"
b0 = np.asarray(L0["b"], np.float32)
betap = np.asarray(L0["lnfold"], np.float32)
W1, b1 = np.asarray(L1["W"], np.float64), np.asarray(L1["b"], np.float32)
W2, b2 = np.asarray(L2["W"], np.float64)[:NX], np.asarray(L2["b"], np.float32)[:NX]
M = W0x @ W2
c = (W0x @ np.asarray(b2, np.float64)).astype(np.float32)


def make_dyn(scheme):
    st = {}

    def dyn(x, u):
        x = np.asarray(x, np.float32)
        if scheme == "f16" or "g" not in st:
            g = mm(x, W0x, 2) + b0
        else:
            g = st["g"]
        q = (g * g).mean(axis=-1, keepdims=True, dtype=np.float32)
        a0 = np.maximum(g * (np.float32(1.0) / np.sqrt(q + np.float32(1e-5))) + betap, 0).astype(np.float32)
        z = np.maximum(mm(a0, W1, 1) + b1, 0).astype(np.float32)
        dx = mm(z, W2, 2) + b2
        if scheme.startswith("affine"):
            st["g"] = (g + (mm(z, M, 1 if scheme == "affine1" else 2) + c)).astype(np.float32)
        return (x + dx).astype(np.float32)
    return dyn


def ctx(b):
    return R.humanoid_context(swing_foot_x=-0.2 + 0.1 * b, swing_knee_x=0.05 * b, swing_vx=0.3 - 0.05 * b,
                              foot_clearance=0.01 * b, leg_clearance=-0.02 if b % 2 else 0.1)


x0s = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"].astype(np.float32)
pre = R.Preset("aff", K=1, H=H, lam=1.0, sigma=0.75)
rs = np.random.RandomState(44)
U0 = (0.1 * rs.randn(64, NU, H)).astype(np.float32)
noise = (0.75 * rs.randn(64, NU, H, 1)).astype(np.float32)
ref = np.array([R.rollout(pre, N.learned_dynamics(stack, NX, precision="fp32"), R.humanoid_v3_cost, x0s[b], U0[b],
                          noise[b], ctx=ctx(b % 8), dtype=np.float32) for b in range(64)])
for s in sys.argv[1:]:
    got = np.array([R.rollout(pre, make_dyn(s), R.humanoid_v3_cost, x0s[b], U0[b], noise[b], ctx=ctx(b % 8),
                              dtype=np.float32) for b in range(64)])
    rel = np.abs(got - ref) / np.abs(ref)
    print(f"ca {s:10s} H={H} max rel {rel.max():.2e}  p99 {np.quantile(rel, 0.99):.2e}  med {np.median(rel):.2e}",
          flush=True)
