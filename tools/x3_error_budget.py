"""Error budget of the split-bf16 (MPPI_PREC_BF16X3) products, CPU emulation against the fp32 oracle (test infrastructure,
like oracle/: nothing in the product imports it).  Every layer of the folded humanoid CA (or the humanoid MLP) computed
with its operands split as named, fp32 accumulation emulated; the H = 64 running costs compared with the fp32 oracle's:
    python tools/x3_error_budget.py ca fp32 bf16x3 bf16x1 bf16x2w bf16x2a bf16x3,bf16x3,bf16x2w ...
schemes per layer (comma list = one per layer): fp32 | bf16x3 (W_lo a_hi + W_hi a_lo + W_hi a_hi, the kernels') |
bf16x2w (W hi + lo, a hi only) | bf16x2a (a hi + lo, W hi only) | bf16x1 (one bf16 product) | f16* (fp16 pairs).
Used in round 5 to decide whether any layer can drop a term (profiles/r05_x3_error_budget.txt): none can at rtol 1e-4."""
import sys, os, numpy as np
SCALE_TOP = int(os.environ.get("SCALE_TOP", "13"))
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "humanoid_mppi-rl_amd"), os.path.join(REPO, "tests")]
from conftest import golden, golden_sd
from oracle import mppi_ref as R, nets_ref as N
from oracle.mppi_ref import bf16_round

def split_bf(a):
    a = np.asarray(a, np.float32)
    h = bf16_round(a); l = bf16_round(a - h)
    return h.astype(np.float64), l.astype(np.float64)

FTZ = os.environ.get("FTZ", "0") == "1"
def ftz(v):
    return np.where(np.abs(v) < 2.0 ** -14, 0.0, v) if FTZ else v
def split_f16(a):
    a = np.asarray(a, np.float32)
    if FTZ:
        h = a.astype(np.float16).astype(np.float32); l = (a - h).astype(np.float16).astype(np.float64)
        return ftz(h.astype(np.float64)), ftz(l)
    h = a.astype(np.float16).astype(np.float32); l = (a - h).astype(np.float16)
    return h.astype(np.float64), l.astype(np.float64)

def mm(a, W, scheme):
    """a [n, k] @ W.T [k, m], operands as `scheme`, fp32 accumulate emulated by float64 sum -> fp32."""
    if scheme == "fp32":
        return (np.asarray(a, np.float32) @ np.asarray(W, np.float32).T).astype(np.float32)
    kind, terms = scheme.split("x") if "x" in scheme else (scheme, "1")
    sp = split_bf if kind == "bf16" else split_f16
    sw = 1.0
    if kind == "f16s":  # W scaled by a power of 2 so that max |W| is in [2^13, 2^14)
        sw = 2.0 ** (SCALE_TOP - np.floor(np.log2(np.abs(W).max())))
    Wh, Wl = sp(np.asarray(W, np.float64) * sw); ah, al = sp(a)
    Wh /= sw; Wl /= sw
    if terms == "1":
        r = ah @ Wh.T
    elif terms == "3":
        r = ah @ Wh.T + al @ Wh.T + ah @ Wl.T
    elif terms == "2w":   # W hi+lo, a single
        r = ah @ (Wh + Wl).T
    elif terms in ("2wq", "2wv"):  # W hi+lo on the qpos (first 28) / qvel (from 28) input columns only, hi elsewhere
        Wm = Wh.copy()
        cols = slice(0, 28) if terms == "2wq" else slice(28, None)
        Wm[:, cols] += Wl[:, cols]
        r = ah @ Wm.T
    elif terms in ("2rq", "2rv"):  # W hi+lo on the qpos (first 28) / qvel (from 28) OUTPUT rows only, hi elsewhere
        Wm = Wh.copy()
        rows = slice(0, 28) if terms == "2rq" else slice(28, None)
        Wm[rows] += Wl[rows]
        r = ah @ Wm.T
    elif terms == "2a":   # a hi+lo, W single
        r = (ah + al) @ Wh.T
    else:
        raise ValueError(scheme)
    return r.astype(np.float32)

def fwd(stack, xin, schemes):
    h = np.asarray(xin, np.float32)
    for L, sc in zip(stack, schemes):
        h = mm(h, L["W"], sc) + np.asarray(L["b"], np.float32)
        if L["ln"] is not None:
            g, b = (np.asarray(a, np.float32) for a in L["ln"])
            mu = h.mean(axis=-1, keepdims=True, dtype=np.float32); d = h - mu
            var = (d * d).mean(axis=-1, keepdims=True, dtype=np.float32)
            h = d * (1.0 / np.sqrt(var + np.float32(1e-5))) * g + b
        if L["relu"]:
            h = np.maximum(h, 0).astype(np.float32)
    return h

def dyn_for(stack, nx, schemes):
    def dyn(x, u):
        d = fwd(stack, np.concatenate([x, u], axis=-1), schemes)
        return (x + d[..., :nx]).astype(np.float32)
    return dyn

NX, NU, H = 55, 21, int(os.environ.get("EB_H", "64"))
x0s = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"].astype(np.float32)
def ctx(b):
    return R.humanoid_context(swing_foot_x=-0.2 + 0.1 * b, swing_knee_x=0.05 * b, swing_vx=0.3 - 0.05 * b,
                              foot_clearance=0.01 * b, leg_clearance=-0.02 if b % 2 else 0.1)
which = sys.argv[1]
schemes_list = sys.argv[2:]
if which == "ca":
    sd = golden_sd("ca_humanoid_weights.npz"); stack = N.ca_fold(sd, 28, 27, 21)
    K, B = int(os.environ.get("EB_K", "1")), 64
else:
    from mppi_hip.nets import synthetic_mlp
    sd = synthetic_mlp(NX, NU, seed=0); stack = N.mlp_stack(sd)
    K, B = 64, 16
pre = R.Preset("c4", K=K, H=H, lam=1.0, sigma=0.75)
rs = np.random.RandomState(44)
U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
ref = []
for b in range(B):
    ref.append(R.rollout(pre, dyn_for(stack, NX, ["fp32"] * len(stack)), R.humanoid_v3_cost, x0s[b % 64], U0[b], noise[b],
                         ctx=ctx(b % 8), dtype=np.float32))
ref = np.array(ref)
for s in schemes_list:
    sch = s.split(",")
    if len(sch) == 1: sch = sch * len(stack)
    got = np.array([R.rollout(pre, dyn_for(stack, NX, sch), R.humanoid_v3_cost, x0s[b % 64], U0[b], noise[b],
                              ctx=ctx(b % 8), dtype=np.float32) for b in range(B)])
    rel = np.abs(got - ref) / np.abs(ref)
    am = [int(np.argmin(got[b]) == np.argmin(ref[b])) for b in range(B)]
    print(f"{which} {s:28s} max rel {rel.max():.2e}  p99 {np.quantile(rel, 0.99):.2e}  med {np.median(rel):.2e}  argmin agree {sum(am)}/{B}", flush=True)
