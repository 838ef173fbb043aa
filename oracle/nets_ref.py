"""numpy restatement of the learned dynamics nets — TEST INFRASTRUCTURE ONLY.

Restates learning/model.py (reference SheffieldWang616/Humanoid_MPPI-RL) in eval mode (dropout off):
  * MLPStatePredictor              learning/model.py:6-46
  * FeatureAttentionStatePredictor learning/model.py:48-153
  * CrossAttentionStatePredictor   learning/model.py:157-202
and the algebraic folding the engine applies to the cross-attention net (exact in real arithmetic):
with one query and one key, nn.MultiheadAttention's softmax is identically 1, so
attn(q, kv) = W_o (W_v kv + b_v) + b_o, and the encoders/projections collapse into one Linear.
Pinned by tests/golden/g3,g5,g8 (outputs of the reference module imported in the build container).

State dicts are plain {torch-key: ndarray} maps (tests/golden/*_weights.npz).
"""
from __future__ import annotations

import numpy as np

from .mppi_ref import bf16_round


def _lin(x, W, b):
    return x @ W.T + b


def _layernorm(x, g, b, eps=1e-5):
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * g + b


def _relu(x):
    return np.maximum(x, 0)


# ---------------------------------------------------------------- MLP (learning/model.py:6-46)

def _mlp_modules(sd: dict) -> list:
    """The nn.Sequential of MLPStatePredictor in index order: ("linear", i) / ("bn", i) (Dropout / ReLU carry no
    parameters; with use_batch_norm=True a BatchNorm1d follows each hidden Linear, learning/model.py:24-39)."""
    mods = {}
    for k in sd:
        if not k.startswith("network."):
            continue
        i, par = int(k.split(".")[1]), k.split(".", 2)[2]
        if par == "running_mean":
            mods[i] = "bn"
        elif par == "weight" and np.ndim(sd[k]) == 2 and i not in mods:
            mods[i] = "linear"
    return [(mods[i], i) for i in sorted(mods)]


def mlp_forward(sd: dict, x: np.ndarray) -> np.ndarray:
    """MLPStatePredictor.forward in eval mode (dropout off; BatchNorm1d with its running statistics, eps 1e-5)."""
    mods = _mlp_modules(sd)
    nlin = sum(1 for m, _ in mods if m == "linear")
    h, seen = np.asarray(x, np.float64), 0
    for j, (m, i) in enumerate(mods):
        p = f"network.{i}."
        if m == "linear":
            h = _lin(h, sd[p + "weight"], sd[p + "bias"])
            seen += 1
        else:
            h = (h - sd[p + "running_mean"]) / np.sqrt(np.asarray(sd[p + "running_var"], np.float64) + 1e-5) * \
                sd[p + "weight"] + sd[p + "bias"]
        nxt = mods[j + 1][0] if j + 1 < len(mods) else None
        if seen < nlin and nxt != "bn":  # ReLU after every Linear (+ BatchNorm) but the last
            h = _relu(h)
    return h


def mlp_stack(sd: dict) -> list:
    """The fc stack of an MLPStatePredictor with every BatchNorm folded into the Linear before it (fp64), the form
    the engine evaluates (csrc/mppi_nets.cpp::mlp_layers)."""
    out = []
    for m, i in _mlp_modules(sd):
        p = f"network.{i}."
        if m == "linear":
            out.append(dict(W=np.asarray(sd[p + "weight"], np.float64), b=np.asarray(sd[p + "bias"], np.float64),
                            ln=None, relu=True))
        else:
            sc = np.asarray(sd[p + "weight"], np.float64) / np.sqrt(np.asarray(sd[p + "running_var"], np.float64) + 1e-5)
            out[-1]["W"] = out[-1]["W"] * sc[:, None]
            out[-1]["b"] = (out[-1]["b"] - np.asarray(sd[p + "running_mean"], np.float64)) * sc + \
                np.asarray(sd[p + "bias"], np.float64)
    out[-1]["relu"] = False
    return out


# ---------------------------------------------------- Cross attention (learning/model.py:157-202)

def _mha_single(q_in, kv_in, in_w, in_b, out_w, out_b, nheads):
    """nn.MultiheadAttention(batch_first) with L=S=1, restated head by head (learning/model.py:195-196)."""
    D = q_in.shape[-1]
    Wq, Wk, Wv = in_w[:D], in_w[D:2 * D], in_w[2 * D:]
    bq, bk, bv = in_b[:D], in_b[D:2 * D], in_b[2 * D:]
    q = _lin(q_in, Wq, bq)
    k = _lin(kv_in, Wk, bk)
    v = _lin(kv_in, Wv, bv)
    hd = D // nheads
    out = np.empty_like(v)
    for h in range(nheads):
        s = slice(h * hd, (h + 1) * hd)
        score = np.sum(q[..., s] * k[..., s], axis=-1, keepdims=True) / np.sqrt(hd)
        p = np.exp(score - score)  # softmax over the single key == 1
        out[..., s] = p * v[..., s]
    return _lin(out, out_w, out_b)


def ca_forward(sd: dict, x: np.ndarray, qpos_dim: int, qvel_dim: int, nheads: int = 4) -> np.ndarray:
    """CrossAttentionStatePredictor.forward (unfolded) — learning/model.py:183-202."""
    qpos = x[..., :qpos_dim]
    qvel = x[..., qpos_dim:qpos_dim + qvel_dim]
    qp = _lin(qpos, sd["qpos_encoder.weight"], sd["qpos_encoder.bias"])
    qv = _lin(qvel, sd["qvel_encoder.weight"], sd["qvel_encoder.bias"])
    a1 = _mha_single(qp, qv, sd["attn_qpos_to_qvel.in_proj_weight"], sd["attn_qpos_to_qvel.in_proj_bias"],
                     sd["attn_qpos_to_qvel.out_proj.weight"], sd["attn_qpos_to_qvel.out_proj.bias"], nheads)
    a2 = _mha_single(qv, qp, sd["attn_qvel_to_qpos.in_proj_weight"], sd["attn_qvel_to_qpos.in_proj_bias"],
                     sd["attn_qvel_to_qpos.out_proj.weight"], sd["attn_qvel_to_qpos.out_proj.bias"], nheads)
    f = np.concatenate([a1, a2], axis=-1)
    h = _relu(_layernorm(f, sd["fusion_layer.0.weight"], sd["fusion_layer.0.bias"]))
    h = _relu(_lin(h, sd["fusion_layer.2.weight"], sd["fusion_layer.2.bias"]))
    return _lin(h, sd["fusion_layer.4.weight"], sd["fusion_layer.4.bias"])


def ca_fold(sd: dict, qpos_dim: int, qvel_dim: int, action_dim: int) -> list:
    """Fold the cross-attention net into an fc stack over the input [x(nx), u(nu)] (fp64).

    fused[:D]  = attn_qpos_to_qvel(value = qvel_feat) = Wo1 (Wv1 (Wqv qvel + bqv) + bv1) + bo1
    fused[D:]  = attn_qvel_to_qpos(value = qpos_feat) = Wo2 (Wv2 (Wqp qpos + bqp) + bv2) + bo2
    The action encoder (learning/model.py:168,192) never reaches the output: its columns are 0.
    """
    f64 = lambda k: np.asarray(sd[k], np.float64)
    D = f64("qpos_encoder.weight").shape[0]
    nx = qpos_dim + qvel_dim
    W1 = np.zeros((2 * D, nx + action_dim))
    b1 = np.zeros(2 * D)
    Wv1 = f64("attn_qpos_to_qvel.in_proj_weight")[2 * D:]
    bv1 = f64("attn_qpos_to_qvel.in_proj_bias")[2 * D:]
    Wo1, bo1 = f64("attn_qpos_to_qvel.out_proj.weight"), f64("attn_qpos_to_qvel.out_proj.bias")
    Wv2 = f64("attn_qvel_to_qpos.in_proj_weight")[2 * D:]
    bv2 = f64("attn_qvel_to_qpos.in_proj_bias")[2 * D:]
    Wo2, bo2 = f64("attn_qvel_to_qpos.out_proj.weight"), f64("attn_qvel_to_qpos.out_proj.bias")
    Wqp, bqp = f64("qpos_encoder.weight"), f64("qpos_encoder.bias")
    Wqv, bqv = f64("qvel_encoder.weight"), f64("qvel_encoder.bias")
    W1[:D, qpos_dim:nx] = Wo1 @ Wv1 @ Wqv
    b1[:D] = Wo1 @ (Wv1 @ bqv + bv1) + bo1
    W1[D:, :qpos_dim] = Wo2 @ Wv2 @ Wqp
    b1[D:] = Wo2 @ (Wv2 @ bqp + bv2) + bo2
    return [
        dict(W=W1, b=b1, ln=(f64("fusion_layer.0.weight"), f64("fusion_layer.0.bias")), relu=True),
        dict(W=f64("fusion_layer.2.weight"), b=f64("fusion_layer.2.bias"), ln=None, relu=True),
        dict(W=f64("fusion_layer.4.weight"), b=f64("fusion_layer.4.bias"), ln=None, relu=False),
    ]


def ln_fold(stack: list) -> list:
    """The engine's LayerNorm fold of a CA stack (humanoid_mppi-rl_amd/csrc/mppi_nets.cpp, CROSS_ATTN), fp64.

    Exact in real arithmetic (tests/test_oracle.py::test_ln_fold_is_exact):
      * layer 0 rows centred, W0 -= 1 (1^T W0)/n, b0 -= mean(b0): the n outputs have mean 0 for every input, so
        LayerNorm's (h - mean) is h and its variance is mean(h^2);
      * rows with gamma < 0 negated (the variance is sign-blind);
      * relu(g z + b) = |g| relu(s z + b/|g|): |g| goes into layer 1's columns, beta' = b/|g|;
      * gamma == 0: the row outputs the constant relu(b), folded into b1 (its layer-1 column zeroed).
    The folded layer 0 evaluates relu(h * rstd + beta'), rstd = 1/sqrt(mean(h^2) + 1e-5) ("lnfold").
    """
    L0, L1 = stack[0], stack[1]
    g, be = (np.asarray(a, np.float64) for a in L0["ln"])
    W0 = np.asarray(L0["W"], np.float64)
    b0 = np.asarray(L0["b"], np.float64)
    W0 = W0 - W0.mean(axis=0, keepdims=True)
    b0 = b0 - b0.mean()
    sgn = np.where(g < 0, -1.0, 1.0)
    W0 = W0 * sgn[:, None]
    b0 = b0 * sgn
    ag = np.abs(g)
    W1 = np.asarray(L1["W"], np.float64) * ag[None, :]
    b1 = np.asarray(L1["b"], np.float64).copy()
    zero = g == 0
    b1 = b1 + np.asarray(L1["W"], np.float64)[:, zero] @ np.maximum(be[zero], 0.0)
    betap = np.where(zero, 0.0, be / np.where(zero, 1.0, ag))
    return [dict(W=W0, b=b0, ln=None, lnfold=betap, relu=True), dict(W=W1, b=b1, ln=None, relu=L1["relu"])] + \
        list(stack[2:])


def fcstack_forward(stack: list, xin: np.ndarray, precision: str = "fp64") -> np.ndarray:
    """Evaluate an fc stack with the engine's rounding points.

    precision "fp64": plain float64.  "fp32": float32 everywhere (MPPI_PREC_FP32).
    "bf16": every layer input and weight rounded to bf16, bias/accumulate/LayerNorm in fp32 (MPPI_PREC_BF16).
    """
    if precision == "fp64":
        h = np.asarray(xin, np.float64)
        for L in stack:
            h = _lin(h, L["W"], L["b"])
            if L["ln"] is not None:
                h = _layernorm(h, *L["ln"])
            if L.get("lnfold") is not None:
                h = h / np.sqrt((h * h).mean(axis=-1, keepdims=True) + 1e-5) + L["lnfold"]
            if L["relu"]:
                h = _relu(h)
        return h
    h = np.asarray(xin, np.float32)
    for L in stack:
        W = np.asarray(L["W"], np.float32)
        if precision == "bf16":
            h = bf16_round(h)
            W = bf16_round(W)
        h = (h @ W.T).astype(np.float32) + np.asarray(L["b"], np.float32)
        if L["ln"] is not None:
            g, b = (np.asarray(a, np.float32) for a in L["ln"])
            mu = h.mean(axis=-1, keepdims=True, dtype=np.float32)
            d = h - mu
            var = (d * d).mean(axis=-1, keepdims=True, dtype=np.float32)
            h = d * (1.0 / np.sqrt(var + np.float32(1e-5))) * g + b
        if L.get("lnfold") is not None:
            q = (h * h).mean(axis=-1, keepdims=True, dtype=np.float32)
            h = (h * (np.float32(1.0) / np.sqrt(q + np.float32(1e-5))) + np.asarray(L["lnfold"], np.float32))
        if L["relu"]:
            h = np.maximum(h, 0).astype(np.float32)
    return h


def learned_dynamics(stack: list, nx: int, precision: str = "fp64"):
    """x_{t+1} = x_t + net(cat(x_t, u_t)) — src/cartpole_mppi_estimator.py:89-93."""
    def dyn(x, u):
        xin = np.concatenate([x, u], axis=-1)
        d = fcstack_forward(stack, xin, precision)
        return (x + d[..., :nx]).astype(x.dtype)
    return dyn


# -------------------------------------------- Feature attention (learning/model.py:48-153)

def fa_forward(sd: dict, x: np.ndarray, state_dim: int, nheads: int) -> np.ndarray:
    """FeatureAttentionStatePredictor.forward, eval mode — learning/model.py:108-153."""
    B, I = x.shape
    D = sd["feature_encoding.0.weight"].shape[0]
    h = x[:, :, None] * sd["feature_encoding.0.weight"][:, 0][None, None, :] + sd["feature_encoding.0.bias"]
    h = _relu(_layernorm(h, sd["feature_encoding.1.weight"], sd["feature_encoding.1.bias"]))
    h = h + sd["pos_embedding"]
    nl = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    hd = D // nheads
    for li in range(nl):
        p = f"layers.{li}."
        xn = _layernorm(h, sd[p + "norm1.weight"], sd[p + "norm1.bias"])
        W, bb = sd[p + "attention.in_proj_weight"], sd[p + "attention.in_proj_bias"]
        q, k, v = _lin(xn, W[:D], bb[:D]), _lin(xn, W[D:2 * D], bb[D:2 * D]), _lin(xn, W[2 * D:], bb[2 * D:])
        o = np.empty_like(v)
        for hh in range(nheads):
            s = slice(hh * hd, (hh + 1) * hd)
            sc = np.einsum("bid,bjd->bij", q[..., s], k[..., s]) / np.sqrt(hd)
            sc = sc - sc.max(axis=-1, keepdims=True)
            pr = np.exp(sc)
            pr = pr / pr.sum(axis=-1, keepdims=True)
            o[..., s] = np.einsum("bij,bjd->bid", pr, v[..., s])
        h = h + _lin(o, sd[p + "attention.out_proj.weight"], sd[p + "attention.out_proj.bias"])
        xn = _layernorm(h, sd[p + "norm2.weight"], sd[p + "norm2.bias"])
        f = _relu(_lin(xn, sd[p + "ffn.0.weight"], sd[p + "ffn.0.bias"]))
        h = h + _lin(f, sd[p + "ffn.3.weight"], sd[p + "ffn.3.bias"])
    out = _lin(h, sd["output_layer.weight"], sd["output_layer.bias"])[..., 0]
    return out[:, :state_dim]


def fa_forward_engine(sd: dict, x: np.ndarray, state_dim: int, nheads: int = 4, precision: str = "fp32") -> np.ndarray:
    """fa_forward with the engine's rounding points (kernels_fa.hip), float32 arithmetic.

    "fp32": float32 everywhere (MPPI_PREC_FP32).  "bf16" (MPPI_PREC_BF16): GEMM weights rounded to bf16 (W_q
    after the 1/sqrt(head_dim) scaling); LayerNorm outputs, q/k/v (bias included), the attention output and the
    FFN hidden activations rounded to bf16 where they are stored, and (D >= 128: MFMA attention) the normalised
    attention probabilities (fa_small_kernel, hidden 64 with L <= 16 tokens, too); residual stream, scores, softmax arithmetic, biases,
    LayerNorms and the output layer in float32.
    """
    f32 = np.float32
    rb = bf16_round if precision == "bf16" else (lambda a: np.asarray(a, f32))
    W = lambda k: np.asarray(sd[k], f32)
    x = np.asarray(x, f32)
    B, I = x.shape
    D = sd["feature_encoding.0.weight"].shape[0]
    hd = D // nheads
    s = 1.0 / np.sqrt(hd)

    def ln(h, g, b):
        mu = h.mean(axis=-1, keepdims=True, dtype=f32)
        d = h - mu
        var = (d * d).mean(axis=-1, keepdims=True, dtype=f32)
        return d * (f32(1.0) / np.sqrt(var + f32(1e-5))) * g + b

    h = x[:, :, None] * W("feature_encoding.0.weight")[:, 0] + W("feature_encoding.0.bias")
    h = np.maximum(ln(h, W("feature_encoding.1.weight"), W("feature_encoding.1.bias")), 0) + W("pos_embedding")[0]
    nl = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    # bf16 small-net kernel (hidden 64, L <= 16): LayerNorm affine maps folded into the next GEMM on the host, W' =
    # W diag(gamma) rounded to bf16 (via float32), b' = b + W beta in float32; the LayerNorm outputs (x - mean) rstd
    nl_ = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    small = precision == "bf16" and D == 64 and I <= 16 and nheads == 4 and nl_ <= 4
    f64 = np.float64
    for li in range(nl):
        p = f"layers.{li}."
        iw, ib = np.asarray(sd[p + "attention.in_proj_weight"], f64), np.asarray(sd[p + "attention.in_proj_bias"], f64)
        iw, ib = np.concatenate([iw[:D] * s, iw[D:]]), np.concatenate([ib[:D] * s, ib[D:]])  # torch scales q
        if small:
            g1, b1 = np.asarray(sd[p + "norm1.weight"], f64), np.asarray(sd[p + "norm1.bias"], f64)
            xn = rb(ln(h, f32(1.0), f32(0.0)))
            ib, iw = (ib + iw @ b1), iw * g1[None, :]
        else:
            xn = rb(ln(h, W(p + "norm1.weight"), W(p + "norm1.bias")))
        q = rb(xn @ rb(iw[:D].astype(f32)).T + ib[:D].astype(f32))
        k = rb(xn @ rb(iw[D:2 * D].astype(f32)).T + ib[D:2 * D].astype(f32))
        v = rb(xn @ rb(iw[2 * D:].astype(f32)).T + ib[2 * D:].astype(f32))
        o = np.empty_like(v)
        for hh in range(nheads):
            sl = slice(hh * hd, (hh + 1) * hd)
            sc = np.einsum("bid,bjd->bij", q[..., sl], k[..., sl])
            pr = np.exp(sc - sc.max(axis=-1, keepdims=True))
            pr = pr / pr.sum(axis=-1, keepdims=True)
            if D >= 128 or small:  # bf16 MFMA attention (kernels_fa.hip: D >= 128, and the small-net
                pr = rb(pr)         # kernel for hidden 64, L <= 16, 4 heads, <= 4 layers): P as bf16
            o[..., sl] = np.einsum("bij,bjd->bid", pr, v[..., sl])
        h = h + rb(o) @ rb(W(p + "attention.out_proj.weight")).T + W(p + "attention.out_proj.bias")
        w1, bb1 = np.asarray(sd[p + "ffn.0.weight"], f64), np.asarray(sd[p + "ffn.0.bias"], f64)
        if small:
            g2, b2 = np.asarray(sd[p + "norm2.weight"], f64), np.asarray(sd[p + "norm2.bias"], f64)
            xn = rb(ln(h, f32(1.0), f32(0.0)))
            bb1, w1 = bb1 + w1 @ b2, w1 * g2[None, :]
        else:
            xn = rb(ln(h, W(p + "norm2.weight"), W(p + "norm2.bias")))
        f = rb(np.maximum(xn @ rb(w1.astype(f32)).T + bb1.astype(f32), 0))
        h = h + f @ rb(W(p + "ffn.3.weight")).T + W(p + "ffn.3.bias")
    out = (h @ W("output_layer.weight")[0]) + W("output_layer.bias")[0]
    return out[:, :state_dim].astype(f32)


def fa_dynamics(sd: dict, nx: int, nheads: int = 4, precision: str = "fp64"):
    """x_{t+1} = x_t + FA(cat(x_t, u_t)) — src/cartpole_mppi_estimator.py:89-93 with the FA net of :28-33."""
    def dyn(x, u):
        xin = np.concatenate([x, u], axis=-1)
        if precision == "fp64":
            d = fa_forward(sd, np.asarray(xin, np.float64), nx, nheads)
        else:
            d = fa_forward_engine(sd, xin, nx, nheads, precision)
        return (x + d).astype(x.dtype)
    return dyn
