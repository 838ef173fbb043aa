"""Learned-dynamics weights -> the engine's weight blob (format: csrc/mppi_nets.cpp header).

Accepts torch-style state dicts ({key: array}) of the reference's learning/model.py modules, e.g. the
arrays of checkpoints/model_cross.pth (saved as tests/golden/ca_humanoid_weights.npz), or seeded synthetic
weights with PyTorch's default nn.Linear init when no checkpoint exists (MLP, quadruped FA).
"""
from __future__ import annotations

import struct

import numpy as np

from . import _lib as L


def pack_blob(kind: int, dims: list[int], state_dict: dict) -> bytes:
    dims = list(dims) + [0] * (8 - len(dims))
    out = [b"MPPW", struct.pack("<II", 1, kind), struct.pack("<8i", *dims), struct.pack("<I", len(state_dict))]
    for name, arr in state_dict.items():
        a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
        nb = name.encode()
        out.append(struct.pack("<I", len(nb)) + nb + struct.pack("<I", a.ndim) + struct.pack(f"<{a.ndim}I", *a.shape))
        out.append(a.tobytes())
    return b"".join(out)


def load_npz(path: str, prefix: str = "") -> dict:
    with np.load(path) as z:
        return {k[len(prefix):]: z[k] for k in z.files if k.startswith(prefix)}


def cross_attention_blob(sd: dict, qpos_dim: int | None = None, qvel_dim: int | None = None,
                         action_dim: int | None = None, hidden_dim: int | None = None,
                         num_heads: int = 6) -> tuple[int, bytes]:
    """CrossAttentionStatePredictor (learning/model.py:157-202), any shape: dims default to the state dict's
    (qpos_encoder.weight [hidden, qpos], qvel_encoder.weight [hidden, qvel], action_encoder.weight [hidden, action]).
    The head count does not enter the folded net (attention over one key is the identity on the values)."""
    D, nq = np.shape(sd["qpos_encoder.weight"])
    nv = np.shape(sd["qvel_encoder.weight"])[1]
    na = np.shape(sd["action_encoder.weight"])[1]
    dims = [nq if qpos_dim is None else qpos_dim, nv if qvel_dim is None else qvel_dim,
            na if action_dim is None else action_dim, D if hidden_dim is None else hidden_dim, num_heads]
    return L.DYN_CROSS_ATTN, pack_blob(L.DYN_CROSS_ATTN, dims, sd)


def mlp_blob(sd: dict, state_dim: int, action_dim: int, hidden_dim: int | None = None,
             hidden_layers: int | None = None) -> tuple[int, bytes]:
    """MLPStatePredictor (learning/model.py:6-46), any width / depth, use_batch_norm either way (the engine folds the
    eval-mode BatchNorm); hidden_dim / hidden_layers default to the state dict's."""
    lin = sorted({int(k.split(".")[1]) for k, v in sd.items() if k.startswith("network.") and k.endswith(".weight")
                  and np.ndim(v) == 2})
    if hidden_dim is None:
        hidden_dim = int(np.shape(sd[f"network.{lin[0]}.weight"])[0])
    if hidden_layers is None:
        hidden_layers = len(lin) - 2
    sd = {k: v for k, v in sd.items() if not k.endswith("num_batches_tracked")}
    return L.DYN_MLP, pack_blob(L.DYN_MLP, [state_dim, action_dim, hidden_dim, hidden_layers], sd)


def feature_attention_blob(sd: dict, state_dim: int, action_dim: int, hidden_dim: int = 64, num_heads: int = 4,
                           attn_layers: int | None = None) -> tuple[int, bytes]:
    """FeatureAttentionStatePredictor (learning/model.py:48-153), e.g. src/cartpole_mppi_estimator.py:28-33
    (4, 1, 64, 4 heads, 2 layers) or src/quadruped_mppi_estimator.py:24-35 (37, 12, 512, 4, 2)."""
    if attn_layers is None:
        attn_layers = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
    return L.DYN_FEATURE_ATTN, pack_blob(L.DYN_FEATURE_ATTN, [state_dim, action_dim, hidden_dim, num_heads, attn_layers],
                                         sd)


def synthetic_feature_attention(state_dim: int, action_dim: int, hidden_dim: int, num_heads: int = 4,
                                attn_layers: int = 2, seed: int = 0) -> dict:
    """Seeded FA weights with PyTorch's default init scales (no quadruped checkpoint ships with the reference:
    checkpoints_quadruped/model_best.pth is listed in .MISSING_LARGE_BLOBS)."""
    rng = np.random.default_rng(seed)
    D, I = hidden_dim, state_dim + action_dim
    sd = {}
    sd["feature_encoding.0.weight"], sd["feature_encoding.0.bias"] = _torch_linear_init(rng, D, 1)
    sd["feature_encoding.1.weight"] = np.ones(D, np.float32)
    sd["feature_encoding.1.bias"] = np.zeros(D, np.float32)
    lim = np.sqrt(6.0 / (I + D))  # xavier_uniform on (1, I, D)
    sd["pos_embedding"] = rng.uniform(-lim, lim, (1, I, D)).astype(np.float32)
    for l in range(attn_layers):
        p = f"layers.{l}."
        sd[p + "norm1.weight"], sd[p + "norm1.bias"] = np.ones(D, np.float32), np.zeros(D, np.float32)
        lim = np.sqrt(6.0 / (D + 3 * D))
        sd[p + "attention.in_proj_weight"] = rng.uniform(-lim, lim, (3 * D, D)).astype(np.float32)
        sd[p + "attention.in_proj_bias"] = np.zeros(3 * D, np.float32)
        sd[p + "attention.out_proj.weight"], _ = _torch_linear_init(rng, D, D)
        sd[p + "attention.out_proj.bias"] = np.zeros(D, np.float32)
        sd[p + "norm2.weight"], sd[p + "norm2.bias"] = np.ones(D, np.float32), np.zeros(D, np.float32)
        sd[p + "ffn.0.weight"], sd[p + "ffn.0.bias"] = _torch_linear_init(rng, 4 * D, D)
        sd[p + "ffn.3.weight"], sd[p + "ffn.3.bias"] = _torch_linear_init(rng, D, 4 * D)
    sd["output_layer.weight"], sd["output_layer.bias"] = _torch_linear_init(rng, 1, D)
    return sd


def _torch_linear_init(rng: np.random.Generator, out_f: int, in_f: int):
    """nn.Linear default init: U(-1/sqrt(in), 1/sqrt(in)) for weight and bias (kaiming_uniform a=sqrt(5))."""
    bound = 1.0 / np.sqrt(in_f)
    return (rng.uniform(-bound, bound, (out_f, in_f)).astype(np.float32),
            rng.uniform(-bound, bound, (out_f,)).astype(np.float32))


def synthetic_mlp(state_dim: int, action_dim: int, hidden_dim: int = 128, hidden_layers: int = 2, seed: int = 0,
                  batch_norm: bool = False, dropout: bool = False) -> dict:
    """Seeded MLPStatePredictor state dict (no MLP checkpoint exists in the reference) with the module indices of
    learning/model.py:21-43: per hidden block Linear [, BatchNorm1d], ReLU [, Dropout].  batch_norm: non-trivial
    running statistics and affine parameters (an eval-mode BatchNorm1d)."""
    rng = np.random.default_rng(seed)
    dims = [state_dim + action_dim] + [hidden_dim] * (hidden_layers + 1) + [state_dim]
    sd, idx = {}, 0
    for i in range(len(dims) - 1):
        w, b = _torch_linear_init(rng, dims[i + 1], dims[i])
        sd[f"network.{idx}.weight"], sd[f"network.{idx}.bias"] = w, b
        idx += 1
        if i == len(dims) - 2:
            break
        if batch_norm:
            n = dims[i + 1]
            sd[f"network.{idx}.weight"] = rng.uniform(0.5, 1.5, n).astype(np.float32)
            sd[f"network.{idx}.bias"] = rng.uniform(-0.2, 0.2, n).astype(np.float32)
            sd[f"network.{idx}.running_mean"] = rng.uniform(-0.3, 0.3, n).astype(np.float32)
            sd[f"network.{idx}.running_var"] = rng.uniform(0.2, 2.0, n).astype(np.float32)
            idx += 1
        idx += 1  # ReLU
        if dropout:
            idx += 1
    return sd
