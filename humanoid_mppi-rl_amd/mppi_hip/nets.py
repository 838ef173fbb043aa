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


def cross_attention_blob(sd: dict, qpos_dim: int = 28, qvel_dim: int = 27, action_dim: int = 21, hidden_dim: int = 128,
                         num_heads: int = 4) -> tuple[int, bytes]:
    """CrossAttentionStatePredictor (learning/model.py:157-202)."""
    return L.DYN_CROSS_ATTN, pack_blob(L.DYN_CROSS_ATTN, [qpos_dim, qvel_dim, action_dim, hidden_dim, num_heads], sd)


def mlp_blob(sd: dict, state_dim: int, action_dim: int, hidden_dim: int = 128, hidden_layers: int = 2) -> tuple[int, bytes]:
    """MLPStatePredictor (learning/model.py:6-46, use_batch_norm=False)."""
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


def synthetic_mlp(state_dim: int, action_dim: int, hidden_dim: int = 128, hidden_layers: int = 2, seed: int = 0) -> dict:
    """Seeded MLPStatePredictor state dict (no MLP checkpoint exists in the reference)."""
    rng = np.random.default_rng(seed)
    dims = [state_dim + action_dim] + [hidden_dim] * (hidden_layers + 1) + [state_dim]
    sd = {}
    for i in range(len(dims) - 1):
        w, b = _torch_linear_init(rng, dims[i + 1], dims[i])
        sd[f"network.{2 * i}.weight"], sd[f"network.{2 * i}.bias"] = w, b
    return sd
