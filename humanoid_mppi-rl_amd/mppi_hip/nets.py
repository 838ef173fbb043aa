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
