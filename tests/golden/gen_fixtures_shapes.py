"""Golden forward outputs of the reference's learning/model.py at the net shapes beyond the shipped checkpoints —
run ONLY in the build container (imports /root/reference/learning/model.py; nothing of it is copied).

The weights are the engine's seeded synthetic state dicts (mppi_hip.nets.synthetic_mlp / synthetic_feature_attention,
regenerated bit-identically by the tests from the seed), loaded into the reference modules with
load_state_dict(strict=True); the fixtures hold only the inputs, the reference module's eval-mode outputs and the
shape / seed:
  g9_mlp_bn_fwd.npz     MLPStatePredictor(55, 21, hidden 512, use_batch_norm=True, dropout 0.2, hidden_layers=6)
                        (the MLP of learning/train.py:70) on 64 logged humanoid (state, action) rows
  g9_fa_h8l7_fwd.npz    FeatureAttentionStatePredictor(30, 21, hidden 512, 8 heads, 7 layers)
                        (learning/train.py:71-72: state = qpos + the two foot heights, 51 tokens) on 16 rows
  g9_fa76_fwd.npz       FeatureAttentionStatePredictor(55, 21, hidden 128, 4 heads, 2 layers) (learning/model.py:215,
                        76 tokens: the full humanoid state + action) on 16 rows
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("MPPI_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REPO, "humanoid_mppi-rl_amd"))

SHAPES = {
    "g9_mlp_bn_fwd": dict(kind="mlp", nx=55, nu=21, hidden=512, layers=6, seed=70, rows=64),
    "g9_fa_h8l7_fwd": dict(kind="fa", nx=30, nu=21, hidden=512, heads=8, layers=7, seed=72, rows=16),
    "g9_fa76_fwd": dict(kind="fa", nx=55, nu=21, hidden=128, heads=4, layers=2, seed=76, rows=16),
}


def weights(spec: dict) -> dict:
    """The seeded state dict of a SHAPES entry (the tests call this too)."""
    from mppi_hip.nets import synthetic_feature_attention, synthetic_mlp
    if spec["kind"] == "mlp":
        return synthetic_mlp(spec["nx"], spec["nu"], spec["hidden"], spec["layers"], seed=spec["seed"], batch_norm=True,
                             dropout=True)
    sd = synthetic_feature_attention(spec["nx"], spec["nu"], spec["hidden"], num_heads=spec["heads"],
                                     attn_layers=spec["layers"], seed=spec["seed"])
    rs = np.random.RandomState(spec["seed"])  # non-trivial LayerNorm affines and biases
    for k in list(sd):
        if k.endswith(("norm1.weight", "norm2.weight")) or k == "feature_encoding.1.weight":
            sd[k] = (1.0 + 0.2 * rs.randn(*sd[k].shape)).astype(np.float32)
        elif k.endswith(("norm1.bias", "norm2.bias", "in_proj_bias", "out_proj.bias")) or k == "feature_encoding.1.bias":
            sd[k] = (0.1 * rs.randn(*sd[k].shape)).astype(np.float32)
    return sd


def inputs(spec: dict) -> np.ndarray:
    """Rows of the reference's humanoid log (tests/golden/g5_ca_humanoid_fwd.npz 'x': 55 states + 21 actions); the
    30-state FA takes qpos (28) and two further state columns, as learning/train.py:41 selects 30 columns."""
    x = np.load(os.path.join(HERE, "g5_ca_humanoid_fwd.npz"))["x"][: spec["rows"]].astype(np.float32)
    if spec["nx"] == 30:
        x = np.concatenate([x[:, :28], x[:, 28:30], x[:, 55:76]], axis=1)
    return x


def main():
    sys.path.insert(0, os.path.join(REF, "learning"))
    import model as M  # the reference module (learning/model.py)
    torch.manual_seed(0)
    for name, spec in SHAPES.items():
        sd = weights(spec)
        if spec["kind"] == "mlp":
            net = M.MLPStatePredictor(state_dim=spec["nx"], action_dim=spec["nu"], hidden_dim=spec["hidden"],
                                      use_batch_norm=True, dropout_rate=0.2, hidden_layers=spec["layers"])
        else:
            net = M.FeatureAttentionStatePredictor(state_dim=spec["nx"], action_dim=spec["nu"], hidden_dim=spec["hidden"],
                                                   num_heads=spec["heads"], attn_layers=spec["layers"])
        tsd = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}
        for k, v in net.state_dict().items():  # BatchNorm's step counter carries no arithmetic
            if k.endswith("num_batches_tracked"):
                tsd[k] = v.clone()
        net.load_state_dict(tsd, strict=True)
        net.eval()
        x = inputs(spec)
        with torch.no_grad():
            y = net(torch.from_numpy(x)).numpy()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, y=y.astype(np.float32),
                            **{k: np.asarray(v) for k, v in spec.items() if k != "kind"})
        print(name, x.shape, y.shape, float(np.abs(y).max()))


if __name__ == "__main__":
    main()
