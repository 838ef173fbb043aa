"""Dynamics-model training on PyTorch-ROCm for the engine's learned surrogates.

Restates the reference's training path: learning/train_quadruped.py:13-187 (Adam, cosine annealing, MSE on the
one-step state delta) over learning/data_loader.py:122-318 (transition pairs of logged MPPI runs, random train/eval
split) for its MLP (learning/model.py:6-46) and FeatureAttention (learning/model.py:48-153) surrogates.  Plain torch
on the HIP device: training is off the MPPI hot path, so it uses no custom kernels.  The trained weights export to
the engine's weight blob (nets.mlp_blob / nets.feature_attention_blob); the MLP trained on the reference's quadruped
logs replaces the checkpoint the reference does not ship (.MISSING_LARGE_BLOBS) for BASELINE config #3 ("learned
MLP dynamics (checkpoints_quadruped)").

    python -m mppi_hip.training --data tests/golden/quad_logs.npz --out tests/golden/quad_mlp_trained.npz
"""
from __future__ import annotations

import argparse
import time

import numpy as np

from . import nets


def log_pairs(states: np.ndarray, actions: np.ndarray, skip: int = 2) -> tuple[np.ndarray, np.ndarray]:
    """Transition pairs of one logged run with the reference loader's row handling.  pd.read_csv takes the file's
    first line as a header and `[1:]` drops the next one (learning/data_loader.py:163-164), so the pairs start at
    file line 3; pair i is (x_i || u_i) -> x_{i+1} - x_i (return_type 'delta', learning/data_loader.py:300-313)."""
    s, a = np.asarray(states, np.float32)[skip:], np.asarray(actions, np.float32)[skip:]
    if len(s) != len(a) or len(s) < 2:
        raise ValueError("a run needs matching state/action rows, at least 2 after the skipped ones")
    return np.concatenate([s[:-1], a[:-1]], axis=1), s[1:] - s[:-1]


def load_log_pairs(path: str) -> tuple[np.ndarray, np.ndarray]:
    """All runs of a logs npz (tests/golden/gen_quad_logs.py: states<i>, actions<i>), pairs concatenated."""
    with np.load(path) as z:
        n = sum(1 for k in z.files if k.startswith("states"))
        parts = [log_pairs(z[f"states{i}"], z[f"actions{i}"]) for i in range(n)]
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def split_pairs(X: np.ndarray, Y: np.ndarray, train_ratio: float = 0.9, seed: int = 42):
    """Random split of the pooled pairs (random_split=True, learning/data_loader.py:203-209)."""
    idx = np.random.RandomState(seed).permutation(len(X))
    n = int(len(X) * train_ratio)
    return (X[idx[:n]], Y[idx[:n]]), (X[idx[n:]], Y[idx[n:]])


def mlp_module(state_dim: int, action_dim: int, hidden_dim: int = 128, hidden_layers: int = 2):
    """torch module with MLPStatePredictor's layer stack and parameter names (learning/model.py:6-46, no batch norm
    or dropout): network.{0,2,..}.weight/bias, so its state dict packs with nets.mlp_blob unchanged."""
    import torch.nn as nn

    dims = [state_dim + action_dim] + [hidden_dim] * (hidden_layers + 1)
    layers = []
    for i in range(len(dims) - 1):
        layers += [nn.Linear(dims[i], dims[i + 1]), nn.ReLU()]
    layers.append(nn.Linear(hidden_dim, state_dim))

    class MLPStatePredictor(nn.Module):
        def __init__(self):
            super().__init__()
            self.network = nn.Sequential(*layers)

        def forward(self, x):
            return self.network(x)

    return MLPStatePredictor()


def fa_module(state_dim: int, action_dim: int, hidden_dim: int = 512, num_heads: int = 4, attn_layers: int = 2,
              dropout: float = 0.1):
    """torch module with FeatureAttentionStatePredictor's parameters and names (learning/model.py:48-153): every
    input scalar is a token (Linear(1, D) -> LayerNorm -> ReLU, + a learned position embedding), pre-LN blocks of
    multi-head self-attention and a D -> 4D -> D FFN (dropout while training), a D -> 1 head on every token, the
    state tokens' outputs are the prediction.  Its state dict packs with nets.feature_attention_blob; the engine
    evaluates it in eval mode (dropout off), as the reference's estimators do."""
    import torch
    import torch.nn as nn

    L, D = state_dim + action_dim, hidden_dim

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.norm1 = nn.LayerNorm(D)
            self.attention = nn.MultiheadAttention(D, num_heads, dropout=dropout, batch_first=True)
            self.norm2 = nn.LayerNorm(D)
            self.ffn = nn.Sequential(nn.Linear(D, 4 * D), nn.ReLU(), nn.Dropout(dropout), nn.Linear(4 * D, D))
            self.drop = nn.Dropout(dropout)

        def forward(self, h):
            n = self.norm1(h)
            h = h + self.drop(self.attention(n, n, n, need_weights=False)[0])
            return h + self.drop(self.ffn(self.norm2(h)))

    class FeatureAttentionStatePredictor(nn.Module):
        def __init__(self):
            super().__init__()
            self.feature_encoding = nn.Sequential(nn.Linear(1, D), nn.LayerNorm(D), nn.ReLU())
            self.pos_embedding = nn.Parameter(torch.empty(1, L, D))
            nn.init.xavier_uniform_(self.pos_embedding)
            self.layers = nn.ModuleList(Block() for _ in range(attn_layers))
            self.output_layer = nn.Linear(D, 1)

        def forward(self, x):
            h = self.feature_encoding(x.reshape(x.shape[0], L, 1)) + self.pos_embedding
            for blk in self.layers:
                h = blk(h)
            return self.output_layer(h)[..., 0][:, :state_dim]

    return FeatureAttentionStatePredictor()


def train(model, X: np.ndarray, Y: np.ndarray, epochs: int = 50, batch: int = 32, lr: float = 1e-4,
          device: str = "cuda", seed: int = 0, eval_set=None, log=print):
    """The reference loop (learning/train_quadruped.py:58-91): Adam(lr 1e-4), CosineAnnealingLR(T_max = epochs,
    eta_min 1e-6), batch 32, MSE on the delta.  Returns (model in eval mode, history) with the mean train / eval
    MSE per epoch."""
    import torch

    dev = torch.device(device)
    model = model.to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=epochs, eta_min=1e-6)
    Xt, Yt = torch.from_numpy(np.ascontiguousarray(X)).to(dev), torch.from_numpy(np.ascontiguousarray(Y)).to(dev)
    Ev = None if eval_set is None else tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in eval_set)
    gen = torch.Generator(device="cpu").manual_seed(seed)
    hist = []

    def eval_mse():
        if Ev is None:
            return float("nan")
        model.eval()
        with torch.no_grad():
            e = float(torch.nn.functional.mse_loss(model(Ev[0]), Ev[1]))
        model.train()
        return e

    for ep in range(epochs):
        t0, tot = time.perf_counter(), torch.zeros((), device=dev)
        perm = torch.randperm(len(Xt), generator=gen).to(dev)
        nb = (len(Xt) + batch - 1) // batch
        for i in range(nb):
            j = perm[i * batch:(i + 1) * batch]
            loss = torch.nn.functional.mse_loss(model(Xt[j]), Yt[j])
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            tot += loss.detach()
        sched.step()
        hist.append((float(tot) / nb, eval_mse()))
        if log:
            log(f"epoch {ep + 1}/{epochs}: train mse {hist[-1][0]:.4e}  eval mse {hist[-1][1]:.4e}  "
                f"({time.perf_counter() - t0:.1f} s)")
    return model.eval(), hist


def train_mlp(X: np.ndarray, Y: np.ndarray, state_dim: int, action_dim: int, hidden_dim: int = 128,
              hidden_layers: int = 2, epochs: int = 50, batch: int = 32, lr: float = 1e-4, device: str = "cuda",
              seed: int = 0, eval_set=None, log=print):
    """train() on a fresh MLPStatePredictor (seeded init)."""
    import torch

    torch.manual_seed(seed)
    return train(mlp_module(state_dim, action_dim, hidden_dim, hidden_layers), X, Y, epochs, batch, lr, device, seed,
                 eval_set, log)


def train_fa(X: np.ndarray, Y: np.ndarray, state_dim: int, action_dim: int, hidden_dim: int = 512, num_heads: int = 4,
             attn_layers: int = 2, epochs: int = 50, batch: int = 32, lr: float = 1e-4, device: str = "cuda",
             seed: int = 0, eval_set=None, log=print):
    """train() on a fresh FeatureAttentionStatePredictor (seeded init; the quadruped estimator's net is
    (37, 12, 512, 4 heads, 2 layers), learning/train_quadruped.py:53-54)."""
    import torch

    torch.manual_seed(seed)
    return train(fa_module(state_dim, action_dim, hidden_dim, num_heads, attn_layers), X, Y, epochs, batch, lr, device,
                 seed, eval_set, log)


def state_dict_numpy(model) -> dict:
    return {k: v.detach().float().cpu().numpy() for k, v in model.state_dict().items()}


def export_mlp_blob(sd: dict, state_dim: int, action_dim: int, hidden_dim: int = 128, hidden_layers: int = 2):
    """(kind, blob) for Engine.load_dynamics."""
    return nets.mlp_blob(sd, state_dim, action_dim, hidden_dim, hidden_layers)


def export_fa_blob(sd: dict, state_dim: int, action_dim: int, hidden_dim: int = 512, num_heads: int = 4):
    """(kind, blob) for Engine.load_dynamics."""
    return nets.feature_attention_blob(sd, state_dim, action_dim, hidden_dim, num_heads)


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--data", required=True, help="logs npz (tests/golden/gen_quad_logs.py)")
    ap.add_argument("--out", required=True, help="trained state dict (npz)")
    ap.add_argument("--arch", choices=["mlp", "fa"], default="mlp")
    ap.add_argument("--state-dim", type=int, default=37)
    ap.add_argument("--action-dim", type=int, default=12)
    ap.add_argument("--hidden", type=int, default=None, help="default: 128 (mlp), 512 (fa)")
    ap.add_argument("--layers", type=int, default=2, help="hidden layers (mlp) / attention layers (fa)")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()
    X, Y = load_log_pairs(args.data)
    if X.shape[1] != args.state_dim + args.action_dim:
        raise SystemExit(f"logs have {X.shape[1]} input columns, expected {args.state_dim + args.action_dim}")
    tr, ev = split_pairs(X, Y)
    print(f"{len(tr[0])} train / {len(ev[0])} eval pairs")
    if args.arch == "mlp":
        model, hist = train_mlp(*tr, args.state_dim, args.action_dim, args.hidden or 128, args.layers, args.epochs,
                                args.batch, args.lr, args.device, eval_set=ev)
    else:
        model, hist = train_fa(*tr, args.state_dim, args.action_dim, args.hidden or 512, 4, args.layers, args.epochs,
                               args.batch, args.lr, args.device, eval_set=ev)
    sd = state_dict_numpy(model)
    np.savez(args.out, **sd, train_mse=np.array([h[0] for h in hist]), eval_mse=np.array([h[1] for h in hist]))
    print(f"wrote {args.out}: eval mse {hist[-1][1]:.4e} (zero-delta baseline {float(np.mean(ev[1] ** 2)):.4e})")


if __name__ == "__main__":
    main()
