"""Surrogate training (mppi_hip/training.py), CPU: the reference loader's pairing on the
reference's own quadruped logs (tests/golden/quad_logs.npz), the torch module against the oracle's fc stack, and a
short training run that lowers the held-out MSE and packs into the engine's weight blob."""
import numpy as np

from conftest import golden
from oracle import nets_ref as N


def test_log_pairs_follow_the_reference_loader():
    from mppi_hip.training import log_pairs
    s = np.arange(6 * 3, dtype=np.float32).reshape(6, 3) ** 1.5
    a = -np.arange(6 * 2, dtype=np.float32).reshape(6, 2)
    X, Y = log_pairs(s, a)
    # rows 0 and 1 dropped (read_csv header + [1:], learning/data_loader.py:163-164); delta targets (:300-313)
    assert X.shape == (3, 5) and Y.shape == (3, 3)
    np.testing.assert_array_equal(X[0], np.concatenate([s[2], a[2]]))
    np.testing.assert_array_equal(Y, s[3:] - s[2:-1])


def test_mlp_module_matches_the_oracle_stack():
    import torch
    from mppi_hip.nets import synthetic_mlp
    from mppi_hip.training import mlp_module
    sd = synthetic_mlp(37, 12, seed=3)
    m = mlp_module(37, 12)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    X = np.random.RandomState(0).randn(16, 49).astype(np.float32)
    with torch.no_grad():
        y = m(torch.from_numpy(X)).numpy()
    np.testing.assert_allclose(y, N.fcstack_forward(N.mlp_stack(sd), X.astype(np.float64)), rtol=1e-5, atol=1e-6)


def test_short_training_lowers_eval_loss_and_packs():
    from mppi_hip import training as T
    g = golden("quad_logs.npz")
    X, Y = T.log_pairs(g["states0"], g["actions0"])
    (Xtr, Ytr), (Xev, Yev) = T.split_pairs(X, Y)
    model, hist = T.train_mlp(Xtr[:2000], Ytr[:2000], 37, 12, epochs=3, lr=1e-3, device="cpu",
                              eval_set=(Xev, Yev), log=None)
    import torch
    with torch.no_grad():  # the untrained weights train_mlp started from (same seed)
        torch.manual_seed(0)
        m0 = T.mlp_module(37, 12)
        e0 = float(torch.nn.functional.mse_loss(m0(torch.from_numpy(Xev)), torch.from_numpy(Yev)))
    assert hist[-1][1] < e0 and hist[-1][1] < hist[0][1]
    sd = T.state_dict_numpy(model)
    assert sorted(sd) == sorted(f"network.{i}.{p}" for i in (0, 2, 4, 6) for p in ("weight", "bias"))
    kind, blob = T.export_mlp_blob(sd, 37, 12)
    assert blob[:4] == b"MPPW" and len(blob) > 4 * sum(v.size for v in sd.values())


def test_fa_module_matches_the_oracle_forward():
    import torch
    from mppi_hip.nets import synthetic_feature_attention
    from mppi_hip.training import fa_module
    sd = synthetic_feature_attention(37, 12, 64, seed=5)
    m = fa_module(37, 12, 64).eval()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    X = 0.3 * np.random.RandomState(1).randn(8, 49).astype(np.float32)
    with torch.no_grad():
        y = m(torch.from_numpy(X)).numpy()
    np.testing.assert_allclose(y, N.fa_forward(sd, X.astype(np.float64), 37, 4), rtol=1e-4, atol=1e-5)
