"""Generate the golden fixtures under tests/golden/ — run ONLY in the build container.

Sources (reference = SheffieldWang616/Humanoid_MPPI-RL mounted at /root/reference, read-only):
  * real MuJoCo cartpole trajectory data/2025-04-21_011138/{states,actions}.csv   -> g1_cartpole_kat.npz
  * trained checkpoints, loaded with torch.load(weights_only=True)                -> *_weights.npz (data)
  * outputs of the reference's own learning/model.py, imported from /root/reference/learning:
        FA cartpole forward   (checkpoints_cartpole/model_best.pth)    -> g3_fa_cartpole_fwd.npz
        CA humanoid forward   (checkpoints/model_cross.pth)            -> g5_ca_humanoid_fwd.npz
        MLP forward           (seeded torch default init, no checkpoint exists) -> g8_mlp_*_fwd.npz
        FA small quadruped    (seeded, d=64; the d=512 checkpoint is missing)   -> g8_fa_quad64_fwd.npz
  * estimator-style MPPI solves whose rollout loop restates src/cartpole_mppi_estimator.py:61-143 in torch
    around the imported reference nets (the estimator scripts themselves import mujoco at module level
    and open a viewer, so they cannot be imported):
        FA cartpole solve      K=256 T=16 lambda=10 sigma=0.5 replace  -> g4_fa_cartpole_solve.npz
        CA humanoid solve      K=128 H=16 lambda=1 sigma=0.75 add      -> g7_ca_humanoid_solve.npz
Only data (arrays) is written; no reference source is copied.
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

REF = os.environ.get("MPPI_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _sd(path):
    sd = torch.load(path, weights_only=True, map_location="cpu")
    return {k: v.detach().cpu().numpy().astype(np.float32) for k, v in sd.items()}


def _csv(path):
    return np.loadtxt(path, delimiter=",", ndmin=2)


def main():
    sys.path.insert(0, os.path.join(REF, "learning"))
    import model as refmodel  # the reference's learning/model.py

    torch.set_num_threads(8)
    out = {}

    # ---- G1: cartpole KAT (real MuJoCo trajectory, dt=0.01)
    d = os.path.join(REF, "data/2025-04-21_011138")
    st, ac = _csv(os.path.join(d, "states.csv")), _csv(os.path.join(d, "actions.csv"))
    np.savez_compressed(os.path.join(OUT, "g1_cartpole_kat.npz"), states=st, actions=ac)
    out["g1"] = st.shape

    # ---- weights (data)
    ca_h = _sd(os.path.join(REF, "checkpoints/model_cross.pth"))
    fa_c = _sd(os.path.join(REF, "checkpoints_cartpole/model_best.pth"))
    ca_c = _sd(os.path.join(REF, "checkpoints_cartpole/model_final.pth"))
    np.savez_compressed(os.path.join(OUT, "ca_humanoid_weights.npz"), **ca_h)
    np.savez_compressed(os.path.join(OUT, "fa_cartpole_weights.npz"), **fa_c)
    np.savez_compressed(os.path.join(OUT, "ca_cartpole_weights.npz"), **ca_c)

    # ---- G3: FA cartpole forward on 256 CSV rows (x || u)
    fa = refmodel.FeatureAttentionStatePredictor(state_dim=4, action_dim=1, hidden_dim=64, num_heads=4,
                                                 attn_layers=2, dropout_rate=0.0)
    fa.load_state_dict({k: torch.from_numpy(v) for k, v in fa_c.items()})
    fa.eval()
    xin = np.concatenate([st[:256], ac[:256]], axis=1).astype(np.float32)
    with torch.no_grad():
        y = fa(torch.from_numpy(xin)).numpy()
    np.savez_compressed(os.path.join(OUT, "g3_fa_cartpole_fwd.npz"), x=xin, y=y)

    # ---- G5: CA humanoid forward on 256 rows of data/2025-04-09_145305 (55 states + 21 actions)
    dh = os.path.join(REF, "data/2025-04-09_145305")
    hs, ha = _csv(os.path.join(dh, "states.csv")), _csv(os.path.join(dh, "actions.csv"))
    ca = refmodel.CrossAttentionStatePredictor(qpos_dim=28, qvel_dim=27, action_dim=21, hidden_dim=128,
                                               num_heads=4, dropout_rate=0.0)
    ca.load_state_dict({k: torch.from_numpy(v) for k, v in ca_h.items()})
    ca.eval()
    rows = np.arange(0, hs.shape[0], max(1, hs.shape[0] // 256))[:256]
    xin = np.concatenate([hs[rows], ha[rows]], axis=1).astype(np.float32)
    with torch.no_grad():
        y = ca(torch.from_numpy(xin)).numpy()
        y_noact = ca(torch.from_numpy(np.concatenate([hs[rows], 0 * ha[rows]], axis=1).astype(np.float32))).numpy()
    assert np.array_equal(y, y_noact), "CA output should not depend on the action (dead action encoder)"
    # x0 rows used by the humanoid benchmark config #4: rows of states.csv with stride 20
    np.savez_compressed(os.path.join(OUT, "g5_ca_humanoid_fwd.npz"), x=xin, y=y,
                        x0_stride20=hs[0:64 * 20:20].astype(np.float32))

    # ---- CA cartpole forward (model_final.pth: qpos 2, qvel 2, action 1, hidden 144, 6 heads; vis.ipynb cell 4)
    cac = refmodel.CrossAttentionStatePredictor(qpos_dim=2, qvel_dim=2, action_dim=1, hidden_dim=144,
                                                num_heads=6, dropout_rate=0.0)
    cac.load_state_dict({k: torch.from_numpy(v) for k, v in ca_c.items()})
    cac.eval()
    xin_c = np.concatenate([st[:256], ac[:256]], axis=1).astype(np.float32)
    with torch.no_grad():
        yc = cac(torch.from_numpy(xin_c)).numpy()
    np.savez_compressed(os.path.join(OUT, "g5_ca_cartpole_fwd.npz"), x=xin_c, y=yc)

    # ---- G8: MLP forward, seeded torch default init (no MLP checkpoint exists)
    for name, (sdim, adim) in {"humanoid": (55, 21), "quad": (37, 12)}.items():
        torch.manual_seed(0)
        mlp = refmodel.MLPStatePredictor(state_dim=sdim, action_dim=adim, hidden_dim=128, use_batch_norm=False,
                                         dropout_rate=0.0, hidden_layers=2)
        mlp.eval()
        g = torch.Generator().manual_seed(1)
        xin = torch.randn(256, sdim + adim, generator=g) * 0.5
        with torch.no_grad():
            y = mlp(xin).numpy()
        w = {k: v.detach().numpy().astype(np.float32) for k, v in mlp.state_dict().items()}
        np.savez_compressed(os.path.join(OUT, f"g8_mlp_{name}_fwd.npz"), x=xin.numpy(), y=y,
                            **{"w." + k: v for k, v in w.items()})

    # ---- G8: small FA quadruped (d=64) forward, seeded
    torch.manual_seed(0)
    faq = refmodel.FeatureAttentionStatePredictor(state_dim=37, action_dim=12, hidden_dim=64, num_heads=4,
                                                  attn_layers=2, dropout_rate=0.0)
    faq.eval()
    g = torch.Generator().manual_seed(2)
    xin = torch.randn(64, 49, generator=g) * 0.5
    with torch.no_grad():
        y = faq(xin).numpy()
    w = {k: v.detach().numpy().astype(np.float32) for k, v in faq.state_dict().items()}
    np.savez_compressed(os.path.join(OUT, "g8_fa_quad64_fwd.npz"), x=xin.numpy(), y=y,
                        **{"w." + k: v for k, v in w.items()})

    # ---- G4: estimator-style FA cartpole solve (restated loop of src/cartpole_mppi_estimator.py:61-143)
    K, T, lam, sigma = 256, 16, 10.0, 0.5
    rs = np.random.RandomState(4)
    noise = (rs.randn(1, T, K) * sigma).astype(np.float32)
    state = np.array([0.05, 0.1, 0.0, 0.0], np.float32)
    U0 = (0.1 * rs.randn(1, T)).astype(np.float32)
    with torch.no_grad():
        x = torch.from_numpy(state)[None].repeat(K, 1)
        nz = torch.from_numpy(noise).permute(2, 1, 0)
        Ut = torch.from_numpy(U0)
        costs = torch.zeros(K)

        def rc(xx):
            return (xx[:, 0] ** 2 + 50.0 * torch.abs(torch.cos(xx[:, 1]) - 1.0) + 0.1 * xx[:, 2] ** 2
                    + 0.1 * xx[:, 3] ** 2)
        for t in range(T):
            u = Ut[:, t][None].repeat(K, 1) + nz[:, t, :]
            x = x + fa(torch.cat([x, u], dim=1))
            costs += rc(x)
        costs += 10.0 * rc(x)
        beta = torch.min(costs)
        w = torch.exp(-1 / lam * (costs - beta))
        w = w / torch.sum(w)
        Unew = torch.sum(torch.from_numpy(noise) * w.reshape(1, 1, K), dim=2)
    np.savez_compressed(os.path.join(OUT, "g4_fa_cartpole_solve.npz"), x0=state, U0=U0, noise=noise,
                        costs=costs.numpy(), weights=w.numpy(), U_new=Unew.numpy(), K=K, T=T, lam=lam)

    # ---- G7: CA humanoid solve (loop of src/Humanoid_mppi_v3.jl:128-170 with x+ = x + net(x,u))
    K, H, lam, sigma = 128, 16, 1.0, 0.75
    rs = np.random.RandomState(7)
    noise = (rs.randn(21, H, K) * sigma).astype(np.float32)
    U0 = (0.2 * rs.randn(21, H)).astype(np.float32)
    x0 = hs[100].astype(np.float32)
    ctx = np.array([2.0, 0.0, 1.28, 0.15, 0.10, -0.02, 0.0, 0.0], np.float32)

    def hcost(xx, uu):
        q0, q1, q2, q3 = xx[:, 3], xx[:, 4], xx[:, 5], xx[:, 6]
        roll = torch.atan2(2 * (q0 * q1 + q2 * q3), 1 - 2 * (q1 ** 2 + q2 ** 2))
        pitch = torch.asin(torch.clamp(2 * (q0 * q2 - q3 * q1), -1, 1))
        yaw = torch.atan2(2 * (q0 * q3 + q1 * q2), 1 - 2 * (q2 ** 2 + q3 ** 2))
        c = 5 * (roll ** 2 + pitch ** 2) + 0.075 * yaw ** 2
        c = c + 12.5 * torch.sqrt((xx[:, 0] - ctx[0]) ** 2 + (xx[:, 1] - ctx[1]) ** 2)
        c = c + 5 * torch.abs(ctx[2] - xx[:, 2])
        c = c + torch.sqrt((xx[:, 28] - 0.3) ** 2 + xx[:, 29] ** 2)
        ftx = xx[:, 0] + 0.5
        c = c + 8 * torch.abs(ctx[3] - ftx) + 3 * (ctx[4] - ftx) ** 2 + ctx[5]
        return c + 0.01 * torch.sum(uu ** 2, dim=1)
    with torch.no_grad():
        x = torch.from_numpy(x0)[None].repeat(K, 1)
        nz = torch.from_numpy(noise).permute(2, 1, 0)
        Ut = torch.from_numpy(U0)
        costs = torch.zeros(K)
        for t in range(H):
            u = Ut[:, t][None].repeat(K, 1) + nz[:, t, :]
            x = x + ca(torch.cat([x, u], dim=1))
            costs += hcost(x, u)
        costs += 10.0 * hcost(x, torch.zeros(K, 21))
        beta = torch.min(costs)
        w = torch.exp(-1 / lam * (costs - beta))
        w = w / torch.sum(w)
        Unew = Ut + torch.sum(torch.from_numpy(noise) * w.reshape(1, 1, K), dim=2)
    np.savez_compressed(os.path.join(OUT, "g7_ca_humanoid_solve.npz"), x0=x0, U0=U0, noise=noise, ctx=ctx,
                        costs=costs.numpy(), weights=w.numpy(), U_new=Unew.numpy(), K=K, H=H, lam=lam)

    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f"{f:32s} {os.path.getsize(os.path.join(OUT, f)):>9d} B")


if __name__ == "__main__":
    main()
