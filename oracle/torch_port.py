"""torch-CPU port of the reference learned-dynamics MPPI solve — CPU BASELINE / TEST INFRASTRUCTURE ONLY.

Mirrors src/cartpole_mppi_estimator.py:61-143 (batched-K rollout, one net forward per horizon step, torch
softmin and weighted-noise sum) with the humanoid cost of src/Humanoid_mppi_v3.jl:27-105 and the
CrossAttentionStatePredictor forward of learning/model.py:183-202 computed the way torch computes it
(all encoders including the dead action encoder, full q/k/v in_proj, per-head attention, out_proj).
bench.py times it on the GPU box's host cores as the "port" CPU baseline (the reference itself cannot
travel to the box, and its MuJoCo/Julia paths cannot run without MuJoCo/Julia).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.nn.functional as F


class CrossAttentionPort(torch.nn.Module):
    def __init__(self, sd: dict, qpos_dim=28, qvel_dim=27, nheads=4):
        super().__init__()
        self.p = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.nq, self.nv, self.h = qpos_dim, qvel_dim, nheads

    def _mha(self, pre, q_in, kv_in):
        p = self.p
        D = q_in.shape[-1]
        W, b = p[pre + ".in_proj_weight"], p[pre + ".in_proj_bias"]
        q = F.linear(q_in, W[:D], b[:D])
        k = F.linear(kv_in, W[D:2 * D], b[D:2 * D])
        v = F.linear(kv_in, W[2 * D:], b[2 * D:])
        B = q.shape[0]
        hd = D // self.h
        q, k, v = (t.view(B, 1, self.h, hd).transpose(1, 2) for t in (q, k, v))
        att = torch.softmax(q @ k.transpose(-1, -2) / hd ** 0.5, dim=-1)
        o = (att @ v).transpose(1, 2).reshape(B, D)
        return F.linear(o, p[pre + ".out_proj.weight"], p[pre + ".out_proj.bias"])

    def forward(self, x):
        p, nq, nv = self.p, self.nq, self.nv
        qp = F.linear(x[:, :nq], p["qpos_encoder.weight"], p["qpos_encoder.bias"])
        qv = F.linear(x[:, nq:nq + nv], p["qvel_encoder.weight"], p["qvel_encoder.bias"])
        _ = F.linear(x[:, nq + nv:], p["action_encoder.weight"], p["action_encoder.bias"])  # computed, unused
        a1 = self._mha("attn_qpos_to_qvel", qp, qv)
        a2 = self._mha("attn_qvel_to_qpos", qv, qp)
        h = torch.cat([a1, a2], dim=-1)
        h = F.relu(F.layer_norm(h, (h.shape[-1],), p["fusion_layer.0.weight"], p["fusion_layer.0.bias"]))
        h = F.relu(F.linear(h, p["fusion_layer.2.weight"], p["fusion_layer.2.bias"]))
        return F.linear(h, p["fusion_layer.4.weight"], p["fusion_layer.4.bias"])


def humanoid_cost_torch(x, u, ctx):
    q0, q1, q2, q3 = x[:, 3], x[:, 4], x[:, 5], x[:, 6]
    roll = torch.atan2(2 * (q0 * q1 + q2 * q3), 1 - 2 * (q1 ** 2 + q2 ** 2))
    pitch = torch.asin(torch.clamp(2 * (q0 * q2 - q3 * q1), -1, 1))
    yaw = torch.atan2(2 * (q0 * q3 + q1 * q2), 1 - 2 * (q2 ** 2 + q3 ** 2))
    c = 5 * (roll ** 2 + pitch ** 2) + 0.075 * yaw ** 2
    c = c + 12.5 * torch.sqrt((x[:, 0] - ctx[0]) ** 2 + (x[:, 1] - ctx[1]) ** 2) + 5 * torch.abs(ctx[2] - x[:, 2])
    c = c + torch.sqrt((x[:, 28] - 0.3) ** 2 + x[:, 29] ** 2)
    ftx = x[:, 0] + 0.5
    c = c + 8 * torch.abs(ctx[3] - ftx) + 3 * (ctx[4] - ftx) ** 2 + ctx[5]
    return c + 0.01 * torch.sum(u ** 2, dim=1)


@torch.no_grad()
def mppi_solve_torch(net, x0, U, noise, ctx, lam=1.0):
    """One humanoid MPPI solve, estimator structure (src/cartpole_mppi_estimator.py:61-143), additive update."""
    nu, T, K = noise.shape
    x = torch.as_tensor(x0, dtype=torch.float32)[None].repeat(K, 1)
    nz = noise.permute(2, 1, 0)
    costs = torch.zeros(K)
    for t in range(T):
        u = U[:, t][None].repeat(K, 1) + nz[:, t, :]
        x = x + net(torch.cat([x, u], dim=1))
        costs += humanoid_cost_torch(x, u, ctx)
    costs += 10.0 * humanoid_cost_torch(x, torch.zeros(K, nu), ctx)
    beta = torch.min(costs)
    w = torch.exp(-1 / lam * (costs - beta))
    w = w / torch.sum(w)
    return U + torch.sum(noise * w.reshape(1, 1, K), dim=2), costs


def time_humanoid_baseline(sd: dict, x0: np.ndarray, K: int, H: int, threads: int, budget_s: float = 15.0,
                           max_solves: int = 20) -> dict:
    """Time full solves (K, H) on `threads` host cores until budget_s; returns traj-steps/s (median)."""
    torch.set_num_threads(threads)
    net = CrossAttentionPort(sd)
    ctx = torch.tensor([2.0, 0.0, 1.28, 0.0, 0.0, 0.0, 0.0, 0.0])
    g = torch.Generator().manual_seed(0)
    U = torch.zeros(21, H)
    times = []
    t_start = time.perf_counter()
    mppi_solve_torch(net, x0, U[:, :2], torch.randn(21, 2, K, generator=g) * 0.75, ctx)  # warm-up (short)
    while len(times) < max_solves and (time.perf_counter() - t_start) < budget_s:
        noise = torch.randn(21, H, K, generator=g) * 0.75
        t0 = time.perf_counter()
        U, _ = mppi_solve_torch(net, x0, U, noise, ctx)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return dict(value=K * H / med, ms_per_solve=med * 1e3, solves=len(times))


class FeatureAttentionPort(torch.nn.Module):
    """FeatureAttentionStatePredictor forward (learning/model.py:108-153) computed the way torch computes it:
    nn.MultiheadAttention (batch_first, need_weights) over the L feature tokens, pre-LN blocks, all L outputs."""

    def __init__(self, sd: dict, state_dim: int, nheads: int = 4):
        super().__init__()
        p = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.p, self.nx = p, state_dim
        D = p["feature_encoding.0.weight"].shape[0]
        self.nl = len({k.split(".")[1] for k in sd if k.startswith("layers.")})
        self.mha = []
        for l in range(self.nl):
            m = torch.nn.MultiheadAttention(D, nheads, batch_first=True)
            m.in_proj_weight.data.copy_(p[f"layers.{l}.attention.in_proj_weight"])
            m.in_proj_bias.data.copy_(p[f"layers.{l}.attention.in_proj_bias"])
            m.out_proj.weight.data.copy_(p[f"layers.{l}.attention.out_proj.weight"])
            m.out_proj.bias.data.copy_(p[f"layers.{l}.attention.out_proj.bias"])
            m.eval()
            self.mha.append(m)

    def forward(self, x):
        p = self.p
        B, L = x.shape
        D = p["feature_encoding.0.weight"].shape[0]
        h = F.linear(x.view(B, L, 1), p["feature_encoding.0.weight"], p["feature_encoding.0.bias"])
        h = F.relu(F.layer_norm(h, (D,), p["feature_encoding.1.weight"], p["feature_encoding.1.bias"]))
        h = h + p["pos_embedding"]
        for l in range(self.nl):
            q = f"layers.{l}."
            xn = F.layer_norm(h, (D,), p[q + "norm1.weight"], p[q + "norm1.bias"])
            h = h + self.mha[l](xn, xn, xn)[0]
            xn = F.layer_norm(h, (D,), p[q + "norm2.weight"], p[q + "norm2.bias"])
            h = h + F.linear(F.relu(F.linear(xn, p[q + "ffn.0.weight"], p[q + "ffn.0.bias"])), p[q + "ffn.3.weight"],
                             p[q + "ffn.3.bias"])
        return F.linear(h, p["output_layer.weight"], p["output_layer.bias"]).squeeze(-1)[:, :self.nx]


def cartpole_est_cost_torch(x, u):  # src/cartpole_mppi_estimator.py:46-52
    return x[:, 0] ** 2 + 50.0 * torch.abs(torch.cos(x[:, 1]) - 1.0) + 0.1 * x[:, 2] ** 2 + 0.1 * x[:, 3] ** 2


def quad_est_cost_torch(x, u):  # src/quadruped_mppi_estimator.py:48-52
    return torch.sum((x[:, :3] - torch.tensor([2.0, 0.0, 0.35])) ** 2, dim=1) + 0.1 * torch.sum(u ** 2, dim=1)


@torch.no_grad()
def mppi_solve_estimator_torch(net, x0, U, noise, cost, lam=10.0):
    """src/cartpole_mppi_estimator.py:61-143 / src/quadruped_mppi_estimator.py:58-95: replace-mode update."""
    nu, T, K = noise.shape
    x = torch.as_tensor(x0, dtype=torch.float32)[None].repeat(K, 1)
    nz = noise.permute(2, 1, 0)
    costs = torch.zeros(K)
    for t in range(T):
        u = U[:, t][None].repeat(K, 1) + nz[:, t, :]
        x = x + net(torch.cat([x, u], dim=1))
        costs += cost(x, u)
    costs += 10.0 * cost(x, torch.zeros(K, nu))
    w = torch.exp(-1 / lam * (costs - torch.min(costs)))
    w = w / torch.sum(w)
    return torch.sum(noise * w.reshape(1, 1, K), dim=2), costs


def time_fa_baseline(sd: dict, x0: np.ndarray, nx: int, nu: int, K: int, H: int, cost: str, sigma: float,
                     threads: int, budget_s: float = 15.0, max_solves: int = 20) -> dict:
    """Time estimator-style FA solves (K, H) on `threads` host cores until budget_s (median traj-steps/s)."""
    torch.set_num_threads(threads)
    net = FeatureAttentionPort(sd, nx)
    cf = cartpole_est_cost_torch if cost == "cartpole_est" else quad_est_cost_torch
    g = torch.Generator().manual_seed(0)
    U = torch.zeros(nu, H)
    times = []
    mppi_solve_estimator_torch(net, x0, U[:, :1], torch.randn(nu, 1, K, generator=g) * sigma, cf)  # warm-up
    t_start = time.perf_counter()
    while len(times) < max_solves and (time.perf_counter() - t_start) < budget_s:
        noise = torch.randn(nu, H, K, generator=g) * sigma
        t0 = time.perf_counter()
        U, _ = mppi_solve_estimator_torch(net, x0, U, noise, cf)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return dict(value=K * H / med, ms_per_solve=med * 1e3, solves=len(times))
