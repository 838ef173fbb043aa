"""Generate G2 (cartpole MPPI solves) and G6 (cost known-answer tests) from the reference's OWN Python functions —
run ONLY in the build container (the reference is mounted read-only at /root/reference and never travels).

The reference scripts import mujoco and open a viewer at module level, so they cannot be imported whole. This script
parses each script with `ast` and executes ONLY the named pure-Python functions (no module-level statement runs),
in a namespace holding numpy / math / torch and the script's MPPI constants:

  G6  g6_cost_kat.npz        running_cost / terminal_cost of
        src/cartpole_mppi.py:44-53            (numpy, per sample)
        src/cartpole_mppi_estimator.py:46-55  (torch, batched)
        src/quadruped_mppi_estimator.py:48-55 (torch, batched; goal_pos of :45)
      on seeded random states/controls.
  G2  g2_cartpole_solve.npz  mppi_step + mppi_controller of src/cartpole_mppi.py:88-106 — the reference's own noise
      draw (np.random.seed(s); np.random.randn(nu,T,K)*sigma), softmin weights, Python-generator weighted sum,
      U update, u0 and the 0.1 decay shift — for (K,T) = (128,30), (4096,50), x0 in {0, (0,pi,0,0)}, U0 = 0 and a
      warm U0.  Its `rollout` (src/cartpole_mppi.py:59-85) needs MuJoCo, which is absent; the costs it would return
      come from the oracle's analytic mj_step rollout (oracle/mppi_ref.py, pinned to the recorded MuJoCo trajectory,
      G1) evaluated with the reference's own running_cost / terminal_cost above.  So G2 pins the solve semantics
      (noise layout and seeding, softmin, update, shift) to the reference code; the dynamics are pinned by G1.

Only arrays are written; no reference source is copied.
"""
from __future__ import annotations

import ast
import math
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("MPPI_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))


def ref_functions(relpath: str, names: list[str], consts: dict) -> dict:
    """Execute only the named top-level function definitions of a reference script; returns the namespace."""
    src = open(os.path.join(REF, relpath)).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    missing = set(names) - {n.name for n in keep}
    if missing:
        raise RuntimeError(f"{relpath}: functions not found: {missing}")
    ns = dict(np=np, math=math, torch=torch, **consts)
    exec(compile(ast.Module(body=keep, type_ignores=[]), os.path.join(REF, relpath), "exec"), ns)
    return ns


def gen_g6() -> dict:
    rs = np.random.RandomState(6)
    out = {}
    # src/cartpole_mppi.py: scalar arguments, control = ctrl vector (nu = 1)
    ns = ref_functions("src/cartpole_mppi.py", ["running_cost", "terminal_cost"], dict(nu=1))
    X = np.column_stack([rs.uniform(-1, 1, 64), rs.uniform(-4, 4, 64), rs.randn(64) * 2, rs.randn(64) * 3])
    Uc = rs.randn(64, 1) * 1.5
    out["cp_x"], out["cp_u"] = X, Uc
    out["cp_running"] = np.array([ns["running_cost"](*X[i], Uc[i]) for i in range(64)])
    out["cp_terminal"] = np.array([ns["terminal_cost"](*X[i]) for i in range(64)])
    # src/cartpole_mppi_estimator.py: torch tensors (batched over K)
    ns = ref_functions("src/cartpole_mppi_estimator.py", ["running_cost", "terminal_cost"], dict(nu=1))
    Xt = torch.from_numpy(X.astype(np.float32))
    out["cpe_running"] = ns["running_cost"](Xt[:, 0], Xt[:, 1], Xt[:, 2], Xt[:, 3], torch.from_numpy(
        Uc.astype(np.float32))).numpy()
    out["cpe_terminal"] = ns["terminal_cost"](Xt[:, 0], Xt[:, 1], Xt[:, 2], Xt[:, 3]).numpy()
    # src/quadruped_mppi_estimator.py: state (K, 37), control (K, 12), goal_pos of :45
    ns = ref_functions("src/quadruped_mppi_estimator.py", ["running_cost", "terminal_cost"],
                       dict(action_dim=12, goal_pos=np.array([2.0, 0.0, 0.35])))
    S = rs.randn(64, 37).astype(np.float32)
    S[:, :3] += np.array([1.0, 0.2, 0.3], np.float32)
    C = (rs.randn(64, 12) * 0.4).astype(np.float32)
    out["q_state"], out["q_ctrl"] = S, C
    out["q_running"] = ns["running_cost"](torch.from_numpy(S), torch.from_numpy(C)).numpy()
    out["q_terminal"] = ns["terminal_cost"](torch.from_numpy(S)).numpy()
    return out


def gen_g2() -> dict:
    from oracle import mppi_ref as R

    cost_ns = ref_functions("src/cartpole_mppi.py", ["running_cost", "terminal_cost"], dict(nu=1))
    rc, tc = cost_ns["running_cost"], cost_ns["terminal_cost"]

    def rollout(model, data, U, noise):
        """Stand-in for the MuJoCo rollout of src/cartpole_mppi.py:59-85: same loop, analytic mj_step (oracle,
        pinned by G1), the reference's cost functions, the unclamped ctrl passed to running_cost (:78)."""
        _, T, K = noise.shape
        costs = np.zeros(K)
        for k in range(K):
            x = np.concatenate([data.qpos, data.qvel]).astype(np.float64)
            c = 0.0
            for t in range(T):
                ctrl = U[:, t] + noise[:, t, k]
                x = R.cartpole_step(x, ctrl)
                c += rc(x[0], x[1], x[2], x[3], ctrl)
            costs[k] = c + tc(x[0], x[1], x[2], x[3])
        return costs

    out = {}
    cases = []
    for K, T in ((128, 30), (4096, 50)):
        for xi, x0 in enumerate((np.zeros(4), np.array([0.0, np.pi, 0.0, 0.0]))):
            for warm in (0, 1):
                cases.append((K, T, xi, x0, warm))
    for ci, (K, T, xi, x0, warm) in enumerate(cases):
        U0 = (0.5 * np.sin(np.arange(T) / 5.0))[None, :] if warm else np.zeros((1, T))
        ns = ref_functions("src/cartpole_mppi.py", ["mppi_step", "mppi_controller"],
                           dict(K=K, T=T, nu=1, _lambda=1.0, sigma=1.0, U_global=U0.copy(), rollout=rollout))
        rec = {}
        step = ns["mppi_step"]

        def step_rec(model, data, _step=step, _ns=ns, _rec=rec):
            _step(model, data)
            _rec["U_new"] = _ns["U_global"].copy()

        ns["mppi_step"] = step_rec
        data = types.SimpleNamespace(qpos=x0[:2].copy(), qvel=x0[2:].copy(), ctrl=np.zeros(1))
        seed = 100 + ci
        np.random.seed(seed)
        # the costs of this draw (the stand-in rollout is deterministic): recomputed from the same noise
        noise = np.random.RandomState(seed).randn(1, T, K) * 1.0
        ns["mppi_controller"](None, data)
        costs = rollout(None, data, U0, noise)
        p = f"c{ci}_"
        # noise is not stored: np.random.RandomState(seed).randn(1, T, K) regenerates it (legacy MT19937 stream)
        out.update({p + "K": K, p + "T": T, p + "seed": seed, p + "x0": x0, p + "U0": U0,
                    p + "costs": costs, p + "U_new": rec["U_new"], p + "u0": data.ctrl.copy(),
                    p + "U_shifted": ns["U_global"].copy()})
    out["n_cases"] = len(cases)
    return out


def main():
    g6 = gen_g6()
    np.savez_compressed(os.path.join(OUT, "g6_cost_kat.npz"), **g6)
    g2 = gen_g2()
    np.savez_compressed(os.path.join(OUT, "g2_cartpole_solve.npz"), **g2)
    print("wrote g6_cost_kat.npz, g2_cartpole_solve.npz", os.path.getsize(os.path.join(OUT, "g2_cartpole_solve.npz")))


if __name__ == "__main__":
    main()
