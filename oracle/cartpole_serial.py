"""Serial per-sample port of the reference cartpole MPPI — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Same loop shape as src/cartpole_mppi.py:59-98 (for k: for t: step; cost; then the Python generator
reduction over K per t), with mujoco.mj_step replaced by the scalar analytic cartpole step that
oracle/mppi_ref.py::cartpole_step vectorises (pinned by the MuJoCo trajectory KAT). bench.py times it on one
host core as the "port" CPU baseline of the cartpole configuration.
"""
from __future__ import annotations

import math

import numpy as np

from .mppi_ref import CARTPOLE

_P = CARTPOLE


def step(x_pos, theta, x_vel, theta_vel, u):
    dt, D, mp, l = _P["dt"], _P["damping"], _P["m_pole"], _P["l"]
    F = _P["gear"] * min(_P["ctrl_hi"], max(_P["ctrl_lo"], u))
    s, c = math.sin(theta), math.cos(theta)
    m11 = _P["m_cart"] + mp + dt * D
    m12 = mp * l * c
    m22 = mp * l * l + _P["inertia"] + dt * D
    f1 = F + mp * l * s * theta_vel * theta_vel - D * x_vel
    f2 = mp * _P["g"] * l * s - D * theta_vel
    det = m11 * m22 - m12 * m12
    a1 = (m22 * f1 - m12 * f2) / det
    a2 = (m11 * f2 - m12 * f1) / det
    x_vel = x_vel + dt * a1
    theta_vel = theta_vel + dt * a2
    return x_pos + dt * x_vel, theta + dt * theta_vel, x_vel, theta_vel


def running_cost(x_pos, theta, x_vel, theta_vel, u0):
    """src/cartpole_mppi.py:44-50."""
    return (1.0 * x_pos ** 2 + 20.0 * (math.cos(theta) - 1.0) ** 2 + 0.1 * x_vel ** 2 + 0.1 * theta_vel ** 2
            + 0.01 * u0 ** 2)


def rollout(x0, U, noise):
    """src/cartpole_mppi.py:59-85 loop structure."""
    nu, T, K = noise.shape
    costs = np.zeros(K)
    for k in range(K):
        s = tuple(float(v) for v in x0)
        cost = 0.0
        for t in range(T):
            u = U[0, t] + noise[0, t, k]
            s = step(*s, u)
            cost += running_cost(*s, u)
        costs[k] = cost + 10.0 * running_cost(*s, 0.0)
    return costs


def mppi_step(x0, U, noise, lam=1.0):
    """src/cartpole_mppi.py:88-98 (U updated in place and returned)."""
    costs = rollout(x0, U, noise)
    beta = np.min(costs)
    weights = np.exp(-1 / lam * (costs - beta))
    weights /= np.sum(weights)
    K = noise.shape[2]
    for t in range(U.shape[1]):
        U[:, t] += sum(weights[k] * noise[:, t, k] for k in range(K))
    return U, costs
