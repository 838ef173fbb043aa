"""Drop-in mirror of the reference controller API, backed by the HIP engine.

The reference scripts keep their state in module globals (U_global, K, T, lambda, sigma) next to a MuJoCo
model; the functions below keep the same names, argument meaning and update semantics, with the globals
gathered into an MPPIModel:

  rollout(model, data, U, noise) -> costs[K]     src/cartpole_mppi.py:59-85, src/Humanoid_mppi_v3.jl:128-152
  mppi_step(model, data)                          src/cartpole_mppi.py:88-98, src/Humanoid_mppi_v3.jl:154-171
  mppi_controller(model, data)                    src/cartpole_mppi.py:101-106, src/Humanoid_mppi_v3.jl:173-179
  mppi_update(model, data)                        src/mppi.jl:83-99 / src/quadruped_datacollection.py:166-187
  rollout_learned_model_batched(model, state, U, noise, device=None) -> costs
                                                  src/cartpole_mppi_estimator.py:61-121

`data` is anything with numpy attributes qpos, qvel, ctrl (a mujoco.MjData, or SimData below).  For the humanoid
costs the reference reads the REAL environment's kinematics (data.xpos, data.cvel) on every call
(src/Humanoid_mppi_v3.jl:53-99, src/Humanoid_mppi.jl:89-106); when `data` carries them, mppi_step /
mppi_controller build the per-solve context row from them on every call, as the reference does.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .engine import Config, Engine
from .nets import cross_attention_blob, feature_attention_blob, mlp_blob

# default cost of each preset (the reference script it mirrors)
PRESET_COST = {"cartpole_py": "cartpole", "cartpole_jl": "cartpole", "cartpole_collect": "cartpole",
               "quad_mppi_jl": "quad_jl", "humanoid_v3": "humanoid_v3", "humanoid_v1": "humanoid_v1",
               "humanoid_collect_v2": "humanoid_v3", "cartpole_est": "cartpole_est", "quad_est": "quad_est"}


@dataclass
class SimData:
    """Minimal stand-in for mujoco.MjData: the fields the controllers read and write."""
    qpos: np.ndarray
    qvel: np.ndarray
    ctrl: np.ndarray
    xpos: np.ndarray | None = None
    cvel: np.ndarray | None = None


class MPPIModel:
    """The reference script's module-level state for one controller, plus the engine handle.

    dynamics: "cartpole" (analytic mj_step restatement), ("cross_attention", state_dict[, dims dict]),
              ("feature_attention", state_dict[, dims dict]) or ("mlp", state_dict[, dims dict]).
    noise:    "device" -> Philox on the GPU (seeded, advances per call);
              "numpy"  -> np.random.randn(nu,T,K)*sigma from numpy's global RNG, exactly the reference's draw
                          (src/cartpole_mppi.py:89), injected into the engine.
    """

    def __init__(self, preset: str = "cartpole_py", dynamics="cartpole", cost: str | None = None, device: int = 0,
                 noise: str = "device", seed: int = 0, precision: int = L.PREC_BF16, ctx=None,
                 body_ids: dict | None = None, u0_before: bool = False, **overrides):
        """body_ids: 0-based MuJoCo body ids of HUMANOID_BODIES (default: src/humanoid.xml's, HUMANOID_BODY_IDS)
        for the per-call humanoid context; u0_before: apply U[:,0] before the update
        (src/quadruped_datacollection.py:170, MPPI_FLAG_U0_BEFORE)."""
        self.preset = preset
        self.body_ids = dict(HUMANOID_BODY_IDS if body_ids is None else body_ids)
        self.u0_before = bool(u0_before)
        self.config = Config.preset(preset, precision=precision, **overrides)
        self.engine = Engine(self.config, device)
        if isinstance(dynamics, str) and dynamics == "cartpole":
            self.engine.load_dynamics(L.DYN_CARTPOLE)
        else:
            kind, sd = dynamics[0], dynamics[1]
            dims = dynamics[2] if len(dynamics) > 2 else {}
            if kind == "cross_attention":
                k, blob = cross_attention_blob(sd, **dims)
            elif kind == "mlp":
                k, blob = mlp_blob(sd, state_dim=self.config.nx, action_dim=self.config.nu, **dims)
            elif kind == "feature_attention":
                dims = {"hidden_dim": np.asarray(sd["feature_encoding.0.weight"]).shape[0], **dims}
                k, blob = feature_attention_blob(sd, state_dim=self.config.nx, action_dim=self.config.nu, **dims)
            else:
                raise ValueError(f"unknown dynamics {kind!r}")
            self.engine.load_dynamics(k, blob)
        self.cost = cost or PRESET_COST[preset]
        self.engine.set_cost(self.cost, ctx)
        # the humanoid goal (ctx[0:3]) the per-call real-env context keeps: the caller's, when one was given
        self.target = tuple(float(v) for v in np.asarray(ctx, np.float64).ravel()[:3]) if ctx is not None \
            else HUMANOID_TARGET
        self.U_global = np.zeros((self.config.nu, self.config.H))
        self.noise = noise
        self.seed = int(seed)
        self.calls = 0
        self.last = None  # SolveResult of the last mppi_step (costs, weights) for inspection

    @property
    def K(self):
        return self.config.K

    @property
    def T(self):
        return self.config.H

    def draw_noise(self):
        c = self.config
        if self.noise == "numpy":
            return np.random.randn(c.nu, c.H, c.K) * c.sigma
        return None

    def next_seed(self) -> int:
        self.calls += 1
        return (self.seed << 32) ^ self.calls

    def close(self):
        self.engine.close()


HUMANOID_TARGET = (2.0, 0.0, 1.28)  # const Position, src/Humanoid_mppi_v3.jl:12
HUMANOID_BODIES = ("shin_left", "shin_right", "foot_left", "foot_right")
# MuJoCo body ids of src/humanoid.xml (world = 0, then the <body> elements depth-first: torso 1, head 2,
# waist_lower 3, pelvis 4, thigh_right 5, shin_right 6, foot_right 7, thigh_left 8, shin_left 9, foot_left 10, ...;
# 18 bodies).  tests/test_host.py checks them against the XML when the reference tree is present.
HUMANOID_BODY_IDS = {"shin_left": 9, "shin_right": 6, "foot_left": 10, "foot_right": 7}


def humanoid_body_ids(mjmodel) -> dict:
    """0-based MuJoCo body ids (what MuJoCo.body(model, name).id returns), via the mujoco Python bindings."""
    import mujoco
    return {n: mujoco.mj_name2id(mjmodel, mujoco.mjtObj.mjOBJ_BODY, n) for n in HUMANOID_BODIES}


def humanoid_context(data, body_ids: dict, target=HUMANOID_TARGET) -> np.ndarray:
    """Per-solve context row (MPPI_CTX_MAX floats) for MPPI_COST_HUMANOID_V3 from the REAL environment's data.

    src/Humanoid_mppi_v3.jl:53-99 reads the global `data` (not the rollout copy), so these terms are constant
    over all k and t of one solve: [tx, ty, tz, swing_foot_x, swing_knee_x, const, 0, 0] with
    const = -0.15*swing_vx + 2*clr^2 [clr < 0.05] + 0.5*lat^2 [lat < 0].
    get_body_vx (:20-23) indexes the flat cvel buffer at 6*id-5+3 (1-based) with a 0-based id, i.e. it reads
    the linear-x velocity of body id-1; that behaviour is kept here.
    """
    cvel = np.asarray(data.cvel, np.float64).ravel()
    xpos = np.asarray(data.xpos, np.float64).reshape(-1, 3)

    def vx(bid):
        return cvel[6 * bid - 5 + 3 - 1]

    il, ir = body_ids["shin_left"], body_ids["shin_right"]
    if vx(il) > vx(ir):
        swing, stance, knee = body_ids["foot_left"], body_ids["foot_right"], il
    else:
        swing, stance, knee = body_ids["foot_right"], body_ids["foot_left"], ir
    const = -0.15 * vx(swing)
    clearance = xpos[swing, 2] - xpos[stance, 2]
    if clearance < 0.05:
        const += 2.0 * clearance ** 2
    lateral = xpos[body_ids["foot_left"], 1] - xpos[body_ids["foot_right"], 1]
    if lateral < 0:
        const += 0.5 * lateral ** 2
    ctx = np.zeros(L.CTX_MAX)
    ctx[:6] = [target[0], target[1], target[2], xpos[swing, 0], xpos[knee, 0], const]
    return ctx


def humanoid_v1_context(data, body_ids: dict, target=HUMANOID_TARGET) -> np.ndarray:
    """Per-solve context row for MPPI_COST_HUMANOID_V1 (src/Humanoid_mppi.jl:31-121) from the REAL environment's
    data.xpos: [2, 0, 1.28, left_foot_x, right_foot_x, 0.01 (right_z - left_z), 0.1 |left_y - right_y|, 0].
    The kernel picks the swing side per rollout step (t % 100 < 50: left swings, :76-87)."""
    xpos = np.asarray(data.xpos, np.float64).reshape(-1, 3)
    fl, fr = xpos[body_ids["foot_left"]], xpos[body_ids["foot_right"]]
    ctx = np.zeros(L.CTX_MAX)
    ctx[:7] = [target[0], target[1], target[2], fl[0], fr[0], 0.01 * (fr[2] - fl[2]), 0.1 * abs(fl[1] - fr[1])]
    return ctx


def env_context(model: "MPPIModel", data):
    """The per-call cost context the reference reads from the real environment, or None (engine default) when the
    cost has no real-env terms or `data` does not carry the kinematics (xpos / cvel).  The goal position ctx[0:3] is
    the model's (MPPIModel(ctx=...) at construction, else HUMANOID_TARGET), not replaced per call."""
    target = getattr(model, "target", HUMANOID_TARGET)
    if model.cost == "humanoid_v3" and getattr(data, "xpos", None) is not None and \
            getattr(data, "cvel", None) is not None:
        return humanoid_context(data, model.body_ids, target)
    if model.cost == "humanoid_v1" and getattr(data, "xpos", None) is not None:
        return humanoid_v1_context(data, model.body_ids, target)
    return None


def _state(data) -> np.ndarray:
    return np.concatenate([np.asarray(data.qpos, np.float64).ravel(), np.asarray(data.qvel, np.float64).ravel()])


def rollout(model: MPPIModel, data, U, noise) -> np.ndarray:
    """costs[K] of the K perturbed sequences U + noise[:, :, k] from data's state (no U update)."""
    state = _state(data)
    res = model.engine.solve(state, np.asarray(U), noise=np.asarray(noise), want_costs=True)
    return res.costs.astype(np.float64)


def rollout_learned_model_batched(model: MPPIModel, state, U, noise, device=None) -> np.ndarray:
    """Estimator form (src/cartpole_mppi_estimator.py:61): same as rollout() but takes the state vector."""
    if hasattr(noise, "detach"):
        noise = noise.detach().cpu().numpy()
    res = model.engine.solve(np.asarray(state, np.float64), np.asarray(U), noise=np.asarray(noise), want_costs=True)
    return res.costs.astype(np.float64)


def mppi_step(model: MPPIModel, data, ctx=None):
    """noise -> rollout -> softmin -> U_global update (add or replace per preset), in place.  ctx None: built from
    data's real-env kinematics for the humanoid costs (env_context), as the reference reads them per call."""
    ctx = env_context(model, data) if ctx is None else ctx
    noise = model.draw_noise()
    res = model.engine.solve(_state(data), model.U_global, noise=noise, seed=model.next_seed(), ctx=ctx,
                             want_costs=True, want_weights=True)
    model.U_global = res.U.astype(np.float64)
    model.last = res
    return res


def mppi_controller(model: MPPIModel, data, ctx=None):
    """mppi_step, then data.ctrl = U[:,0] and the receding-horizon shift (fill = preset's 0.1 or 0)."""
    ctx = env_context(model, data) if ctx is None else ctx
    noise = model.draw_noise()
    res = model.engine.solve(_state(data), model.U_global, noise=noise, seed=model.next_seed(), ctx=ctx,
                             want_costs=True, want_weights=True, shift=True, u0_before=model.u0_before)
    model.U_global = res.U.astype(np.float64)
    model.last = res
    data.ctrl[:] = res.u0
    return res


mppi_update = mppi_controller  # src/mppi.jl:83-99 names the same step mppi_update!
