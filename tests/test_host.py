"""Host-side logic that needs no GPU: the humanoid real-env context builder vs the oracle's cost terms, and the
trajectory CSV writer vs the reference's file layout and loader."""
import os

import numpy as np

from mppi_hip.controller import SimData, humanoid_context
from oracle import mppi_ref as R

IDS = {"shin_left": 3, "shin_right": 6, "foot_left": 4, "foot_right": 7}


def _data(rs, nbody=9):
    return SimData(qpos=np.zeros(28), qvel=np.zeros(27), ctrl=np.zeros(21), xpos=rs.randn(nbody, 3),
                   cvel=rs.randn(nbody, 6))


def _expected(d):
    """Direct restatement of src/Humanoid_mppi_v3.jl:53-99 with Julia's 1-based indexing spelled out."""
    flat = d.cvel.ravel()
    vx = lambda bid: flat[(bid * 6 - 5 + 3) - 1]  # get_body_vx, :20-23
    left_swings = vx(IDS["shin_left"]) > vx(IDS["shin_right"])
    swing = IDS["foot_left"] if left_swings else IDS["foot_right"]
    stance = IDS["foot_right"] if left_swings else IDS["foot_left"]
    knee = IDS["shin_left"] if left_swings else IDS["shin_right"]
    return R.humanoid_context(swing_foot_x=d.xpos[swing, 0], swing_knee_x=d.xpos[knee, 0], swing_vx=vx(swing),
                              foot_clearance=d.xpos[swing, 2] - d.xpos[stance, 2],
                              leg_clearance=d.xpos[IDS["foot_left"], 1] - d.xpos[IDS["foot_right"], 1])


def test_humanoid_context_matches_oracle_terms():
    rs = np.random.RandomState(3)
    for _ in range(50):
        d = _data(rs)
        np.testing.assert_allclose(humanoid_context(d, IDS), _expected(d), rtol=0, atol=1e-15)


def test_humanoid_context_enters_cost_as_constant():
    rs = np.random.RandomState(4)
    d = _data(rs)
    ctx = humanoid_context(d, IDS)
    x = rs.randn(5, 55) * 0.1
    u = rs.randn(5, 21) * 0.1
    c = R.humanoid_v3_cost(x, u, ctx)
    ctx2 = ctx.copy()
    ctx2[5] += 1.0
    np.testing.assert_allclose(R.humanoid_v3_cost(x, u, ctx2) - c, 1.0, atol=1e-12)


def test_trajectory_csv_matches_reference_layout(tmp_path):
    """mppi_hip.trajectory writes the files of src/Humanoid_datacollection_v2.jl:238-249 (',' delimited, no
    header); read the way learning/data_loader.py:160-161 reads them, rows 2.. come back."""
    import pandas as pd
    from mppi_hip.trajectory import write_trajectory_csv
    rs = np.random.RandomState(0)
    T = 9
    st, ac = rs.randn(T, 4), rs.randn(T, 1)
    for layout in ("ft", "run"):
        p = write_trajectory_csv(str(tmp_path / layout), st, ac, dt=0.01, stamp="2025-01-01_000000", layout=layout)
        assert all(os.path.exists(v) for v in p.values())
        loaded = pd.read_csv(p["states"]).values.astype(np.float32)[1:]
        np.testing.assert_array_equal(loaded, st[2:].astype(np.float32))
        raw = np.loadtxt(p["states"], delimiter=",")
        np.testing.assert_array_equal(raw, st)  # full precision round trip, no header line
        np.testing.assert_allclose(np.loadtxt(p["times"]), 0.01 * np.arange(T))
        np.testing.assert_array_equal(np.loadtxt(p["actions"], delimiter=",").reshape(T, 1), ac)
    p = write_trajectory_csv(str(tmp_path / "x"), st, ac, extra_state_columns=rs.randn(T, 2))  # humanoid foot z
    assert np.loadtxt(p["states"], delimiter=",").shape == (T, 6)


# ------------------------------------------------------------------------------ humanoid context across the boundary

class _RecordingEngine:
    """Stands in for the HIP Engine (no GPU here): records the ctx each solve receives."""

    def __init__(self, nu, H):
        self.nu, self.H, self.ctx = nu, H, []

    def solve(self, x0, U, noise=None, seed=0, ctx=None, **kw):
        from mppi_hip.engine import SolveResult
        self.ctx.append(None if ctx is None else np.asarray(ctx, np.float64).copy())
        return SolveResult(U=np.asarray(U, np.float32), costs=np.zeros(4, np.float32), weights=np.zeros(4, np.float32),
                           u0=np.zeros(self.nu, np.float32))


def _model(cost):
    from mppi_hip.controller import HUMANOID_BODY_IDS, MPPIModel
    m = MPPIModel.__new__(MPPIModel)  # the reference's module state without a device handle
    m.preset, m.cost, m.noise, m.seed, m.calls, m.last = "humanoid_v3", cost, "device", 0, 0, None
    m.body_ids, m.u0_before = dict(HUMANOID_BODY_IDS), False
    m.U_global = np.zeros((21, 8))
    from types import SimpleNamespace
    m.config = SimpleNamespace(nu=21, H=8, K=4, sigma=0.75)
    m.engine = _RecordingEngine(21, 8)
    return m


def test_controller_passes_real_env_context_every_call():
    """mppi_controller / mppi_step with a data object carrying xpos / cvel pass, on every call, the context row an
    explicit humanoid_context(data, ids) gives (src/Humanoid_mppi_v3.jl:53-99 reads the global data per call); the
    v1 cost gets humanoid_v1_context; data without the kinematics leaves the engine default."""
    from mppi_hip.controller import HUMANOID_BODY_IDS, humanoid_v1_context, mppi_controller, mppi_step
    rs = np.random.RandomState(8)
    for cost, ref in (("humanoid_v3", humanoid_context), ("humanoid_v1", humanoid_v1_context)):
        m = _model(cost)
        for call in range(4):
            d = _data(rs, nbody=18)
            (mppi_controller if call % 2 else mppi_step)(m, d)
            np.testing.assert_array_equal(m.engine.ctx[-1], ref(d, HUMANOID_BODY_IDS))
        explicit = np.arange(8.0)
        mppi_controller(m, _data(rs, nbody=18), ctx=explicit)
        np.testing.assert_array_equal(m.engine.ctx[-1], explicit)
        mppi_step(m, SimData(qpos=np.zeros(28), qvel=np.zeros(27), ctrl=np.zeros(21)))
        assert m.engine.ctx[-1] is None
        # a goal given at construction (MPPIModel(ctx=...): the engine default) is kept in the per-call rows
        m.target = (3.0, -1.0, 1.1)
        d = _data(rs, nbody=18)
        mppi_step(m, d)
        np.testing.assert_array_equal(m.engine.ctx[-1][:3], m.target)
        np.testing.assert_array_equal(m.engine.ctx[-1][3:], ref(d, HUMANOID_BODY_IDS)[3:])
        np.testing.assert_array_equal(m.engine.ctx[-1], ref(d, HUMANOID_BODY_IDS, m.target))


def test_humanoid_body_ids_match_the_model_xml():
    """HUMANOID_BODY_IDS are the MuJoCo body ids of src/humanoid.xml (world 0, then <body> elements depth-first)."""
    import pytest
    import xml.etree.ElementTree as ET
    from mppi_hip.controller import HUMANOID_BODY_IDS
    path = "/root/reference/src/humanoid.xml"
    if not os.path.exists(path):
        pytest.skip("reference tree not present")
    names = ["world"]

    def walk(e):
        for b in e.findall("body"):
            names.append(b.get("name"))
            walk(b)
    walk(ET.parse(path).getroot().find("worldbody"))
    assert {n: names.index(n) for n in HUMANOID_BODY_IDS} == HUMANOID_BODY_IDS


def test_humanoid_v1_context_and_phase():
    """humanoid_v1_context carries both feet (src/Humanoid_mppi.jl:89-106); the oracle's cost picks the swing foot
    by the 1-based rollout step (phase = t % 100 < 50: left, :76-87) and flips the sign of the 0.01 dz term."""
    from mppi_hip.controller import HUMANOID_BODY_IDS, humanoid_v1_context
    rs = np.random.RandomState(5)
    d = _data(rs, nbody=18)
    ctx = humanoid_v1_context(d, HUMANOID_BODY_IDS)
    fl, fr = d.xpos[HUMANOID_BODY_IDS["foot_left"]], d.xpos[HUMANOID_BODY_IDS["foot_right"]]
    np.testing.assert_allclose(ctx, R.humanoid_v1_context(fl, fr), atol=1e-15)
    x = rs.randn(6, 55) * 0.1
    u = rs.randn(6, 21) * 0.1
    px = x[:, 0]
    base = R.humanoid_v1_cost(x, u, ctx, 1) - 10 * (fl[0] - px - 0.5) ** 2 - ctx[5]
    for t, left in ((1, True), (49, True), (50, False), (99, False), (100, True), (149, True), (150, False)):
        sw = fl[0] if left else fr[0]
        exp = base + 10 * (sw - px - 0.5) ** 2 + (ctx[5] if left else -ctx[5])
        np.testing.assert_allclose(R.humanoid_v1_cost(x, u, ctx, t), exp, rtol=1e-12, atol=1e-12)
