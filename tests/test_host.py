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
