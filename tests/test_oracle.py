"""The oracle (CPU restatement of the reference hot path) checked against the reference's golden vectors.
CPU-only: these run in the build container and on the GPU box."""
import numpy as np
import pytest

from conftest import golden, golden_sd
from oracle import mppi_ref as R
from oracle import nets_ref as N


def test_cartpole_step_reproduces_mujoco_trajectory():
    """G1: data/2025-04-21_011138 was produced by mujoco.mj_step on models/cartpole.xml (dt=0.01)."""
    g = golden("g1_cartpole_kat.npz")
    st, ac = g["states"], g["actions"]
    assert st.shape == (1018, 4) and ac.shape == (1018, 1)
    pred = R.cartpole_step(st[:-1], ac[:-1])
    assert np.max(np.abs(pred - st[1:])) < 1e-15


def test_cartpole_constants_match_mujoco_compile():
    p = R.CARTPOLE
    assert p["m_cart"] == pytest.approx(8.0)
    assert p["m_pole"] == pytest.approx(4.198738581522758, rel=1e-14)
    assert p["inertia"] == pytest.approx(0.15497066975016233, rel=1e-12)


def test_ca_humanoid_forward_matches_reference_module():
    """G5: learning/model.py CrossAttentionStatePredictor + checkpoints/model_cross.pth."""
    g = golden("g5_ca_humanoid_fwd.npz")
    sd = golden_sd("ca_humanoid_weights.npz")
    y = N.ca_forward(sd, g["x"].astype(np.float64), 28, 27)
    np.testing.assert_allclose(y, g["y"], rtol=2e-5, atol=2e-5)


def test_ca_fold_is_exact():
    g = golden("g5_ca_humanoid_fwd.npz")
    sd = golden_sd("ca_humanoid_weights.npz")
    x = g["x"].astype(np.float64)
    y_unf = N.ca_forward(sd, x, 28, 27)
    y_fold = N.fcstack_forward(N.ca_fold(sd, 28, 27, 21), x)
    assert np.max(np.abs(y_unf - y_fold)) < 1e-10
    # the action never reaches the output (dead action encoder, learning/model.py:168,192)
    x2 = x.copy()
    x2[:, 55:] = 7.0
    assert np.array_equal(N.fcstack_forward(N.ca_fold(sd, 28, 27, 21), x2), y_fold)


def test_ln_fold_is_exact():
    """The engine's LayerNorm fold (centred layer 0, gamma in layer 1) equals the reference net in fp64, also with
    negative and zero gammas (synthetic) -- oracle/nets_ref.py::ln_fold, mppi_nets.cpp CROSS_ATTN."""
    g = golden("g5_ca_humanoid_fwd.npz")
    sd = golden_sd("ca_humanoid_weights.npz")
    x = g["x"].astype(np.float64)
    stack = N.ca_fold(sd, 28, 27, 21)
    y = N.fcstack_forward(stack, x)
    assert np.max(np.abs(N.fcstack_forward(N.ln_fold(stack), x) - y)) < 1e-10
    gam, bet = stack[0]["ln"]
    gam = gam.copy()
    gam[::7] *= -1.0
    gam[3::11] = 0.0
    st2 = [dict(stack[0], ln=(gam, bet))] + stack[1:]
    y2 = N.fcstack_forward(st2, x)
    assert np.max(np.abs(N.fcstack_forward(N.ln_fold(st2), x) - y2)) < 1e-10


def test_ca_cartpole_forward_matches_reference_module():
    g = golden("g5_ca_cartpole_fwd.npz")
    sd = golden_sd("ca_cartpole_weights.npz")
    np.testing.assert_allclose(N.ca_forward(sd, g["x"].astype(np.float64), 2, 2, nheads=6), g["y"], rtol=1e-5,
                               atol=1e-6)


def test_fa_forward_matches_reference_module():
    g = golden("g3_fa_cartpole_fwd.npz")
    sd = golden_sd("fa_cartpole_weights.npz")
    np.testing.assert_allclose(N.fa_forward(sd, g["x"].astype(np.float64), 4, 4), g["y"], rtol=1e-5, atol=1e-6)
    g = golden("g8_fa_quad64_fwd.npz")
    sd = {k[2:]: v for k, v in g.items() if k.startswith("w.")}
    np.testing.assert_allclose(N.fa_forward(sd, g["x"].astype(np.float64), 37, 4), g["y"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", ["humanoid", "quad"])
def test_mlp_forward_matches_reference_module(name):
    g = golden(f"g8_mlp_{name}_fwd.npz")
    sd = {k[2:]: v for k, v in g.items() if k.startswith("w.")}
    np.testing.assert_allclose(N.mlp_forward(sd, g["x"].astype(np.float64)), g["y"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(N.fcstack_forward(N.mlp_stack(sd), g["x"]), g["y"], rtol=1e-5, atol=1e-6)


def test_estimator_fa_cartpole_solve_matches_fixture():
    """G4: estimator loop (src/cartpole_mppi_estimator.py:61-143) around the reference FA net."""
    g = golden("g4_fa_cartpole_solve.npz")
    sd = golden_sd("fa_cartpole_weights.npz")
    pre = R.Preset("g4", K=int(g["K"]), H=int(g["T"]), lam=float(g["lam"]), sigma=0.5, update="replace")

    def dyn(x, u):
        return x + N.fa_forward(sd, np.concatenate([x, u], axis=-1), 4, 4)
    out = R.mppi_solve(pre, dyn, R.cartpole_est_running_cost, g["x0"], g["U0"], g["noise"])
    np.testing.assert_allclose(out["costs"], g["costs"], rtol=1e-4)
    np.testing.assert_allclose(out["U_new"], g["U_new"], atol=1e-5)


def test_humanoid_ca_solve_matches_fixture():
    """G7: Humanoid_mppi_v3 loop with x+ = x + CA(x,u), cost restated independently in torch."""
    g = golden("g7_ca_humanoid_solve.npz")
    sd = golden_sd("ca_humanoid_weights.npz")
    pre = R.Preset("g7", K=int(g["K"]), H=int(g["H"]), lam=float(g["lam"]), sigma=0.75)
    dyn = N.learned_dynamics(N.ca_fold(sd, 28, 27, 21), 55)
    out = R.mppi_solve(pre, dyn, R.humanoid_v3_cost, g["x0"], g["U0"], g["noise"], ctx=g["ctx"].astype(np.float64))
    np.testing.assert_allclose(out["costs"], g["costs"], rtol=2e-4)
    np.testing.assert_allclose(out["weights"], g["weights"], atol=2e-4)
    np.testing.assert_allclose(out["U_new"], g["U_new"], atol=2e-4)


def test_softmin_update_shift_semantics():
    pre = R.PRESETS["cartpole_py"]
    c = np.array([3.0, 1.0, 2.0, np.nan])
    w = R.softmin_weights(c, 1.0)
    assert w[3] == 0.0 and w.sum() == pytest.approx(1.0)
    assert w[1] == pytest.approx(1.0 / (1.0 + np.exp(-1.0) + np.exp(-2.0)))
    U = np.arange(6, dtype=float).reshape(1, 6)
    u0, Us = R.shift_U(pre, U)
    assert u0[0] == 0.0 and list(Us[0]) == [1, 2, 3, 4, 5, 0.5]
    u0, Us = R.shift_U(R.PRESETS["quad_mppi_jl"], U)
    assert Us[0, -1] == 0.0
    noise = np.ones((1, 6, 4))
    Un = R.update_U(R.PRESETS["quad_mppi_jl"], U * 10, noise, np.full(4, 0.25))
    assert Un.max() == 10.0  # clamped to +-10 (src/mppi.jl:93)


def test_serial_port_matches_vectorised_oracle():
    """oracle/cartpole_serial.py (the reference's per-sample loop shape) == the batched restatement."""
    from oracle import cartpole_serial as S
    pre = R.PRESETS["cartpole_py"]
    noise = R.reference_noise(0, 1, 30, 16, 1.0)
    x0 = np.array([0.0, 0.3, 0.0, 0.0])
    U = np.zeros((1, 30))
    c_serial = S.rollout(x0, U, noise)
    c_vec = R.rollout(pre, R.cartpole_step, R.cartpole_running_cost, x0, U, noise)
    np.testing.assert_allclose(c_serial, c_vec, rtol=1e-13)


def test_bf16_round_is_rne():
    x = np.array([1.0, 1.00390625, 1.005859375, -2.5, 3.0e38], np.float32)
    r = R.bf16_round(x)
    assert r[0] == 1.0 and r[1] == 1.0 and r[2] == np.float32(1.0078125) and r[3] == -2.5


def test_torch_ports_match_fixtures():
    """The CPU-baseline torch ports (oracle/torch_port.py) compute what the reference modules compute."""
    import torch
    from oracle import torch_port as T
    sd = golden_sd("fa_cartpole_weights.npz")
    net = T.FeatureAttentionPort(sd, 4)
    g = golden("g3_fa_cartpole_fwd.npz")
    with torch.no_grad():
        np.testing.assert_allclose(net(torch.from_numpy(g["x"]).float()).numpy(), g["y"], rtol=1e-5, atol=1e-6)
    g = golden("g4_fa_cartpole_solve.npz")
    U, c = T.mppi_solve_estimator_torch(net, g["x0"], torch.from_numpy(g["U0"]), torch.from_numpy(g["noise"]),
                                        T.cartpole_est_cost_torch)
    np.testing.assert_allclose(c.numpy(), g["costs"], rtol=1e-5)
    np.testing.assert_allclose(U.numpy(), g["U_new"], atol=1e-6)
    sd = golden_sd("ca_humanoid_weights.npz")
    g = golden("g5_ca_humanoid_fwd.npz")
    with torch.no_grad():
        y = T.CrossAttentionPort(sd)(torch.from_numpy(g["x"][:64]).float()).numpy()
    np.testing.assert_allclose(y, g["y"][:64], rtol=2e-5, atol=2e-5)


def test_costs_match_reference_functions_g6():
    """G6: the reference's own running_cost / terminal_cost functions (tests/golden/gen_fixtures_ref_loop.py ran
    them from src/cartpole_mppi.py:44-53, src/cartpole_mppi_estimator.py:46-55, src/quadruped_mppi_estimator.py:
    48-55) on seeded states; the oracle's cost restatements reproduce them."""
    g = golden("g6_cost_kat.npz")
    X, Uc = g["cp_x"], g["cp_u"]
    np.testing.assert_allclose(R.cartpole_running_cost(X, Uc), g["cp_running"], rtol=1e-14)
    np.testing.assert_allclose(10.0 * R.cartpole_running_cost(X, np.zeros_like(Uc)), g["cp_terminal"], rtol=1e-14)
    Xf = X.astype(np.float32)
    np.testing.assert_allclose(R.cartpole_est_running_cost(Xf, Uc), g["cpe_running"], rtol=2e-6)
    np.testing.assert_allclose(10.0 * R.cartpole_est_running_cost(Xf, None), g["cpe_terminal"], rtol=2e-6)
    S, C = g["q_state"], g["q_ctrl"]
    np.testing.assert_allclose(R.quad_est_running_cost(S, C), g["q_running"], rtol=2e-6)
    np.testing.assert_allclose(10.0 * R.quad_est_running_cost(S, np.zeros_like(C)), g["q_terminal"], rtol=2e-6)


def test_cartpole_solve_matches_reference_loop_g2():
    """G2: the reference's own mppi_step / mppi_controller (src/cartpole_mppi.py:88-106: noise draw, softmin,
    generator-sum update, u0, decay shift) around the oracle rollout; BASELINE configs #1 and #2 shapes."""
    g = golden("g2_cartpole_solve.npz")
    for ci in range(int(g["n_cases"])):
        p = f"c{ci}_"
        K, T = int(g[p + "K"]), int(g[p + "T"])
        noise = R.reference_noise(int(g[p + "seed"]), 1, T, K, 1.0)
        ref = R.mppi_solve(R.Preset("g2", K=K, H=T, lam=1.0, sigma=1.0), R.cartpole_step, R.cartpole_running_cost,
                           g[p + "x0"], g[p + "U0"], noise)
        np.testing.assert_allclose(ref["costs"], g[p + "costs"], rtol=1e-12)
        np.testing.assert_allclose(ref["U_new"], g[p + "U_new"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(ref["u0"], g[p + "u0"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(ref["U_shifted"], g[p + "U_shifted"], rtol=1e-10, atol=1e-12)


def _shape_fixture(name):
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("gen_fixtures_shapes", os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "golden", "gen_fixtures_shapes.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod, mod.SHAPES[name], golden(name + ".npz")


def test_mlp_batchnorm_forward_matches_reference_module():
    """MLPStatePredictor(55, 21, 512, use_batch_norm=True, dropout 0.2, hidden_layers=6) (learning/train.py:70) in eval
    mode: the oracle's forward and its BatchNorm-folded fc stack (the engine's form) against the reference module's
    outputs (tests/golden/gen_fixtures_shapes.py), rtol 1e-5."""
    mod, spec, g = _shape_fixture("g9_mlp_bn_fwd")
    sd = mod.weights(spec)
    np.testing.assert_allclose(N.mlp_forward(sd, g["x"]), g["y"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(N.fcstack_forward(N.mlp_stack(sd), g["x"]), g["y"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["g9_fa_h8l7_fwd", "g9_fa76_fwd"])
def test_fa_general_shapes_match_reference_module(name):
    """FeatureAttentionStatePredictor at 8 heads x 7 layers, hidden 512, 51 tokens (learning/train.py:71-72) and at
    76 tokens (learning/model.py:215): the oracle's forward vs the reference module's, rtol 1e-4."""
    mod, spec, g = _shape_fixture(name)
    sd = mod.weights(spec)
    y = N.fa_forward(sd, g["x"].astype(np.float64), int(spec["nx"]), int(spec["heads"]))
    np.testing.assert_allclose(y, g["y"], rtol=1e-4, atol=2e-5)
