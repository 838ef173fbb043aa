"""HIP engine vs the oracle, through the C-ABI (libmppi_hip.so). Needs an MI355X.

Tolerances (fp32 engine vs fp64 oracle), written per test:
  analytic cartpole: costs rtol 1e-5, weights atol 1e-5, U atol 1e-4
  learned fp32 (exact-f32 MFMA): costs rtol 1e-4, U atol 1e-4
  learned bf16: vs the bf16-emulating oracle costs rtol 5e-3; vs the fp32 oracle U atol 2e-2
End-to-end U is compared when the softmin is well conditioned (oracle weights of the engine's costs within
1e-3 of the oracle weights); otherwise the engine's own weights are checked against its costs and the U update
against its weights (the "tie guard" of SURVEY 8d).
"""
import ctypes

import os

import numpy as np
import pytest

from conftest import golden, golden_sd
from oracle import mppi_ref as R
from oracle import nets_ref as N
from philox_ref import device_noise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(gpu_available):
    import mppi_hip
    return mppi_hip


def _engine(M, preset, **kw):
    from mppi_hip import _lib as L
    cfg = M.Config.preset(preset, **kw)
    return M.Engine(cfg)


def _check_solve(res, ref, pre, U0, noise, cost_rtol, u_atol, w_atol=1e-5):
    """res: SolveResult (single solve, shifted=False); ref: oracle mppi_solve dict."""
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=cost_rtol, atol=cost_rtol * 1e-3)
    # softmin of the engine's own costs
    w_own = R.softmin_weights(res.costs.astype(np.float64), pre.lam, pre.norm_eps)
    np.testing.assert_allclose(res.weights, w_own, atol=w_atol)
    # the reduce/update applied to the engine's weights
    U_own = R.update_U(pre, np.asarray(U0, np.float64), np.asarray(noise, np.float64), res.weights.astype(np.float64))
    np.testing.assert_allclose(res.U, U_own, atol=1e-5)
    # end to end, when well conditioned
    if np.max(np.abs(w_own - ref["weights"])) < 1e-3:
        np.testing.assert_allclose(res.U, ref["U_new"], atol=u_atol)


# ------------------------------------------------------------------------------------------ cartpole

@pytest.mark.parametrize("K,H", [(128, 30), (4096, 50), (30, 100), (75, 17)])
@pytest.mark.parametrize("theta0", [0.0, np.pi])
@pytest.mark.parametrize("warm", [False, True])
def test_cartpole_matches_oracle(M, K, H, theta0, warm):
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=1.0)
    eng = _engine(M, "cartpole_py", K=K, H=H, precision=0)
    eng.load_dynamics(1).set_cost("cartpole")
    noise = R.reference_noise(K + H, 1, H, K, 1.0)
    x0 = np.array([0.05, theta0, 0.0, 0.0])
    U0 = 0.3 * np.sin(np.arange(H))[None, :] if warm else np.zeros((1, H))
    ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0, U0, noise)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    _check_solve(res, ref, pre, U0, noise, cost_rtol=1e-5, u_atol=1e-4)
    eng.close()


@pytest.mark.parametrize("ci", range(8))
def test_cartpole_reference_loop_fixture_g2(M, ci):
    """G2 (tests/golden/gen_fixtures_ref_loop.py): the reference's own mppi_step + mppi_controller
    (src/cartpole_mppi.py:88-106) on its own seeded noise, BASELINE configs #1 (K=128 T=30) and #2 (K=4096 T=50).
    Engine fp32 with the injected noise: costs rtol 1e-5; U_new, u0 and the shifted U atol 1e-4."""
    g = golden("g2_cartpole_solve.npz")
    p = f"c{ci}_"
    K, T = int(g[p + "K"]), int(g[p + "T"])
    noise = R.reference_noise(int(g[p + "seed"]), 1, T, K, 1.0)
    eng = _engine(M, "cartpole_py", K=K, H=T, precision=0)
    eng.load_dynamics(1).set_cost("cartpole")
    res = eng.solve(g[p + "x0"], g[p + "U0"], noise=noise, shift=True, want_weights=True)
    np.testing.assert_allclose(res.costs, g[p + "costs"], rtol=1e-5)
    pre = R.Preset("g2", K=K, H=T, lam=1.0, sigma=1.0)
    w_own = R.softmin_weights(res.costs.astype(np.float64), 1.0)
    w_ref = R.softmin_weights(g[p + "costs"], 1.0)
    # the engine's reduce + update + shift applied to its own weights (always exact to fp32)
    u0_own, Us_own = R.shift_U(pre, R.update_U(pre, g[p + "U0"], noise, res.weights.astype(np.float64)))
    np.testing.assert_allclose(res.u0, u0_own, atol=1e-5)
    np.testing.assert_allclose(res.U, Us_own, atol=1e-5)
    # end to end against the reference loop; the tie guard of SURVEY 8d: with peaked weights (theta0 = pi) fp32 cost
    # rounding moves the softmin weights, and U then moves by at most sum_k |w_own - w_ref|_k |eps_t,k| (added to the
    # 1e-4 fp32 tolerance; the U the engine computes from its own weights is checked to 1e-5 above)
    atol = 1e-4 + float(np.max(np.einsum("utk,k->ut", np.abs(noise), np.abs(w_own - w_ref))))
    np.testing.assert_allclose(res.u0, g[p + "u0"], atol=atol)
    np.testing.assert_allclose(res.U, g[p + "U_shifted"], atol=atol)
    eng.close()


def test_cartpole_controller_shift_and_u0(M):
    K, H = 256, 40
    pre = R.PRESETS["cartpole_py"]
    eng = _engine(M, "cartpole_py", K=K, H=H)
    eng.load_dynamics(1).set_cost("cartpole")
    noise = R.reference_noise(3, 1, H, K, 1.0)
    x0 = np.array([0.0, 0.2, 0.1, 0.0])
    U0 = np.linspace(-0.5, 0.5, H)[None, :]
    ref = R.mppi_solve(R.Preset("t", K=K, H=H, lam=1.0, sigma=1.0), R.cartpole_step, R.cartpole_running_cost, x0, U0,
                       noise)
    res = eng.solve(x0, U0, noise=noise, shift=True, want_weights=True)
    U_new = R.update_U(pre, U0, noise, res.weights.astype(np.float64))
    u0, Us = R.shift_U(pre, U_new)
    np.testing.assert_allclose(res.u0, u0, atol=1e-5)
    np.testing.assert_allclose(res.U, Us, atol=1e-5)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-5)


def test_cartpole_batched_solves_are_independent(M):
    K, H, B = 512, 25, 5
    eng = _engine(M, "cartpole_py", K=K, H=H, max_batch=8)
    eng.load_dynamics(1).set_cost("cartpole")
    rs = np.random.RandomState(1)
    x0 = np.stack([[0.0, th, 0.0, 0.0] for th in np.linspace(0, np.pi, B)])
    U0 = 0.2 * rs.randn(B, 1, H)
    noise = rs.randn(B, 1, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=1.0)
    for b in range(B):
        ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0[b], U0[b], noise[b])
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=1e-5)
        U_own = R.update_U(pre, U0[b], noise[b], res.weights[b].astype(np.float64))
        np.testing.assert_allclose(res.U[b], U_own, atol=1e-5)


def test_cartpole_device_philox_noise(M):
    """Device noise == numpy Philox restatement (same counters); solve is deterministic per seed."""
    K, H, seed = 1024, 20, 0x1234_5678_9ABC
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=1.0)
    eng = _engine(M, "cartpole_py", K=K, H=H)
    eng.load_dynamics(1).set_cost("cartpole")
    x0 = np.array([0.0, 0.4, 0.0, 0.0])
    U0 = np.zeros((1, H))
    r1 = eng.solve(x0, U0, seed=seed, want_weights=True)
    r2 = eng.solve(x0, U0, seed=seed, want_weights=True)
    r3 = eng.solve(x0, U0, seed=seed + 1)
    assert np.array_equal(r1.U, r2.U) and np.array_equal(r1.costs, r2.costs)
    assert not np.array_equal(r1.costs, r3.costs)
    noise = device_noise(seed, 1, 1, H, K, 1.0)[0]
    assert abs(noise.mean()) < 0.02 and abs(noise.std() - 1.0) < 0.02
    ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0, U0, noise)
    np.testing.assert_allclose(r1.costs, ref["costs"], rtol=2e-5)
    U_own = R.update_U(pre, U0, noise, r1.weights.astype(np.float64))
    np.testing.assert_allclose(r1.U, U_own, atol=2e-5)


def test_cartpole_colmajor_layout(M):
    """Julia Array layouts (MPPI_FLAG_COLMAJOR): U (nu,H) and noise (nu,H,K) column-major."""
    K, H = 128, 30
    eng = _engine(M, "cartpole_jl", K=K, H=H)
    eng.load_dynamics(1).set_cost("cartpole")
    noise = R.reference_noise(9, 1, H, K, 1.0)
    x0 = np.array([0.0, np.pi, 0.0, 0.0])
    U0 = 0.1 * np.arange(H, dtype=float)[None, :] / H
    a = eng.solve(x0, U0, noise=noise)
    b = eng.solve(x0, U0.T.copy(), noise=np.transpose(noise, (2, 1, 0)).copy(), colmajor=True)
    np.testing.assert_array_equal(a.costs, b.costs)
    np.testing.assert_array_equal(a.U, b.U.T)


def test_quad_clamp_and_zero_fill_semantics(M):
    """mppi.jl variant on the cartpole plant: ctrl clamp, U clamp, +1e-10, zero-fill shift."""
    K, H = 64, 12
    eng = M.Engine(M.Config(nx=4, nu=1, H=H, K=K, lambda_=0.2, sigma=0.3, ctrl_clamp=0.5, U_clamp=0.4,
                            norm_eps=1e-10, shift_fill=0.0, terminal_weight=0.0))
    eng.load_dynamics(1).set_cost("cartpole")
    pre = R.Preset("t", K=K, H=H, lam=0.2, sigma=0.3, ctrl_clamp=0.5, U_clamp=0.4, norm_eps=1e-10, shift_fill=0.0,
                   terminal_weight=0.0)
    noise = R.reference_noise(5, 1, H, K, 2.0)
    x0 = np.array([0.0, 0.1, 0.0, 0.0])
    U0 = np.full((1, H), 0.35)
    ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0, U0, noise)
    res = eng.solve(x0, U0, noise=noise, shift=True, want_weights=True)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-5)
    Un = R.update_U(pre, U0, noise, res.weights.astype(np.float64))
    assert np.abs(Un).max() <= 0.4 + 1e-7
    u0, Us = R.shift_U(pre, Un)
    np.testing.assert_allclose(res.U, Us, atol=1e-5)
    assert res.U[0, -1] == 0.0


def test_cartpole_fused_epilogue_replace_clamp_ragged(M):
    """The analytic cartpole finishes its solve inside the rollout (block softmin partials, last-block combine and
    update): replace-mode update, U clamp, u0 taken before the update, zero-eps weights, B = 3 solves, K = 300 over
    two 256-sample blocks (the second one ragged), the cartpole_est cost.  Costs rtol 1e-5 vs the oracle; weights vs
    the softmin of the engine's costs atol 1e-5; U vs the update + shift of those weights atol 1e-5."""
    K, H, B = 300, 23, 3
    eng = M.Engine(M.Config(nx=4, nu=1, H=H, K=K, lambda_=0.5, sigma=0.8, U_clamp=0.6, update_mode=1, shift_fill=0.1,
                            terminal_weight=10.0, max_batch=B))
    eng.load_dynamics(1).set_cost("cartpole_est")
    pre = R.Preset("t", K=K, H=H, lam=0.5, sigma=0.8, U_clamp=0.6, update="replace")
    rs = np.random.RandomState(11)
    x0 = np.stack([[0.1 * b, 0.5 * b, 0.0, 0.2] for b in range(B)])
    U0 = (0.3 * rs.randn(B, 1, H)).astype(np.float32)
    noise = 0.8 * rs.randn(B, 1, H, K)
    res = eng.solve(x0, U0, noise=noise, shift=True, u0_before=True, want_weights=True)
    for b in range(B):
        ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_est_running_cost, x0[b], U0[b], noise[b])
        # 50 |cos(theta) - 1| has no relative precision near theta = 0 in fp32 (one ulp of cos is 6e-8, x50 per
        # step over H + 10 terminal weights): atol 1e-4 beside rtol 1e-5
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=1e-5, atol=1e-4)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        _, Us = R.shift_U(pre, R.update_U(pre, U0[b], noise[b], res.weights[b].astype(np.float64)))
        np.testing.assert_allclose(res.U[b], Us, atol=1e-5)
        np.testing.assert_array_equal(res.u0[b], U0[b][:, 0])  # MPPI_FLAG_U0_BEFORE: the pre-update U[:, 0]
    assert np.abs(res.U).max() <= 0.6 + 1e-7


def test_nonfinite_costs_flagged(M):
    from mppi_hip import MPPIError
    K, H = 64, 5
    eng = _engine(M, "cartpole_py", K=K, H=H)
    eng.load_dynamics(1).set_cost("cartpole")
    x0 = np.array([np.nan, 0.0, 0.0, 0.0])
    with pytest.raises(MPPIError) as e:
        eng.solve(x0, np.zeros((1, H)), noise=np.zeros((1, H, K)), raise_nonfinite=True)
    assert e.value.code == -4


# ------------------------------------------------------------------------------------------ learned

def _ca_setup(M, K, H, precision, B=1):
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    eng = _engine(M, "humanoid_v3", K=K, H=H, precision=precision, max_batch=B)
    eng.load_dynamics(*cross_attention_blob(sd))
    return eng, sd


@pytest.mark.parametrize("precision", [0, 1])
def test_ca_humanoid_g7_fixture(M, precision):
    """G7 fixture: estimator-style CA humanoid solve restated around the imported reference module."""
    g = golden("g7_ca_humanoid_solve.npz")
    K, H = int(g["K"]), int(g["H"])
    eng, sd = _ca_setup(M, K, H, precision)
    eng.set_cost("humanoid_v3", g["ctx"])
    res = eng.solve(g["x0"], g["U0"], noise=g["noise"], want_weights=True)
    pre = R.Preset("g7", K=K, H=H, lam=1.0, sigma=0.75)
    if precision == 0:
        np.testing.assert_allclose(res.costs, g["costs"], rtol=1e-4)
        np.testing.assert_allclose(res.U, g["U_new"], atol=1e-4)
    else:
        # bf16 engine rounding of the engine's net: the LayerNorm-folded CA stack (oracle/nets_ref.py::ln_fold)
        dyn = N.learned_dynamics(N.ln_fold(N.ca_fold(sd, 28, 27, 21)), 55, precision="bf16")
        ref = R.mppi_solve(pre, dyn, R.humanoid_v3_cost, g["x0"].astype(np.float32), g["U0"], g["noise"],
                           ctx=g["ctx"], dtype=np.float32)
        np.testing.assert_allclose(res.costs, ref["costs"], rtol=5e-3)
        np.testing.assert_allclose(res.U, g["U_new"], atol=2e-2)


@pytest.mark.parametrize("precision", [0, 1])
def test_ca_humanoid_batched_rows(M, precision):
    """B=4 solves from logged humanoid states (data/2025-04-09_145305, stride 20), K=256, H=12."""
    K, H, B = 256, 12, 4
    eng, sd = _ca_setup(M, K, H, precision, B=B)
    ctx = R.humanoid_context(swing_foot_x=0.2, swing_knee_x=0.1, swing_vx=0.3, foot_clearance=0.01)
    eng.set_cost("humanoid_v3", ctx)
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B]
    rs = np.random.RandomState(11)
    U0 = 0.1 * rs.randn(B, 21, H)
    noise = 0.75 * rs.randn(B, 21, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    stack = N.ca_fold(sd, 28, 27, 21)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.75)
    for b in range(B):
        if precision == 0:
            dyn = N.learned_dynamics(stack, 55, precision="fp32")
            ref = R.mppi_solve(pre, dyn, R.humanoid_v3_cost, x0[b].astype(np.float32), U0[b], noise[b], ctx=ctx,
                               dtype=np.float32)
            _check_solve(_row(res, b), ref, pre, U0[b], noise[b], cost_rtol=1e-4, u_atol=1e-4)
        else:
            dyn = N.learned_dynamics(N.ln_fold(stack), 55, precision="bf16")
            ref = R.mppi_solve(pre, dyn, R.humanoid_v3_cost, x0[b].astype(np.float32), U0[b], noise[b], ctx=ctx,
                               dtype=np.float32)
            np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=5e-3)


@pytest.mark.parametrize("H", [1, 3, 5, 400])
@pytest.mark.parametrize("precision", [0, 1, 2])
def test_ca_horizon_tails_and_long_U(M, H, precision):
    """The fc body's control loads (fc_rollout.h): U and eps prefetched kCtrlPrefetch steps ahead over a step loop
    unrolled by that distance, with a shorter tail (H = 1, 3, 5) and a long horizon (H = 400).  Every precision's
    kernel (M-split bf16, fp32, split-bf16 two-tile at prefetch 1) against the oracle, K = 64."""
    K = 64
    eng, sd = _ca_setup(M, K, H, precision)
    ctx = R.humanoid_context(swing_foot_x=0.2, swing_knee_x=0.1, swing_vx=0.3, foot_clearance=0.01)
    eng.set_cost("humanoid_v3", ctx)
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][3]
    rs = np.random.RandomState(12)
    U0 = 0.1 * rs.randn(21, H)
    noise = 0.75 * rs.randn(21, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    stack = N.ca_fold(sd, 28, 27, 21)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.75)
    dyn = (N.learned_dynamics(N.ln_fold(stack), 55, precision="bf16") if precision == 1 else
           N.learned_dynamics(stack, 55, precision="fp32"))
    ref = R.rollout(pre, dyn, R.humanoid_v3_cost, x0.astype(np.float32), U0, noise, ctx=ctx, dtype=np.float32)
    np.testing.assert_allclose(res.costs, ref, rtol=5e-3 if precision == 1 else 1e-4)


def _row(res, b):
    from mppi_hip.engine import SolveResult
    return SolveResult(U=res.U[b], costs=res.costs[b], weights=res.weights[b], u0=res.u0[b])


@pytest.mark.parametrize("name,nx,nu,cost", [("humanoid", 55, 21, "humanoid_v3"), ("quad", 37, 12, "quad_est"),
                                             ("quad", 37, 12, "quad_jl")])
@pytest.mark.parametrize("precision", [0, 1])
def test_mlp_dynamics(M, name, nx, nu, cost, precision):
    from mppi_hip.nets import mlp_blob
    g = golden(f"g8_mlp_{name}_fwd.npz")
    sd = {k[2:]: v for k, v in g.items() if k.startswith("w.")}
    K, H = 192, 10
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=1.0, sigma=0.5, precision=precision))
    eng.load_dynamics(*mlp_blob(sd, nx, nu))
    eng.set_cost(cost)
    rs = np.random.RandomState(2)
    x0 = 0.3 * rs.randn(nx)
    U0 = 0.1 * rs.randn(nu, H)
    noise = 0.5 * rs.randn(nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.5)
    cfun = R.COSTS[cost]
    ctx = np.array([2.0, 0.0, 1.28, 0, 0, 0, 0, 0]) if cost == "humanoid_v3" else (
        np.array([2.0, 0.0, 0.35]) if cost == "quad_est" else None)
    prec = "fp32" if precision == 0 else "bf16"
    dyn = N.learned_dynamics(N.mlp_stack(sd), nx, precision=prec)
    ref = R.mppi_solve(pre, dyn, cfun, x0.astype(np.float32), U0, noise, ctx=ctx, dtype=np.float32)
    if precision == 0:
        _check_solve(res, ref, pre, U0, noise, cost_rtol=1e-4, u_atol=1e-4)
    else:
        np.testing.assert_allclose(res.costs, ref["costs"], rtol=5e-3)


@pytest.mark.parametrize("precision", [0, 1])
def test_trained_quad_mlp_from_logs(M, precision):
    """train the MLP surrogate on the reference's quadruped logs on the GPU (mppi_hip.training,
    a few epochs), load it through the weight blob and solve from a logged state (quad_est preset, replace update);
    costs vs the oracle with the same trained weights: fp32 rtol 1e-4, bf16 rtol 5e-3 (bf16-rounding oracle)."""
    from mppi_hip import training as T
    g = golden("quad_logs.npz")
    X, Y = T.log_pairs(g["states1"], g["actions1"])
    model, hist = T.train_mlp(X, Y, 37, 12, epochs=4, lr=1e-3, device="cuda", log=None)
    assert hist[-1][0] < hist[0][0]
    sd = T.state_dict_numpy(model)
    K, H = 256, 12
    eng = M.Engine(M.Config.preset("quad_est", K=K, H=H, precision=precision))
    eng.load_dynamics(*T.export_mlp_blob(sd, 37, 12)).set_cost("quad_est")
    rs = np.random.RandomState(4)
    x0 = g["states1"][100].astype(np.float64)
    U0 = 0.1 * rs.randn(12, H)
    noise = 0.4 * rs.randn(12, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    dyn = N.learned_dynamics(N.mlp_stack(sd), 37, precision="fp32" if precision == 0 else "bf16")
    ref = R.mppi_solve(pre, dyn, R.quad_est_running_cost, x0.astype(np.float32), U0, noise,
                       ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-4 if precision == 0 else 5e-3)


def test_trained_quad_fa_from_logs(M):
    """The FeatureAttention surrogate (hidden 64) trained on the GPU on the reference's quadruped logs
    (mppi_hip.training.train_fa, 2 epochs) and solved through the engine in exact-fp32 mode: costs vs the oracle's
    FA forward with the same trained weights, rtol 1e-4."""
    from mppi_hip import training as T
    g = golden("quad_logs.npz")
    X, Y = T.log_pairs(g["states2"], g["actions2"])
    model, hist = T.train_fa(X[:2048], Y[:2048], 37, 12, hidden_dim=64, epochs=2, lr=1e-3, device="cuda", log=None)
    sd = T.state_dict_numpy(model)
    K, H = 96, 4
    eng = M.Engine(M.Config.preset("quad_est", K=K, H=H, precision=0))
    eng.load_dynamics(*T.export_fa_blob(sd, 37, 12, 64)).set_cost("quad_est")
    rs = np.random.RandomState(6)
    x0 = g["states2"][200].astype(np.float64)
    U0 = 0.1 * rs.randn(12, H)
    noise = 0.4 * rs.randn(12, H, K)
    res = eng.solve(x0, U0, noise=noise)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    ref = R.mppi_solve(pre, N.fa_dynamics(sd, 37, precision="fp32"), R.quad_est_running_cost, x0.astype(np.float32),
                       U0, noise, ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-4)


# ------------------------------------------------------------------------------------------ reference API mirror

def test_controller_api_matches_reference_loop(M):
    """mppi_controller over 6 control steps (src/cartpole_mppi.py:101-117 loop, env stepped by the analytic
    plant), with the reference's own numpy noise stream (np.random.seed)."""
    from mppi_hip import MPPIModel, SimData, mppi_controller
    K, T = 256, 40
    model = MPPIModel("cartpole_py", noise="numpy", K=K, H=T, precision=0)
    data = SimData(qpos=np.array([0.0, np.pi - 0.3]), qvel=np.zeros(2), ctrl=np.zeros(1))
    pre = R.Preset("t", K=K, H=T, lam=1.0, sigma=1.0)
    U_ref = np.zeros((1, T))
    x_ref = np.concatenate([data.qpos, data.qvel])
    np.random.seed(0)
    for step in range(6):
        state_before = np.random.get_state()
        mppi_controller(model, data)
        np.random.set_state(state_before)
        noise = np.random.randn(1, T, K) * 1.0  # the draw the controller just made
        costs = R.rollout(pre, R.cartpole_step, R.cartpole_running_cost, x_ref, U_ref, noise)
        np.testing.assert_allclose(model.last.costs, costs, rtol=1e-5)
        w = model.last.weights.astype(np.float64)
        U_ref = R.update_U(pre, U_ref, noise, w)
        u0, U_ref = R.shift_U(pre, U_ref)
        np.testing.assert_allclose(data.ctrl, u0, atol=1e-5)
        np.testing.assert_allclose(model.U_global, U_ref, atol=1e-5)
        U_ref = model.U_global.copy()  # keep the two loops on the same fp32-rounded U
        x_ref = R.cartpole_step(x_ref[None], data.ctrl[None])[0]
        data.qpos[:], data.qvel[:] = x_ref[:2], x_ref[2:]


def test_device_pointer_solve_with_torch(M):
    """MPPI_FLAG_DEVICE path used by bench.py: inputs resident in HBM, stream shared with torch."""
    import torch
    K, H, B = 512, 16, 3
    eng = _engine(M, "cartpole_py", K=K, H=H, max_batch=B)
    eng.load_dynamics(1).set_cost("cartpole")
    rs = np.random.RandomState(3)
    x0 = np.stack([[0.0, 0.5 * b, 0.0, 0.0] for b in range(B)]).astype(np.float32)
    U0 = (0.1 * rs.randn(B, 1, H)).astype(np.float32)
    noise = rs.randn(B, 1, H, K).astype(np.float32)
    host = eng.solve(x0, U0, noise=noise, shift=True)
    dev = torch.device("cuda")
    tx, tU, tn = (torch.from_numpy(a).to(dev) for a in (x0, U0, noise))
    tc = torch.empty(B, K, device=dev)
    tu0 = torch.empty(B, 1, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), costs_ptr=tc.data_ptr(), u0_ptr=tu0.data_ptr(),
                     shift=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tU.cpu().numpy(), host.U)
    np.testing.assert_array_equal(tc.cpu().numpy(), host.costs)
    np.testing.assert_array_equal(tu0.cpu().numpy(), host.u0)


@pytest.mark.parametrize("K,H,B", [(1024, 64, 8), (8192, 128, 2)])
def test_ca_full_size_softmin_and_update_properties(M, K, H, B):
    """BASELINE configs #4 (K=1024, H=64, 8 solves) and #5 (K=8192, H=128) at full size, bf16, through the
    device-pointer path: size-independent properties against torch float64 on the engine's own outputs --
    weights = softmin(costs) (src/Humanoid_mppi_v3.jl:160-163) summing to 1, and U_new - U_old = sum_k w_k eps_k
    (:164-170, additive, no clamp) for injected noise."""
    import torch
    eng, _ = _ca_setup(M, K, H, 1, B=B)
    eng.set_cost("humanoid_v3")
    g = golden("g5_ca_humanoid_fwd.npz")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(11)
    tx = torch.from_numpy(np.ascontiguousarray(g["x0_stride20"][:B], dtype=np.float32)).to(dev)
    tU = 0.05 * torch.randn(B, 21, H, device=dev, generator=gen)
    tn = 0.75 * torch.randn(B, 21, H, K, device=dev, generator=gen)
    U_old = tU.double().clone()
    tc = torch.empty(B, K, device=dev)
    tw = torch.empty(B, K, device=dev)
    tu0 = torch.empty(B, 21, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), costs_ptr=tc.data_ptr(), u0_ptr=tu0.data_ptr(),
                     weights_ptr=tw.data_ptr(), shift=False)
    torch.cuda.synchronize()
    c, w = tc.double(), tw.double()
    assert torch.isfinite(c).all()
    w_ref = torch.softmax(-(c - c.min(dim=1, keepdim=True).values) / 1.0, dim=1)  # lambda = 1 (humanoid_v3)
    torch.testing.assert_close(w, w_ref, rtol=1e-4, atol=1e-7)
    torch.testing.assert_close(w.sum(dim=1), torch.ones(B, dtype=torch.float64, device=dev), rtol=0, atol=1e-5)
    dU = torch.einsum("bk,buhk->buh", w, tn.double())
    torch.testing.assert_close(tU.double() - U_old, dU, rtol=0, atol=2e-6)
    torch.testing.assert_close(tu0.double(), tU.double()[:, :, 0], rtol=0, atol=0)


@pytest.mark.parametrize("u0_before", [False, True])
def test_ca_full_size_clamp_shift_u0(M, u0_before):
    """Config #4 size (K=1024, H=64, 8 solves, bf16) with U clamp, receding-horizon shift (fill 0.1) and both u0
    conventions (src/Humanoid_mppi_v3.jl:173-179; src/quadruped_datacollection.py:170 takes u0 before the
    update): the reduce's block-local update (B * nu = 168 >= 128: one u-row per block) against torch float64 on
    the engine's own weights."""
    import torch
    from mppi_hip.nets import cross_attention_blob
    K, H, B, nu = 1024, 64, 8, 21
    eng = _engine(M, "humanoid_v3", K=K, H=H, precision=1, max_batch=B, U_clamp=0.3)
    eng.load_dynamics(*cross_attention_blob(golden_sd("ca_humanoid_weights.npz"))).set_cost("humanoid_v3")
    g = golden("g5_ca_humanoid_fwd.npz")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(12)
    tx = torch.from_numpy(np.ascontiguousarray(g["x0_stride20"][:B], dtype=np.float32)).to(dev)
    tU = 0.25 * torch.randn(B, nu, H, device=dev, generator=gen)
    tn = 0.75 * torch.randn(B, nu, H, K, device=dev, generator=gen)
    U_old = tU.double().clone()
    tw = torch.empty(B, K, device=dev)
    tu0 = torch.empty(B, nu, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    io = M._lib.mppi_io(tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), None, tw.data_ptr(), tu0.data_ptr(), None)
    flags = (M._lib.FLAG_DEVICE | M._lib.FLAG_SHIFT | (M._lib.FLAG_U0_BEFORE if u0_before else 0))
    M._lib.check(eng.lib.mppi_solve_ex(eng._h, B, ctypes.byref(io), ctypes.c_uint64(0), flags))
    torch.cuda.synchronize()
    Un = (U_old + torch.einsum("bk,buhk->buh", tw.double(), tn.double())).clamp(-0.3, 0.3)
    Us = torch.cat([Un[:, :, 1:], 0.1 * Un[:, :, -1:]], dim=2)
    torch.testing.assert_close(tU.double(), Us, rtol=0, atol=2e-6)
    torch.testing.assert_close(tu0.double(), (U_old if u0_before else Un)[:, :, 0], rtol=0, atol=2e-6)


# ------------------------------------------------------------------------------------------ feature attention

def test_fa_quad_full_size_replace_update_properties(M):
    """BASELINE config #3 at full size (quadruped FA D=512, K=2048, H=40, bf16, synthetic weights), replace-mode
    update of src/quadruped_mppi_estimator.py:93-95: U_new = sum_k w_k eps_k with w = softmin(costs / lambda=10),
    checked in torch float64 on the engine's own costs / weights for injected noise."""
    import torch
    from mppi_hip.nets import synthetic_feature_attention
    K, H, nx, nu = 2048, 40, 37, 12
    sd = synthetic_feature_attention(nx, nu, 512, seed=0)
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, lam=10.0, sigma=0.4, cost="quad_est")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(5)
    tx = 0.1 * torch.randn(1, nx, device=dev, generator=gen)
    tU = 0.05 * torch.randn(1, nu, H, device=dev, generator=gen)
    tn = 0.4 * torch.randn(1, nu, H, K, device=dev, generator=gen)
    tc = torch.empty(1, K, device=dev)
    tw = torch.empty(1, K, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(1, tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), costs_ptr=tc.data_ptr(),
                     weights_ptr=tw.data_ptr(), shift=False)
    torch.cuda.synchronize()
    c, w = tc.double(), tw.double()
    assert torch.isfinite(c).all() and c.std() > 0
    w_ref = torch.softmax(-(c - c.min()) / 10.0, dim=1)
    torch.testing.assert_close(w, w_ref, rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(tU.double(), torch.einsum("bk,buhk->buh", w, tn.double()), rtol=0, atol=2e-6)


def _fa_engine(M, sd, nx, nu, K, H, precision, lam=10.0, sigma=0.5, B=1, cost="cartpole_est", update_mode=1, nh=4):
    from mppi_hip.nets import feature_attention_blob
    D = sd["feature_encoding.0.weight"].shape[0]
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=lam, sigma=sigma, precision=precision, max_batch=B,
                            update_mode=update_mode, shift_fill=0.1, terminal_weight=10.0))
    eng.load_dynamics(*feature_attention_blob(sd, nx, nu, D, num_heads=nh))
    eng.set_cost(cost)
    return eng


@pytest.mark.parametrize("precision", [0, 1])
def test_fa_cartpole_g4_fixture(M, precision):
    """G4: src/cartpole_mppi_estimator.py:61-143 run with the reference FA module and checkpoints_cartpole
    (replace-mode update, lambda 10).  fp32: costs rtol 1e-4, U atol 1e-4.  bf16: costs rtol 1e-2 vs the
    bf16-rounding oracle, U atol 2e-2 vs the fixture."""
    g = golden("g4_fa_cartpole_solve.npz")
    sd = golden_sd("fa_cartpole_weights.npz")
    K, H = int(g["K"]), int(g["T"])
    eng = _fa_engine(M, sd, 4, 1, K, H, precision)
    res = eng.solve(g["x0"], g["U0"], noise=g["noise"], want_weights=True)
    if precision == 0:
        np.testing.assert_allclose(res.costs, g["costs"], rtol=1e-4)
        np.testing.assert_allclose(res.weights, g["weights"], atol=1e-4)
        np.testing.assert_allclose(res.U, g["U_new"], atol=1e-4)
    else:
        pre = R.Preset("g4", K=K, H=H, lam=10.0, sigma=0.5, update="replace")
        dyn = N.fa_dynamics(sd, 4, precision="bf16")
        ref = R.mppi_solve(pre, dyn, R.cartpole_est_running_cost, g["x0"], g["U0"], g["noise"], dtype=np.float32)
        np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-2)
        np.testing.assert_allclose(res.U, g["U_new"], atol=2e-2)


@pytest.mark.parametrize("precision", [0, 1])
def test_fa_quad64_ragged_batched(M, precision):
    """FA with 49 tokens (quadruped nx=37, nu=12) at hidden 64, seeded weights of G8 (one sample per
    workgroup), B=2 solves, K=70 (ragged vs the 64-sample pitch), quad_est cost, H=5."""
    g = golden("g8_fa_quad64_fwd.npz")
    sd = {k[2:]: v for k, v in g.items() if k.startswith("w.")}
    K, H, B, nx, nu = 70, 5, 2, 37, 12
    eng = _fa_engine(M, sd, nx, nu, K, H, precision, lam=10.0, sigma=0.4, B=B, cost="quad_est")
    rs = np.random.RandomState(5)
    x0 = 0.2 * rs.randn(B, nx)
    U0 = 0.1 * rs.randn(B, nu, H)
    noise = 0.4 * rs.randn(B, nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    dyn = N.fa_dynamics(sd, nx, precision="fp32" if precision == 0 else "bf16")
    for b in range(B):
        ref = R.mppi_solve(pre, dyn, R.quad_est_running_cost, x0[b].astype(np.float32), U0[b], noise[b],
                           ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
        if precision == 0:
            _check_solve(_row(res, b), ref, pre, U0[b], noise[b], cost_rtol=1e-4, u_atol=1e-4)
        else:
            np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=1e-2)


@pytest.mark.parametrize("D", [128, 512])
def test_fa_wide_bf16(M, D):
    """FA hidden 128 and 512 (the quadruped estimator's width, src/quadruped_mppi_estimator.py:24-35; its
    checkpoint is missing, so seeded weights), bf16, vs the bf16-rounding oracle."""
    from mppi_hip.nets import synthetic_feature_attention
    nx, nu, K, H = 37, 12, 24, 3
    sd = synthetic_feature_attention(nx, nu, D, seed=D)
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, lam=10.0, sigma=0.4, cost="quad_est")
    rs = np.random.RandomState(D)
    x0 = 0.2 * rs.randn(nx)
    U0 = 0.1 * rs.randn(nu, H)
    noise = 0.4 * rs.randn(nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    ref = R.mppi_solve(pre, N.fa_dynamics(sd, nx, precision="bf16"), R.quad_est_running_cost,
                       x0.astype(np.float32), U0, noise, ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-2)
    w_own = R.softmin_weights(res.costs.astype(np.float64), pre.lam)
    np.testing.assert_allclose(res.weights, w_own, atol=1e-5)
    if D == 512:  # the layer-by-layer path on the same solve: oracle parity, and it is a different kernel chain
        os.environ["MPPI_FA_LAYERED"] = "1"
        try:
            eng2 = _fa_engine(M, sd, nx, nu, K, H, 1, lam=10.0, sigma=0.4, cost="quad_est")
            res2 = eng2.solve(x0, U0, noise=noise, want_weights=True)
        finally:
            del os.environ["MPPI_FA_LAYERED"]
        np.testing.assert_allclose(res2.costs, ref["costs"], rtol=1e-2)
        assert not np.array_equal(res2.costs, res.costs)


@pytest.fixture
def fa_layered(monkeypatch):
    """Route hidden-512 FA solves through the layer-by-layer path (kernels_fa_layered.hip; read per launch)."""
    monkeypatch.setenv("MPPI_FA_LAYERED", "1")


@pytest.mark.parametrize("nh", [4, 8])
def test_fa_d512_layered_batch(M, nh, fa_layered):
    """The layer-by-layer hidden-512 path (kernels_fa_layered.hip) over a batch: B = 2 solves x K = 70 samples x 49
    tokens = 6,860 token rows (the last 128-row GEMM tile part padding, the last sample's 64-token attention window
    past the real rows), 4 heads (head dim 128) and 8 heads (64), LayerNorm affines and biases perturbed off their
    init values, additive update.  Costs rtol 1e-2 vs the
    bf16-rounding oracle (oracle/nets_ref.py::fa_forward_engine, the same rounding points); weights = softmin of
    the engine's own costs and U / u0 the update they give, exactly as the other solves."""
    nx, nu, K, H, B = 37, 12, 70, 4, 2
    sd = _perturbed_fa(nx, nu, 512, 2, seed=5 + nh, num_heads=nh)  # non-trivial LayerNorm affines and biases
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, lam=10.0, sigma=0.4, B=B, cost="quad_est", update_mode=0, nh=nh)
    rs = np.random.RandomState(nh)
    x0 = 0.2 * rs.randn(B, nx)
    U0 = 0.1 * rs.randn(B, nu, H)
    noise = 0.4 * rs.randn(B, nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4)
    dyn = N.fa_dynamics(sd, nx, nheads=nh, precision="bf16")
    for b in range(B):
        ref = R.mppi_solve(pre, dyn, R.quad_est_running_cost, x0[b].astype(np.float32), U0[b], noise[b],
                           ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
        _check_solve(_row(res, b), ref, pre, U0[b], noise[b], cost_rtol=1e-2, u_atol=2e-2)


def test_fa_d512_layered_env_step(M, fa_layered):
    """MPPI_FLAG_ENV_STEP through the layer-by-layer hidden-512 path: x0 <- f(x0, u0) for each of B = 3 solves
    (one sample per solve: a 147-row batch) vs the bf16-rounding oracle step, atol 2e-3: the state delta comes out
    of two 512-wide layers whose activations are rounded to bf16 (2^-8 relative) in both, where a different fp32
    summation order flips single roundings."""
    import torch
    from mppi_hip.nets import synthetic_feature_attention
    nx, nu, K, H, B = 37, 12, 40, 3, 3
    sd = synthetic_feature_attention(nx, nu, 512, seed=9)
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, B=B, cost="quad_est")
    dyn = N.fa_dynamics(sd, nx, precision="bf16")
    rs = np.random.RandomState(11)
    x0 = (0.2 * rs.randn(B, nx)).astype(np.float32)
    U0 = (0.1 * rs.randn(B, nu, H)).astype(np.float32)
    dev = torch.device("cuda")
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    tu0 = torch.empty(B, nu, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=4, u0_ptr=tu0.data_ptr(), shift=True, env_step=True)
    torch.cuda.synchronize()
    u0, xn = tu0.cpu().numpy(), tx.cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(xn[b], dyn(x0[b][None], u0[b][None])[0], rtol=0, atol=2e-3)
    assert not np.allclose(xn, x0)


@pytest.mark.parametrize("nx,nu,cost", [(4, 1, "cartpole"), (4, 2, "cartpole"), (10, 6, "quad_est")])
def test_fa_small_net_bf16(M, nx, nu, cost):
    """The small-net FA kernel (hidden 64, L = nx + nu <= 16 tokens, bf16: kernels_fa.hip::fa_small_kernel) with
    16 // L = 3, 2, 1 samples per 16-row tile, B = 2 solves, K = 70 (the last workgroup partly empty), costs with a
    control term and the additive update.  Costs rtol 1e-2 vs the bf16-rounding oracle (LayerNorm affine folded as
    the kernel's); weights = softmin of the engine's own costs and U = the update they give, exactly as the other
    solves."""
    from mppi_hip.nets import synthetic_feature_attention
    K, H, B = 70, 6, 2
    sd = synthetic_feature_attention(nx, nu, 64, seed=nx + 10 * nu)
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, lam=1.0, sigma=0.4, B=B, cost=cost, update_mode=0)
    rs = np.random.RandomState(nx * nu)
    x0 = 0.2 * rs.randn(B, nx)
    U0 = 0.1 * rs.randn(B, nu, H)
    noise = 0.4 * rs.randn(B, nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.4)
    dyn = N.fa_dynamics(sd, nx, precision="bf16")
    ctx = np.array(R.QUAD_GOAL) if cost == "quad_est" else None
    for b in range(B):
        ref = R.mppi_solve(pre, dyn, R.COSTS[cost], x0[b].astype(np.float32), U0[b], noise[b], ctx=ctx,
                           dtype=np.float32)
        _check_solve(_row(res, b), ref, pre, U0[b], noise[b], cost_rtol=1e-2, u_atol=2e-2)


def test_fa_small_net_env_step_bf16(M):
    """MPPI_FLAG_ENV_STEP through the small-net FA kernel (bf16): x0 <- f(x0, u0) for every solve of the batch,
    vs the bf16-rounding oracle step (rtol 1e-3: one step of float32 arithmetic in a different order)."""
    import torch
    K, H, B = 96, 5, 3
    sd = golden_sd("fa_cartpole_weights.npz")
    eng = _fa_engine(M, sd, 4, 1, K, H, 1, B=B)
    dyn = N.fa_dynamics(sd, 4, precision="bf16")
    x0 = np.stack([[0.05, 0.1 * b, 0.0, 0.0] for b in range(B)]).astype(np.float32)
    U0 = (0.1 * np.random.RandomState(3).randn(B, 1, H)).astype(np.float32)
    dev = torch.device("cuda")
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    tu0 = torch.empty(B, 1, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=4, u0_ptr=tu0.data_ptr(), shift=True, env_step=True)
    torch.cuda.synchronize()
    u0, xn = tu0.cpu().numpy(), tx.cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(xn[b], dyn(x0[b][None], u0[b][None])[0], rtol=1e-3, atol=1e-5)
    assert not np.allclose(xn, x0)


# ------------------------------------------------------------------------------------------ receding-horizon stream

def _dev_setup(M, kind, K, H, B, precision=0):
    """(engine, x0 [B,nx], U0 [B,nu,H], one-step dynamics (x, u) -> x_next in float64/32 for the oracle)."""
    rs = np.random.RandomState(7)
    if kind == "cartpole":
        eng = _engine(M, "cartpole_py", K=K, H=H, max_batch=B)
        eng.load_dynamics(1).set_cost("cartpole")
        x0 = np.stack([[0.0, 0.3 * b, 0.0, 0.0] for b in range(B)])
        f = lambda x, u: R.cartpole_step(x[None], u[None])[0]  # noqa: E731
        nu = 1
    elif kind == "ca":
        eng, sd = _ca_setup(M, K, H, precision, B=B)
        eng.set_cost("humanoid_v3")
        x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float64)
        dyn = N.learned_dynamics(N.ca_fold(sd, 28, 27, 21), 55, precision="fp32")
        f = lambda x, u: dyn(x[None].astype(np.float32), u[None].astype(np.float32))[0]  # noqa: E731
        nu = 21
    else:  # FA cartpole estimator
        sd = golden_sd("fa_cartpole_weights.npz")
        eng = _fa_engine(M, sd, 4, 1, K, H, precision, B=B)
        x0 = np.stack([[0.05, 0.1 * b, 0.0, 0.0] for b in range(B)])
        dyn = N.fa_dynamics(sd, 4, precision="fp32")
        f = lambda x, u: dyn(x[None].astype(np.float32), u[None].astype(np.float32))[0]  # noqa: E731
        nu = 1
    U0 = 0.1 * rs.randn(B, nu, H)
    return eng, x0.astype(np.float32), U0.astype(np.float32), f


@pytest.mark.parametrize("kind", ["cartpole", "ca", "fa"])
def test_env_step_advances_state(M, kind):
    """MPPI_FLAG_ENV_STEP: x0 <- f(x0, u0) on device with the loaded dynamics (fp32 engine vs oracle step)."""
    import torch
    K, H, B = 128, 8, 2
    eng, x0, U0, f = _dev_setup(M, kind, K, H, B)
    dev = torch.device("cuda")
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    tu0 = torch.empty(B, U0.shape[1], device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=3, u0_ptr=tu0.data_ptr(), shift=True, env_step=True)
    torch.cuda.synchronize()
    u0 = tu0.cpu().numpy()
    xn = tx.cpu().numpy()
    for b in range(B):
        ref = f(x0[b].astype(np.float64), u0[b].astype(np.float64))
        np.testing.assert_allclose(xn[b], ref, rtol=1e-4, atol=1e-5)
    assert not np.allclose(xn, x0)


@pytest.mark.parametrize("net", ["ca", "mlp"])
def test_env_step_with_forced_wave_kernels(M, net):
    """MPPI_FLAG_ENV_STEP while MPPI_FC_WAVE forces the per-wave kernels (2: 16x16, 3: 32x32): the env-step launch
    (one 16-sample group) takes the M-split kernel, so x0 advances exactly as with the per-wave kernels off (CA: the
    state step ignores u0, bitwise; MLP: u0 comes from a different rollout kernel, bf16 tolerance)."""
    import os
    import torch
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    K, H, B = 128, 8, 2
    dev = torch.device("cuda")
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    U0 = (0.1 * np.random.RandomState(3).randn(B, 21, H)).astype(np.float32)
    out = {}
    for wave in ("0", "2", "3"):
        os.environ["MPPI_FC_WAVE"] = wave
        try:
            eng = _engine(M, "humanoid_v3", K=K, H=H, precision=1, max_batch=B)
            if net == "ca":
                eng.load_dynamics(*M.cross_attention_blob(golden_sd("ca_humanoid_weights.npz")))
            else:
                eng.load_dynamics(*mlp_blob(synthetic_mlp(55, 21, seed=0), 55, 21))
            eng.set_cost("humanoid_v3")
            eng.set_stream(torch.cuda.current_stream().cuda_stream)
            tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
            tu0 = torch.empty(B, 21, device=dev)
            eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=5, u0_ptr=tu0.data_ptr(), shift=True,
                             env_step=True)
            torch.cuda.synchronize()
            out[wave] = tx.cpu().numpy()
            eng.close()
        finally:
            os.environ.pop("MPPI_FC_WAVE", None)
        assert np.isfinite(out[wave]).all() and not np.allclose(out[wave], x0), f"MPPI_FC_WAVE={wave}: x0 not advanced"
    for wave in ("2", "3"):
        if net == "ca":
            np.testing.assert_array_equal(out[wave], out["0"])
        else:
            np.testing.assert_allclose(out[wave], out["0"], rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("kind,precision", [("cartpole", 0), ("ca", 1), ("fa", 1)])
def test_graph_stream_replays_the_solve_loop(M, kind, precision):
    """mppi_graph_capture of n chained solves (shift + env step, seed counter) == the same n solves issued one
    by one, bitwise; a second replay continues the stream (fresh noise keys)."""
    import torch
    K, H, B, n = 256, 12, 2, 5
    dev = torch.device("cuda")
    outs = []
    for mode in ("loop", "graph"):
        eng, x0, U0, _ = _dev_setup(M, kind, K, H, B, precision)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
        tu0 = torch.zeros(B, U0.shape[1], device=dev)
        if mode == "loop":
            for _ in range(n):
                eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=9, u0_ptr=tu0.data_ptr(), shift=True,
                                 env_step=True, seed_counter=True)
        else:
            eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=9)
            torch.cuda.synchronize()
            assert np.array_equal(tx.cpu().numpy(), x0)  # capture does not execute
            eng.graph_launch(sync=True)
        torch.cuda.synchronize()
        outs.append((tx.cpu().numpy(), tU.cpu().numpy(), tu0.cpu().numpy()))
        if mode == "graph":
            first = outs[-1]
            eng.graph_launch(sync=True)
            second = tx.cpu().numpy()
            assert not np.array_equal(second, first[0])
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("kind", ["cartpole", "ca"])
def test_stream_trajectory_log(M, kind):
    """mppi_graph_capture_traj: the logged (x_t, u_t) rows are the states the env steps started from and the
    controls they applied; x_{t+1} = f(x_t, u_t) (oracle step); rows equal an explicit solve loop bitwise."""
    import torch
    from mppi_hip.trajectory import run_stream
    K, H, B, n = 128, 10, 2, 6
    eng, x0, U0, f = _dev_setup(M, kind, K, H, B, precision=0)
    states, actions, U_end = run_stream(eng, x0, U0, n, seed=4, launches=2)
    assert states.shape == (2 * n, B, x0.shape[1])
    np.testing.assert_array_equal(states[0], x0)
    for i in range(2 * n - 1):
        for b in range(B):
            ref = f(states[i, b].astype(np.float64), actions[i, b].astype(np.float64))
            np.testing.assert_allclose(states[i + 1, b], ref, rtol=1e-4, atol=1e-5)
    # the same solves issued one by one
    eng2, _, _, _ = _dev_setup(M, kind, K, H, B, precision=0)
    dev = torch.device("cuda")
    eng2.set_stream(torch.cuda.current_stream().cuda_stream)
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    tu0 = torch.zeros(B, U0.shape[1], device=dev)
    for i in range(2 * n):
        np.testing.assert_array_equal(tx.cpu().numpy(), states[i])
        eng2.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=4, u0_ptr=tu0.data_ptr(), shift=True,
                          env_step=True, seed_counter=True)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(tu0.cpu().numpy(), actions[i])
    np.testing.assert_array_equal(tU.cpu().numpy(), U_end)


@pytest.mark.parametrize("kind,precision", [("cartpole", 0), ("ca", 1)])
def test_graph_noise_prefetch_mixed_with_plain_solves(M, kind, precision):
    """Graph streams generate the next solve's noise inside the current solve's reduce (double-buffered, one
    counter value ahead). Interleaving graph launches (odd and even stream lengths, a re-capture) with plain
    counter solves must reproduce the same key sequence as a loop of plain solves, bitwise."""
    import torch
    K, H, B = 128, 8, 2
    dev = torch.device("cuda")
    plan = [("graph", 3), ("plain", 1), ("graph", 2), ("graph", 2), ("plain", 2), ("graph", 3)]
    outs = []
    for mode in ("loop", "mixed"):
        eng, x0, U0, _ = _dev_setup(M, kind, K, H, B, precision)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
        tu0 = torch.zeros(B, U0.shape[1], device=dev)
        captured = None
        for what, n in plan:
            if mode == "loop" or what == "plain":
                for _ in range(n):
                    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=5, u0_ptr=tu0.data_ptr(),
                                     shift=True, env_step=True, seed_counter=True)
            else:
                if captured != n:  # re-capture only when the stream length changes
                    eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=5)
                    captured = n
                eng.graph_launch(sync=False)
        torch.cuda.synchronize()
        outs.append((tx.cpu().numpy(), tU.cpu().numpy(), tu0.cpu().numpy()))
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


def test_k_sharded_solve_with_engines(M):
    """SURVEY 8e second mode with real engines: the K samples of one cartpole solve split in two shards (two
    replace-mode engines standing in for two ranks), combined by the same online-softmin rule; equals one add-mode
    engine solve over all K (atol 1e-5).  The collectives themselves run at world size 1 (gloo); the multi-rank
    combine is covered on CPU (tests/test_distributed.py)."""
    import os
    import socket

    import torch.distributed as dist
    from mppi_hip.distributed import combine_k_shards, solve_k_sharded
    K, H = 512, 20
    noise = R.reference_noise(8, 1, H, K, 1.0)
    x0 = np.array([0.0, 0.5, 0.0, 0.0])
    U0 = 0.2 * np.cos(np.arange(H))[None, :]
    full = _engine(M, "cartpole_py", K=K, H=H, precision=0)
    full.load_dynamics(1).set_cost("cartpole")
    ref = full.solve(x0, U0, noise=noise, shift=True)
    halves = []
    for lo, hi in ((0, K // 2), (K // 2, K)):
        e = M.Engine(M.Config(nx=4, nu=1, H=H, K=hi - lo, lambda_=1.0, sigma=1.0, update_mode=1, shift_fill=0.1,
                              terminal_weight=10.0))
        e.load_dynamics(1).set_cost("cartpole")
        r = e.solve(x0, U0, noise=noise[:, :, lo:hi])
        halves.append((r.costs.astype(np.float64), r.U.astype(np.float64)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        # emulate the two ranks' partials: at world size 1 the collectives are identities, so combine them by hand
        # with the same rule, then check the one-rank path too
        beta = min(c.min() for c, _ in halves)
        parts = [(np.exp(-(c.min() - beta)) * np.exp(-(c - c.min())).sum(), dU) for c, dU in halves]
        dU = sum(f * d for f, d in parts) / sum(f for f, _ in parts)
        Un = U0 + dU
        Us = np.concatenate([Un[:, 1:], 0.1 * Un[:, -1:]], axis=1)
        np.testing.assert_allclose(Us, ref.U, atol=1e-5)
        one = solve_k_sharded(lambda x, U: (ref.costs, np.zeros((1, H))), x0, U0, lam=1.0, shift_fill=0.1)
        assert one[0].shape == (1, H)
        np.testing.assert_allclose(combine_k_shards(*halves[0], lam=1.0), halves[0][1], atol=1e-12)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,precision", [("cartpole", 0), ("ca", 1), ("fa", 1)])
def test_kernel_clock_times_graph_replays(M, kind, precision):
    """mppi_kernel_clock (bench.py's timed-region rollout timing): a graph of n solves captured with the clock on
    stamps exactly n rollout launches per replay; the launch durations agree with HIP events around the same
    rollouts issued as plain solves (within 2x: events also bracket the launch overhead); stamping changes no
    result bit (the graph replay with the clock equals one without)."""
    import torch
    K, H, B, n, reps = 1024, 16, 2, 3, 4
    dev = torch.device("cuda")
    outs = []
    for clock in (False, True):
        eng, x0, U0, _ = _dev_setup(M, kind, K, H, B, precision)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
        tu0 = torch.zeros(B, U0.shape[1], device=dev)
        if clock:
            eng.kernel_clock(True)
        eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=4)
        for _ in range(reps):
            eng.graph_launch(sync=False)
        torch.cuda.synchronize()
        outs.append((tx.cpu().numpy(), tU.cpu().numpy(), tu0.cpu().numpy()))
        if clock:
            launches, total_us, max_us = eng.kernel_clock_read()
            assert launches == n * reps
            avg = total_us / launches
            assert 0.0 < avg <= max_us < 1e5
            eng.profile(True)  # HIP events around plain solves of the same shape (no clock: slot-free)
            eng.kernel_clock(False)
            for _ in range(4):
                eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=5, u0_ptr=tu0.data_ptr(), shift=True,
                                 seed_counter=True)
            torch.cuda.synchronize()
            ne, ms = eng.kernel_time("rollout")
            ev = 1e3 * ms / ne
            assert 0.5 * ev < avg < 2.0 * ev, (avg, ev)
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("shift,u0_before", [(False, False), (True, False), (True, True)])
def test_replace_update_block_local_reduce(M, shift, u0_before):
    """Replace-mode update (src/cartpole_mppi_estimator.py:141-143) through the reduce's block-local update
    (B * nu >= 128: one u-row per block): humanoid MLP (seeded weights), B = 8, K = 1024, H = 64, bf16, U clamp;
    U_new = clamp(sum_k w_k eps_k) [shifted], u0 before / after the update, in torch float64 on the engine's own
    weights."""
    import torch
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    K, H, B, nx, nu = 1024, 64, 8, 55, 21
    cfg = M.Config.preset("humanoid_v3", K=K, H=H, precision=1, max_batch=B, U_clamp=0.2,
                          update_mode=M._lib.UPDATE_REPLACE)
    eng = M.Engine(cfg).load_dynamics(*mlp_blob(synthetic_mlp(nx, nu, seed=3), nx, nu)).set_cost("humanoid_v3")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(13)
    tx = torch.from_numpy(np.ascontiguousarray(golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B],
                                               dtype=np.float32)).to(dev)
    tU = 0.25 * torch.randn(B, nu, H, device=dev, generator=gen)
    tn = 0.75 * torch.randn(B, nu, H, K, device=dev, generator=gen)
    U_old = tU.double().clone()
    tw = torch.empty(B, K, device=dev)
    tu0 = torch.empty(B, nu, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    io = M._lib.mppi_io(tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), None, tw.data_ptr(), tu0.data_ptr(), None)
    flags = (M._lib.FLAG_DEVICE | (M._lib.FLAG_SHIFT if shift else 0) |
             (M._lib.FLAG_U0_BEFORE if u0_before else 0))
    M._lib.check(eng.lib.mppi_solve_ex(eng._h, B, ctypes.byref(io), ctypes.c_uint64(0), flags))
    torch.cuda.synchronize()
    w = tw.double()
    torch.testing.assert_close(w.sum(dim=1), torch.ones(B, dtype=torch.float64, device=dev), rtol=0, atol=1e-5)
    Un = torch.einsum("bk,buhk->buh", w, tn.double()).clamp(-0.2, 0.2)
    Us = torch.cat([Un[:, :, 1:], 0.1 * Un[:, :, -1:]], dim=2) if shift else Un
    torch.testing.assert_close(tU.double(), Us, rtol=0, atol=2e-6)
    torch.testing.assert_close(tu0.double(), (U_old if u0_before else Un)[:, :, 0], rtol=0, atol=2e-6)


# ------------------------------------------------------------------------------------------ maximum sizes

def test_max_K_cartpole_matches_oracle(M):
    """The largest K the engine takes (kMaxK = 32768: the reduce stages K softmin weights in LDS, the fused cartpole
    epilogue combines Kp/256 = 128 block records in its last block) vs the fp64 oracle: costs rtol 1e-5, U atol 1e-4
    (SURVEY 8d), peaked weights at theta0 = pi."""
    K, H = 32768, 8
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=1.0)
    eng = _engine(M, "cartpole_py", K=K, H=H, precision=0)
    eng.load_dynamics(1).set_cost("cartpole")
    noise = R.reference_noise(5, 1, H, K, 1.0)
    x0 = np.array([0.05, np.pi, 0.0, 0.0])
    U0 = 0.2 * np.cos(np.arange(H))[None, :]
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    ref = R.mppi_solve(pre, R.cartpole_step, R.cartpole_running_cost, x0, U0, noise)
    _check_solve(res, ref, pre, U0, noise, cost_rtol=1e-5, u_atol=1e-4)


def test_max_K_ca_softmin_and_update_properties(M):
    """CA humanoid at K = kMaxK = 32768 (2048 sample groups, bf16): weights = softmin(costs) summing to 1 and
    U_new - U_old = sum_k w_k eps_k, in torch float64 on the engine's own outputs (injected noise)."""
    import torch
    K, H = 32768, 4
    eng, _ = _ca_setup(M, K, H, 1, B=1)
    eng.set_cost("humanoid_v3")
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(21)
    tx = torch.from_numpy(np.ascontiguousarray(golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:1],
                                               dtype=np.float32)).to(dev)
    tU = 0.05 * torch.randn(1, 21, H, device=dev, generator=gen)
    tn = 0.75 * torch.randn(1, 21, H, K, device=dev, generator=gen)
    U_old = tU.double().clone()
    tc, tw = torch.empty(1, K, device=dev), torch.empty(1, K, device=dev)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.solve_device(1, tx.data_ptr(), tU.data_ptr(), tn.data_ptr(), costs_ptr=tc.data_ptr(),
                     weights_ptr=tw.data_ptr(), shift=False)
    torch.cuda.synchronize()
    c, w = tc.double(), tw.double()
    assert torch.isfinite(c).all() and c.std() > 0
    torch.testing.assert_close(w, torch.softmax(-(c - c.min()), dim=1), rtol=1e-4, atol=1e-8)
    torch.testing.assert_close(w.sum(), torch.tensor(1.0, dtype=torch.float64, device=dev), rtol=0, atol=1e-5)
    torch.testing.assert_close(tU.double() - U_old, torch.einsum("bk,buhk->buh", w, tn.double()), rtol=0, atol=2e-6)


@pytest.mark.parametrize("precision", [0, 1])
def test_max_dims_mlp_long_horizon(M, precision):
    """The fc-stack maxima at once: nx = 64 state slots, nu = 32 control slots, and nu * H = 16384 (the U row limit,
    H = 512), seeded MLPStatePredictor(64, 32) weights, quad_est cost (replace update), vs the oracle: fp32 costs
    rtol 1e-4 and the full solve checks; bf16 costs rtol 5e-3 vs the bf16-rounding oracle."""
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    nx, nu, K, H = 64, 32, 48, 512
    sd = synthetic_mlp(nx, nu, seed=9)
    # a small output layer keeps the 512-step state bounded (the test checks arithmetic, not a trained model)
    sd["network.6.weight"] = 0.05 * sd["network.6.weight"]
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=10.0, sigma=0.4, precision=precision,
                            update_mode=M._lib.UPDATE_REPLACE))
    eng.load_dynamics(*mlp_blob(sd, nx, nu)).set_cost("quad_est")
    rs = np.random.RandomState(4)
    x0 = 0.1 * rs.randn(nx)
    U0 = 0.1 * rs.randn(nu, H)
    noise = 0.4 * rs.randn(nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    dyn = N.learned_dynamics(N.mlp_stack(sd), nx, precision="fp32" if precision == 0 else "bf16")
    ref = R.mppi_solve(pre, dyn, R.quad_est_running_cost, x0.astype(np.float32), U0, noise,
                       ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    assert np.isfinite(ref["costs"]).all()
    if precision == 0:
        _check_solve(res, ref, pre, U0, noise, cost_rtol=1e-4, u_atol=1e-4)
    else:
        np.testing.assert_allclose(res.costs, ref["costs"], rtol=5e-3)


def test_max_tokens_feature_attention(M):
    """FeatureAttention with the most tokens a workgroup holds (L = nx + nu = 64: one sample per 64-row workgroup),
    hidden 64, fp32 (exact MFMA) vs the oracle's FA forward: costs rtol 1e-4 and the full solve checks."""
    from mppi_hip.nets import synthetic_feature_attention
    nx, nu, K, H = 48, 16, 10, 3
    sd = synthetic_feature_attention(nx, nu, 64, seed=64)
    eng = _fa_engine(M, sd, nx, nu, K, H, 0, lam=10.0, sigma=0.4, cost="quad_est")
    rs = np.random.RandomState(64)
    x0 = 0.2 * rs.randn(nx)
    U0 = 0.1 * rs.randn(nu, H)
    noise = 0.4 * rs.randn(nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=10.0, sigma=0.4, update="replace")
    ref = R.mppi_solve(pre, N.fa_dynamics(sd, nx, precision="fp32"), R.quad_est_running_cost, x0.astype(np.float32),
                       U0, noise, ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    _check_solve(res, ref, pre, U0, noise, cost_rtol=1e-4, u_atol=1e-4)


@pytest.mark.parametrize("overlap", ["1", "0", "toggle"])
@pytest.mark.parametrize("kind,precision", [("cartpole", 0), ("ca", 1), ("fa", 1)])
def test_chained_solves_equal_plain_solves(M, kind, precision, overlap):
    """MPPI_FLAG_CHAIN (the stream-launched form of a graph stream: the next solve's noise prefetched, by default inside
    the reduce, reduce_kernel<GEN>; MPPI_GEN_OVERLAP=1, an A/B arm, on the handle's generator stream concurrently with
    the rollout) interleaved with
    plain counter solves, graph launches and a seed change reproduces a loop of plain solves bitwise (the same Philox
    keys, the same results); "toggle" switches the overlap between consecutive chained segments."""
    import os
    import torch
    K, H, B = 128, 8, 2
    dev = torch.device("cuda")
    plan = [("chain", 3, 5), ("plain", 1, 5), ("graph", 2, 5), ("chain", 2, 5), ("chain", 2, 6), ("graph", 2, 5),
            ("chain", 1, 5), ("chain", 3, 5), ("plain", 2, 5)]
    outs = []
    try:
        for mode in ("loop", "mixed"):
            eng, x0, U0, _ = _dev_setup(M, kind, K, H, B, precision)
            eng.set_stream(torch.cuda.current_stream().cuda_stream)
            tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
            tu0 = torch.zeros(B, U0.shape[1], device=dev)
            for j, (what, n, seed) in enumerate(plan):
                os.environ["MPPI_GEN_OVERLAP"] = str(j % 2) if overlap == "toggle" else overlap
                if what == "graph" and mode == "mixed":
                    eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=seed)
                    eng.graph_launch(sync=False)
                    continue
                for _ in range(n):
                    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=seed, u0_ptr=tu0.data_ptr(),
                                     shift=True, env_step=True, seed_counter=True,
                                     chain=(mode == "mixed" and what == "chain"))
            torch.cuda.synchronize()
            outs.append((tx.cpu().numpy(), tU.cpu().numpy(), tu0.cpu().numpy()))
            eng.close()
    finally:
        os.environ.pop("MPPI_GEN_OVERLAP", None)
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


def test_kernel_clock_error_paths(M):
    """mppi_kernel_clock_read before the clock is enabled is MPPI_E_STATE; past kClockSlots (65536) stamped launches
    since the reset it is MPPI_E_UNSUPPORTED (slots would be reused); solves without the seed counter are not
    stamped (their launch has no slot)."""
    import torch
    from mppi_hip import _lib as L
    K, H, B = 64, 2, 1
    eng, x0, U0, _ = _dev_setup(M, "cartpole", K, H, B)
    dev = torch.device("cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    with pytest.raises(L.MPPIError) as e:
        eng.kernel_clock_read()
    assert e.value.code == L.MPPI_E_STATE
    eng.kernel_clock(True)
    for _ in range(3):  # no seed counter: not stamped
        eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=1)
    assert eng.kernel_clock_read()[0] == 0
    for _ in range(65537):
        eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=1, seed_counter=True)
    torch.cuda.synchronize()
    with pytest.raises(L.MPPIError) as e:
        eng.kernel_clock_read()
    assert e.value.code == L.MPPI_E_UNSUPPORTED
    eng.kernel_clock(True)  # reset
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=1, seed_counter=True)
    n, total, mx = eng.kernel_clock_read()
    assert n == 1 and 0.0 < total == mx


def test_seed_counter_get_set_warm_start(M):
    """mppi_get_seed_counter (checkpoint / resume): every counter solve advances the device noise key by one;
    saving the counter and U after solve i and restoring both into a FRESH engine continues the stream bitwise (solve
    i + 1 draws the noise it would have drawn)."""
    import torch
    K, H, B = 128, 8, 2
    eng, x0, U0, _ = _dev_setup(M, "cartpole", K, H, B)
    dev = torch.device("cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
    eng.set_seed_counter(40)
    assert eng.get_seed_counter() == 40
    for _ in range(3):
        eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=5, seed_counter=True, shift=True)
    assert eng.get_seed_counter() == 43
    saved_U, saved_ctr = tU.clone(), eng.get_seed_counter()
    eng.solve_device(B, tx.data_ptr(), tU.data_ptr(), None, seed=5, seed_counter=True, shift=True)
    torch.cuda.synchronize()
    want = tU.cpu().numpy()
    eng2, *_ = _dev_setup(M, "cartpole", K, H, B)
    eng2.set_stream(torch.cuda.current_stream().cuda_stream)
    eng2.set_seed_counter(saved_ctr)
    tU2 = saved_U.clone()
    eng2.solve_device(B, tx.data_ptr(), tU2.data_ptr(), None, seed=5, seed_counter=True, shift=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tU2.cpu().numpy(), want)
    assert eng2.get_seed_counter() == saved_ctr + 1


@pytest.mark.parametrize("mode", ["chain", "graph"])
def test_seed_counter_resume_chained_and_graph(M, mode):
    """The warm-start save / restore on a receding-horizon stream: after chained solves (MPPI_FLAG_CHAIN)
    or a graph launch the next solve's noise is already prefetched and the device counter one past its key, so
    mppi_get_seed_counter reports the LOGICAL counter (the key the next solve draws).  Saving it with U after a few
    stream solves and restoring both into a FRESH engine continues the stream bitwise: the restored engine's next
    chained solve (or graph launch) produces exactly the U the first engine's did.  Also: get() after get() and a
    plain counter solve interleaved agree with a loop of plain solves (one key per solve)."""
    import torch
    K, H, B, n = 128, 8, 2, 3
    eng, x0, U0, _ = _dev_setup(M, "cartpole", K, H, B)
    dev = torch.device("cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    tx, tU, tu0 = (torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev),
                   torch.zeros(B, 1, device=dev))
    eng.set_seed_counter(10)

    def step(e, U):
        if mode == "chain":
            e.solve_device(B, tx.data_ptr(), U.data_ptr(), None, seed=3, seed_counter=True, shift=True, chain=True)
        else:
            e.graph_launch()

    if mode == "graph":
        eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=3, env_step=False)
    for _ in range(2):
        step(eng, tU)
    per = 1 if mode == "chain" else n
    assert eng.get_seed_counter() == 10 + 2 * per
    assert eng.get_seed_counter() == 10 + 2 * per  # reading it changes nothing
    saved_U, saved_ctr = tU.clone(), eng.get_seed_counter()
    step(eng, tU)
    torch.cuda.synchronize()
    want = tU.cpu().numpy()
    assert eng.get_seed_counter() == saved_ctr + per
    eng2, *_ = _dev_setup(M, "cartpole", K, H, B)
    eng2.set_stream(torch.cuda.current_stream().cuda_stream)
    tU2 = saved_U.clone()
    if mode == "graph":
        eng2.graph_capture(B, n, tx.data_ptr(), tU2.data_ptr(), tu0.data_ptr(), seed=3, env_step=False)
    eng2.set_seed_counter(saved_ctr)
    step(eng2, tU2)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tU2.cpu().numpy(), want)
    assert eng2.get_seed_counter() == saved_ctr + per
    eng.close()
    eng2.close()


# ------------------------------------------------------------------------------------------ bench launch path

@pytest.mark.parametrize("ranks", [2, 3])
def test_bench_two_ranks_complete(M, ranks):
    """bench.py --gpus 2 (ranks under torch.distributed.run, here two gloo ranks sharing device 0; the driver's
    scaling runs use RCCL, one rank per GPU): every rank runs the clock ramp, warmup and timed steps with the
    pipelined control gather, and rank 0 prints one JSON line with n_gpus = 2.  Guards the ramp against collectives:
    each rank times its own ramp, so a gather per ramp step would pair up different step counts and deadlock."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MPPI_DIST_BACKEND="gloo")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", str(ranks), "--steps", "4",
                        "--warmup", "2", "--ramp-ms", "60", "--no-cpu-baseline", "--no-traffic", "--no-kernel-trace"],
                       capture_output=True, text=True, timeout=150, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == ranks and line["steps"] == 4 and line["value"] > 0
    # the default: config #4's 64 states split over the ranks (strong scaling); 3 ranks: uneven shards
    # -- shard_bounds: 22 / 22 / 20 (rank 0 reports its own 22), the gather sized for 22
    assert line["scaling"] == "strong" and line["config"]["solves_per_gpu"] == -(-64 // ranks)
    assert line["config"]["global_solves"] == 64


def _perturbed_fa(nx, nu, D, layers, seed, num_heads=4):
    """Seeded FA weights with non-trivial LayerNorm affines and attention / out-proj biases (the synthetic init has
    gamma = 1 and zero biases there), so the host folds of the small-net kernel are exercised."""
    from mppi_hip.nets import synthetic_feature_attention
    sd = synthetic_feature_attention(nx, nu, D, num_heads=num_heads, attn_layers=layers, seed=seed)
    rs = np.random.RandomState(seed + 1)
    for k in list(sd):
        if k.endswith(("norm1.weight", "norm2.weight")) or k == "feature_encoding.1.weight":
            sd[k] = (1.0 + 0.2 * rs.randn(*sd[k].shape)).astype(np.float32)
        elif k.endswith(("norm1.bias", "norm2.bias", "in_proj_bias", "out_proj.bias")) or k == "feature_encoding.1.bias":
            sd[k] = (0.1 * rs.randn(*sd[k].shape)).astype(np.float32)
    return sd


@pytest.mark.parametrize("layers", [1, 3, 4])
def test_fa_small_net_layers_bf16(M, layers):
    """The small-net FA kernel at 1, 3 and 4 (the maximum) attention layers: its LDS layout (staged out-proj
    fragments per layer, then the FFN2 exchange, O rows, XU) moves with the layer count.  Non-trivial LayerNorm
    affines and biases, B = 2, K = 70 (last workgroup partly empty), H = 2.  These seeded nets are untrained and
    the dynamics amplify single bf16 rounding flips (scripts/fa_layers_probe.py: the median error stays ~1e-6 at
    every depth while up to ~10 % of the samples reach 1e-2, with the same profile for the earlier two-pass
    LayerNorm build), so the costs are checked in distribution: median rel err < 1e-4, 95th percentile < 3e-2,
    max < 5e-2.  A layout error moves every sample: the build before the LDS-aliasing fix returned inf for all
    costs at 3 and 4 layers (its O rows overwrote the last layer's staged out-proj fragments).  Weights and update
    are then exact functions of the engine's own costs, as in the other solves."""
    nx, nu, K, H, B = 4, 1, 70, 2, 2
    sd = _perturbed_fa(nx, nu, 64, layers, seed=40 + layers)
    eng = _fa_engine(M, sd, nx, nu, K, H, 1, lam=1.0, sigma=0.4, B=B, cost="cartpole", update_mode=0)
    rs = np.random.RandomState(layers)
    x0 = 0.2 * rs.randn(B, nx)
    U0 = 0.1 * rs.randn(B, nu, H)
    noise = 0.4 * rs.randn(B, nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.4)
    dyn = N.fa_dynamics(sd, nx, precision="bf16")
    for b in range(B):
        ref = R.mppi_solve(pre, dyn, R.COSTS["cartpole"], x0[b].astype(np.float32), U0[b], noise[b],
                           dtype=np.float32)
        rel = np.abs(res.costs[b] - ref["costs"]) / np.abs(ref["costs"])
        assert np.median(rel) < 1e-4 and np.quantile(rel, 0.95) < 3e-2 and rel.max() < 5e-2, (
            np.median(rel), np.quantile(rel, 0.95), rel.max())
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam, pre.norm_eps)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        U_own = R.update_U(pre, np.asarray(U0[b], np.float64), np.asarray(noise[b], np.float64),
                           res.weights[b].astype(np.float64))
        np.testing.assert_allclose(res.U[b], U_own, atol=1e-5)


@pytest.mark.parametrize("variant", ["fa_small_1layer", "fa_small_4layers", "fa_d128", "fa_d512_layered", "mlp_quad"])
def test_graph_replays_bitwise_reproducible(M, variant, monkeypatch):
    """Two fresh engines replaying the same captured stream of chained solves (device noise, env step) end in
    bit-identical states and controls.  Every kernel reduces in a fixed order, so any difference is a race (the
    small-net FA kernel once had one: scratch regions that aliased, visible only with some wave timings).
    fa_d512_layered: the layer-by-layer hidden-512 chain (11 launches per step) captured into the graph, its
    persistent GEMMs and their LDS stage ring under replay."""
    import torch
    from mppi_hip.nets import mlp_blob
    if variant == "fa_d512_layered":
        monkeypatch.setenv("MPPI_FA_LAYERED", "1")
    B, n, reps = 2, 3, 3
    dev = torch.device("cuda")
    outs = []
    for _ in range(2):
        if variant.startswith("fa_small"):
            layers = 1 if variant.endswith("1layer") else 4
            sd = _perturbed_fa(4, 1, 64, layers, seed=7)
            eng, nx, nu, K, H = _fa_engine(M, sd, 4, 1, 1024, 12, 1, B=B), 4, 1, 1024, 12
        elif variant == "fa_d128":
            sd = _perturbed_fa(10, 6, 128, 2, seed=9)
            eng, nx, nu, K, H = _fa_engine(M, sd, 10, 6, 256, 6, 1, B=B, cost="quad_est"), 10, 6, 256, 6
        elif variant == "fa_d512_layered":
            sd = _perturbed_fa(37, 12, 512, 2, seed=13)
            eng, nx, nu, K, H = _fa_engine(M, sd, 37, 12, 96, 4, 1, B=B, cost="quad_est"), 37, 12, 96, 4
        else:
            g = golden("g8_mlp_quad_fwd.npz")
            msd = {k[2:]: v for k, v in g.items() if k.startswith("w.")}
            eng = _engine(M, "quad_est", K=1024, H=16, precision=1, max_batch=B)
            eng.load_dynamics(*mlp_blob(msd, 37, 12))
            eng.set_cost("quad_est")
            nx, nu, K, H = 37, 12, 1024, 16
        rs = np.random.RandomState(11)
        x0 = (0.1 * rs.randn(B, nx)).astype(np.float32)
        U0 = (0.1 * rs.randn(B, nu, H)).astype(np.float32)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
        tu0 = torch.zeros(B, nu, device=dev)
        eng.graph_capture(B, n, tx.data_ptr(), tU.data_ptr(), tu0.data_ptr(), seed=21)
        for _ in range(reps):
            eng.graph_launch(sync=False)
        torch.cuda.synchronize()
        outs.append((tx.cpu().numpy(), tU.cpu().numpy(), tu0.cpu().numpy()))
        assert np.isfinite(outs[-1][1]).all()
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("layers", [1, 3, 4])
@pytest.mark.parametrize("D,precision", [(64, 0), (128, 1)])
def test_fa_general_layers(M, D, precision, layers):
    """The general FA kernel (fa_rollout_kernel) at 1, 3 and 4 attention layers, non-trivial LayerNorm affines and
    biases: fp32 at hidden 64 (VALU attention, cartpole tokens) against the fp64 oracle, costs rtol 1e-4; bf16 at
    hidden 128 with the quadruped's 49 tokens (MFMA attention, 4 token tiles) against the bf16-rounding oracle,
    costs rtol 1e-2 as test_fa_wide_bf16 (every sample sits ~1e-3 off at 3-4 layers: this kernel's bf16 rounding
    points are modelled less exactly than the small-net kernel's; a layout error gives inf or garbage).
    H = 2, K = 40."""
    nx, nu, cost = (4, 1, "cartpole") if D == 64 else (37, 12, "quad_est")
    K, H = 40, 2
    sd = _perturbed_fa(nx, nu, D, layers, seed=D + layers)
    eng = _fa_engine(M, sd, nx, nu, K, H, precision, lam=1.0, sigma=0.4, cost=cost, update_mode=0)
    rs = np.random.RandomState(layers + D)
    x0 = 0.2 * rs.randn(nx)
    U0 = 0.1 * rs.randn(nu, H)
    noise = 0.4 * rs.randn(nu, H, K)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    pre = R.Preset("t", K=K, H=H, lam=1.0, sigma=0.4)
    ctx = np.array(R.QUAD_GOAL) if cost == "quad_est" else None
    dyn = N.fa_dynamics(sd, nx) if precision == 0 else N.fa_dynamics(sd, nx, precision="bf16")
    ref = R.mppi_solve(pre, dyn, R.COSTS[cost], x0.astype(np.float32), U0, noise, ctx=ctx,
                       dtype=np.float64 if precision == 0 else np.float32)
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=1e-4 if precision == 0 else 1e-2)
    w_own = R.softmin_weights(res.costs.astype(np.float64), pre.lam)
    np.testing.assert_allclose(res.weights, w_own, atol=1e-5)


def test_resident_U_mirror_chain(M):
    """MPPI_FLAG_RESIDENT_U with a device io.U: U stays in the handle and every solve's update kernel also writes the
    new U (and u0) to io.U -- a different buffer each solve here, as bench.py's gather slots -- bitwise equal to the
    same chained solves run on a caller-owned U in place (CA humanoid bf16, B = 2, the ticketed update)."""
    import torch
    K, H, B, n = 256, 8, 2, 4
    dev = torch.device("cuda")
    runs = []
    for resident in (False, True):
        eng, x0, U0, _ = _dev_setup(M, "ca", K, H, B, 1)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        tx, tU = torch.from_numpy(x0).to(dev), torch.from_numpy(U0).to(dev)
        if resident:
            eng.set_U(U0, B)
        outs = []
        for i in range(n):
            dst = torch.full_like(tU, float("nan")) if resident else tU
            du0 = torch.full((B, U0.shape[1]), float("nan"), device=dev)
            eng.solve_device(B, tx.data_ptr(), dst.data_ptr(), None, seed=3, u0_ptr=du0.data_ptr(), shift=True,
                             resident_U=resident, seed_counter=True, chain=True)
            torch.cuda.synchronize()
            outs.append((dst.cpu().numpy().copy(), du0.cpu().numpy()))
        if resident:
            np.testing.assert_array_equal(eng.get_U(B), outs[-1][0])
        runs.append(outs)
    for (Ua, ua), (Ub, ub) in zip(*runs):
        np.testing.assert_array_equal(Ua, Ub)
        np.testing.assert_array_equal(ua, ub)


@pytest.mark.parametrize("extra", [["--workload", "humanoid_ca_stream"], ["--steps", "10"],
                                   ["--weak", "--steps", "10"],
                                   ["--workload", "cartpole", "--steps", "20"]])
def test_bench_line_default_steps(M, extra):
    """bench.py at its default step count (50) for the receding-horizon stream (config #5: 256 solves per step, 12800
    stamped rollout launches, past round 2's 8192 clock slots), config #4's whole 64-state batch on one GPU (the
    default: config #4's 64 states split over the ranks, strong scaling; --weak: 64 per GPU, weak scaling), and the
    analytic cartpole, whose line must report the fp32 it runs."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--warmup", "1", "--ramp-ms", "30",
                        "--no-cpu-baseline", "--no-traffic", "--no-kernel-trace", "--no-plain-pass"] + extra,
                       capture_output=True, text=True, timeout=110, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["value"] > 0 and line["roofline"]["launches"] > 0
    if "cartpole" in extra:
        assert line["dtype"] == "fp32"
    if extra == ["--steps", "10"]:
        assert line["config"]["solves_per_gpu"] == 64 and line["scaling"] == "strong"
        # the fp16 form of the per-wave kernel is named in dtype, with the probes' decisions and errors in config
        assert line["dtype"] == "f16x2w/l1:f16x1" and line["config"]["x3_f16_form"] is True
        assert 0.0 <= line["config"]["x3_f16_probe_rel_err"] <= 7.5e-5
        assert line["config"]["x3_layer1_products"] == 2 and 0.0 <= line["config"]["x3_layer1_probe_rel_err"] <= 7.5e-5
        assert line["config"]["rollout_kernel"] == "fc_wave32_x3p_kernel<f16>"
        # the split mode's second pricing: against peak / (MFMAs per product) of the per-wave kernel 64 solves run
        roof = line["roofline"]
        # fc_wave32_x3p_kernel's fp16 form: statistic 12, layer 0 28, layer 1 64, the last layer 32 per wave-step for 102
        assert roof["split_mfma_per_product"] == round(136 / 102, 4)
        assert 0 < roof["frac"] < roof["frac_of_split_ceiling"] < 1
    if "--weak" in extra:
        assert line["config"]["solves_per_gpu"] == 64 and line["scaling"] == "weak"
