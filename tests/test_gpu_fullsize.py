"""BASELINE config #4 at full size against the oracle, and the humanoid_v1 cost. Needs an MI355X.

Config #4 is benched as 8 solves per GPU, K = 1024, H = 64, the folded CrossAttention surrogate
(checkpoints/model_cross.pth), x0 = logged humanoid states (data/2025-04-09_145305, stride 20), a per-solve
real-env context (src/Humanoid_mppi_v3.jl:53-99), shift on.  The tests run exactly that through the C-ABI
(host pointers, injected seeded noise) and compare two of the 8 solves with the oracle (each ~0.5 s of numpy):

  costs   vs the oracle at the engine's precision: fp32 rtol 1e-4; bf16 rtol 5e-3 against the bf16-emulating oracle
          (every layer input and weight rounded to bf16, fp32 accumulate; the LayerNorm folded as the kernel folds it,
          oracle/nets_ref.py::ln_fold)
  weights = softmin of the engine's own costs, atol 1e-5;  U, u0 = update + shift of those weights, atol 1e-5
  U, u0   end to end vs the fp32 oracle (src/Humanoid_mppi_v3.jl:154-179): atol 1e-4 (fp32) / 2e-2 (bf16) when the
          softmin is well conditioned (oracle weights within 1e-3 of the engine's), else the tie guard of SURVEY 8d
          (the bound sum_k |w_own - w_ref|_k |eps_k| added to the tolerance; SURVEY 8d, tests/test_gpu_parity.py)

The CA surrogate ignores the action, so its samples differ only through the control term and the softmin
is well conditioned in both precisions; the humanoid MLP (seeded MLPStatePredictor(55, 21, 128, 2), action-sensitive)
gives peaked weights whose argmin both precisions must agree on.
"""
import numpy as np
import pytest

from conftest import golden, golden_sd
from oracle import mppi_ref as R
from oracle import nets_ref as N

pytestmark = pytest.mark.gpu

K4, H4, B4, NU, NX = 1024, 64, 8, 21, 55
CHECKED = (0, 5)  # solves compared with the oracle


@pytest.fixture(scope="module")
def M(gpu_available):
    import mppi_hip
    return mppi_hip


def _ctx(b):
    """A different real-env context per solve (swing foot / knee ahead of or behind the root, clearance terms on)."""
    return R.humanoid_context(swing_foot_x=-0.2 + 0.1 * b, swing_knee_x=0.05 * b, swing_vx=0.3 - 0.05 * b,
                              foot_clearance=0.01 * b, leg_clearance=-0.02 if b % 2 else 0.1)


def _net(M, net):
    if net == "ca":
        from mppi_hip.nets import cross_attention_blob
        sd = golden_sd("ca_humanoid_weights.npz")
        return cross_attention_blob(sd), N.ca_fold(sd, 28, 27, 21)
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    sd = synthetic_mlp(NX, NU, seed=0)  # bench.py's humanoid_mlp weights
    return mlp_blob(sd, NX, NU), N.mlp_stack(sd)


def _oracle_dyn(stack, net, precision):
    if precision == "bf16":
        return N.learned_dynamics(N.ln_fold(stack) if net == "ca" else stack, NX, precision="bf16")
    return N.learned_dynamics(stack, NX, precision="fp32")


@pytest.mark.parametrize("net", ["ca", "mlp"])
@pytest.mark.parametrize("precision", [1, 0, 2])
def test_config4_full_size_matches_oracle(M, net, precision):
    """precision 2 = MPPI_PREC_BF16X3 (split bf16, hi + lo pairs, three bf16 MFMAs per product): held to the fp32 bar
    against the fp32 oracle (costs rtol 1e-4, U / u0 atol 1e-4)."""
    blob, stack = _net(M, net)
    eng = M.Engine(M.Config.preset("humanoid_v3", K=K4, H=H4, precision=precision, max_batch=B4))
    eng.load_dynamics(*blob).set_cost("humanoid_v3")
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B4].astype(np.float32)
    rs = np.random.RandomState(44)
    U0 = (0.1 * rs.randn(B4, NU, H4)).astype(np.float32)
    noise = (0.75 * rs.randn(B4, NU, H4, K4)).astype(np.float32)
    ctx = np.stack([_ctx(b) for b in range(B4)])
    res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
    eng.close()
    assert np.isfinite(res.costs).all() and np.isfinite(res.U).all()
    pre = R.Preset("c4", K=K4, H=H4, lam=1.0, sigma=0.75)
    prec = "bf16" if precision == 1 else "fp32"  # BF16X3 against the fp32 oracle
    cost_rtol, u_atol = (5e-3, 2e-2) if precision == 1 else (1e-4, 1e-4)
    well = 0
    for b in CHECKED:
        ref = R.mppi_solve(pre, _oracle_dyn(stack, net, prec), R.humanoid_v3_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                           dtype=np.float32)
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=cost_rtol)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        u0_own, Us_own = R.shift_U(pre, R.update_U(pre, U0[b].astype(np.float64), noise[b].astype(np.float64),
                                                   res.weights[b].astype(np.float64)))
        np.testing.assert_allclose(res.U[b], Us_own, atol=1e-5)
        np.testing.assert_allclose(res.u0[b], u0_own, atol=1e-5)
        # end to end: the chosen control sequence against the fp32 oracle
        ref32 = ref if prec == "fp32" else R.mppi_solve(pre, _oracle_dyn(stack, net, "fp32"), R.humanoid_v3_cost, x0[b],
                                                        U0[b], noise[b], ctx=ctx[b], dtype=np.float32)
        dw = np.abs(w_own - ref32["weights"])
        if dw.max() < 1e-3:
            well += 1
            atol = u_atol
        else:  # tie guard
            atol = u_atol + float(np.max(np.einsum("utk,k->ut", np.abs(noise[b]).astype(np.float64), dw)))
        np.testing.assert_allclose(res.U[b], ref32["U_shifted"], atol=atol)
        np.testing.assert_allclose(res.u0[b], ref32["u0"], atol=atol)
        if net == "mlp":  # peaked weights: both precisions pick the same best sample
            assert int(np.argmin(res.costs[b])) == int(np.argmin(ref32["costs"]))
    assert well == len(CHECKED), "the checked solves were expected to be well conditioned (see the module doc)"


@pytest.mark.parametrize("net", ["ca", "mlp"])
@pytest.mark.parametrize("precision", [0, 1, 2])
def test_humanoid_v1_cost_matches_oracle(M, net, precision):
    """MPPI_COST_HUMANOID_V1 (src/Humanoid_mppi.jl:31-121) through the fc rollout: H = 120 crosses the swing-foot
    phase switches at t = 50 and t = 100 (t % 100 < 50: left foot swings, :76-87) and the terminal term uses t = H.
    Two solves with different foot positions; costs vs the oracle at the engine's precision (fp32 rtol 1e-4, bf16
    5e-3), weights / update / shift from the engine's own costs atol 1e-5."""
    blob, stack = _net(M, net)
    K, H, B = 256, 120, 2
    eng = M.Engine(M.Config.preset("humanoid_v1", K=K, H=H, precision=precision, max_batch=B))
    eng.load_dynamics(*blob).set_cost("humanoid_v1")
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][3:3 + B].astype(np.float32)
    rs = np.random.RandomState(7)
    U0 = (0.05 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.3 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([R.humanoid_v1_context(left_foot=(0.3, 0.1, 0.05 + 0.1 * b), right_foot=(-0.1, -0.12, 0.08))
                    for b in range(B)])
    res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
    eng.close()
    pre = R.Preset("v1", K=K, H=H, lam=1.0, sigma=1.0)
    prec = "bf16" if precision == 1 else "fp32"
    for b in range(B):
        ref = R.mppi_solve(pre, _oracle_dyn(stack, net, prec), R.humanoid_v1_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                           dtype=np.float32)
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=5e-3 if precision else 1e-4)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        u0_own, Us_own = R.shift_U(pre, R.update_U(pre, U0[b].astype(np.float64), noise[b].astype(np.float64),
                                                   res.weights[b].astype(np.float64)))
        np.testing.assert_allclose(res.U[b], Us_own, atol=1e-5)
    # the phase matters: the same solve with the v3 cost differs
    assert not np.allclose(R.rollout(pre, _oracle_dyn(stack, net, "fp32"), R.humanoid_v1_cost, x0[0], U0[0], noise[0],
                                     ctx=ctx[0], dtype=np.float32),
                           R.rollout(pre, _oracle_dyn(stack, net, "fp32"), R.humanoid_v3_cost, x0[0], U0[0], noise[0],
                                     ctx=ctx[0], dtype=np.float32))


def test_controller_builds_context_from_data(M):
    """mppi_controller with a data object carrying xpos / cvel (the real env) solves with the context the reference
    reads from it (src/Humanoid_mppi_v3.jl:53-99): the same solve with the explicit humanoid_context is bitwise
    equal, and a different data context changes the costs."""
    from mppi_hip import MPPIModel, SimData, mppi_controller
    from mppi_hip.controller import HUMANOID_BODY_IDS, humanoid_context
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    sd = synthetic_mlp(NX, NU, seed=0)
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][2]
    rs = np.random.RandomState(2)
    xpos, cvel = rs.randn(18, 3), rs.randn(18, 6)
    outs = []
    for explicit in (False, True, None):
        model = MPPIModel("humanoid_v3", dynamics=("mlp", sd), noise="numpy", K=128, H=10, precision=0)
        data = SimData(qpos=x0[:28].copy(), qvel=x0[28:].copy(), ctrl=np.zeros(NU),
                       xpos=xpos if explicit is not None else 1.5 * xpos, cvel=cvel)
        np.random.seed(3)
        ctx = humanoid_context(data, HUMANOID_BODY_IDS) if explicit else None
        mppi_controller(model, data, ctx=ctx)
        outs.append(model.last.costs.copy())
        model.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    assert not np.array_equal(outs[0], outs[2])


# ------------------------------------------------------------------------------------------ any fc-stack shape

def _solve_vs_oracle(M, blob, stack, nx, nu, cost, precision, K=96, H=8, B=2, lam=1.0, sigma=0.4, seed=0, ctx=None,
                     update="add", x0=None):
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=lam, sigma=sigma, precision=precision, max_batch=B,
                            update_mode=1 if update == "replace" else 0))
    eng.load_dynamics(*blob).set_cost(cost)
    rs = np.random.RandomState(seed)
    x0 = (0.2 * rs.randn(B, nx)).astype(np.float32) if x0 is None else x0
    U0 = (0.1 * rs.randn(B, nu, H)).astype(np.float32)
    noise = (sigma * rs.randn(B, nu, H, K)).astype(np.float32)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    eng.close()
    pre = R.Preset("g", K=K, H=H, lam=lam, sigma=sigma, update=update)
    prec = "bf16" if precision == 1 else "fp32"
    out = []
    for b in range(B):
        ref = R.mppi_solve(pre, N.learned_dynamics(stack, nx, precision=prec), R.COSTS[cost], x0[b], U0[b], noise[b],
                           ctx=ctx, dtype=np.float32)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        Un = R.update_U(pre, U0[b].astype(np.float64), noise[b].astype(np.float64), res.weights[b].astype(np.float64))
        np.testing.assert_allclose(res.U[b], Un, atol=1e-5)
        out.append((res.costs[b], ref["costs"]))
    return out


@pytest.mark.parametrize("precision", [0, 1])
def test_generic_mlp_batchnorm_deep_wide(M, precision):
    """MLPStatePredictor(55, 21, hidden 512, BatchNorm, 6 hidden layers) -- learning/train.py:70's net, the oracle
    pinned to the reference module by tests/golden/g9_mlp_bn_fwd.npz -- through the generic fc kernel (the
    register-resident kernel takes hidden 128 x 2 only): costs vs the oracle with the BatchNorm folded, fp32 rtol 1e-4,
    bf16 rtol 1e-2 (eight bf16-rounded layers), humanoid_v3 cost, logged x0."""
    import importlib.util
    import os
    spec_ = importlib.util.spec_from_file_location("gfs", os.path.join(os.path.dirname(__file__), "golden",
                                                                       "gen_fixtures_shapes.py"))
    mod = importlib.util.module_from_spec(spec_)
    spec_.loader.exec_module(mod)
    sd = mod.weights(mod.SHAPES["g9_mlp_bn_fwd"])
    from mppi_hip.nets import mlp_blob
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:2].astype(np.float32)
    for got, ref in _solve_vs_oracle(M, mlp_blob(sd, NX, NU), N.mlp_stack(sd), NX, NU, "humanoid_v3", precision,
                                     ctx=R.humanoid_context(), x0=x0):
        np.testing.assert_allclose(got, ref, rtol=1e-4 if precision == 0 else 1e-2)


@pytest.mark.parametrize("precision", [0, 1])
def test_generic_ca_cartpole_checkpoint(M, precision):
    """checkpoints_cartpole/model_final.pth -- a CrossAttentionStatePredictor(qpos 2, qvel 2, action 1, hidden 144)
    (Visualization/vis.ipynb; the oracle pinned to the reference module by tests/golden/g5_ca_cartpole_fwd.npz) -- as
    the estimator's dynamics (cartpole_est preset: lambda 10, sigma 0.5, replace update), through the generic fc kernel:
    costs vs the oracle's folded net, fp32 rtol 1e-4, bf16 rtol 1e-2 (against the bf16-rounding oracle)."""
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_cartpole_weights.npz")
    stack = N.ca_fold(sd, 2, 2, 1)
    if precision == 1:
        stack = N.ln_fold(stack)
    x0 = np.array([[0.05, 0.3, 0.0, 0.1], [0.0, 3.0, 0.2, 0.0]], np.float32)
    for got, ref in _solve_vs_oracle(M, cross_attention_blob(sd), stack, 4, 1, "cartpole_est", precision, K=256, H=20,
                                     lam=10.0, sigma=0.5, update="replace", x0=x0):
        np.testing.assert_allclose(got, ref, rtol=1e-4 if precision == 0 else 1e-2)


@pytest.mark.parametrize("net", ["ca", "mlp"])
def test_generic_kernel_agrees_with_specialised(M, net):
    """MPPI_FC_GENERIC=1 routes the headline shapes (folded humanoid CA, MLP 128 x 2) through the generic fc kernel:
    exact fp32, costs equal to the register-resident kernel's within 1e-5 (the same arithmetic, another summation
    order)."""
    import os
    blob, _ = _net(M, net)
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:2].astype(np.float32)
    rs = np.random.RandomState(3)
    U0 = (0.1 * rs.randn(2, NU, 12)).astype(np.float32)
    noise = (0.5 * rs.randn(2, NU, 12, 128)).astype(np.float32)
    costs = []
    for generic in (False, True):
        if generic:
            os.environ["MPPI_FC_GENERIC"] = "1"
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=128, H=12, precision=0, max_batch=2))
            eng.load_dynamics(*blob).set_cost("humanoid_v3")
        finally:
            os.environ.pop("MPPI_FC_GENERIC", None)
        costs.append(eng.solve(x0, U0, noise=noise).costs)
        eng.close()
    np.testing.assert_allclose(costs[1], costs[0], rtol=1e-5)


def test_generic_mlp_shapes(M):
    """MLP widths / depths around the tile edges through the generic kernel: hidden 48 with 1 hidden layer and
    hidden 200 with 3, quadruped dims (37, 12), quad_est cost, exact fp32 vs the oracle rtol 1e-4."""
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    for h, hl in ((48, 1), (200, 3)):
        sd = synthetic_mlp(37, 12, h, hl, seed=h)
        for got, ref in _solve_vs_oracle(M, mlp_blob(sd, 37, 12), N.mlp_stack(sd), 37, 12, "quad_est", 0,
                                         ctx=np.array(R.QUAD_GOAL)):
            np.testing.assert_allclose(got, ref, rtol=1e-4)


# ------------------------------------------------------------------------------------------ FeatureAttention shapes

def _fa_case(M, sd, nx, nu, heads, precision, cost, K, H, seed, x0=None, ctx=None, rtol=None):
    from mppi_hip.nets import feature_attention_blob
    D = sd["feature_encoding.0.weight"].shape[0]
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=1.0, sigma=0.3, precision=precision, max_batch=1))
    eng.load_dynamics(*feature_attention_blob(sd, nx, nu, D, num_heads=heads)).set_cost(cost, ctx)
    rs = np.random.RandomState(seed)
    x0 = (0.2 * rs.randn(nx)).astype(np.float32) if x0 is None else x0
    U0 = (0.1 * rs.randn(nu, H)).astype(np.float32)
    noise = (0.3 * rs.randn(nu, H, K)).astype(np.float32)
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    eng.close()
    pre = R.Preset("fa", K=K, H=H, lam=1.0, sigma=0.3)
    dyn = N.fa_dynamics(sd, nx, nheads=heads, precision="fp32" if precision == 0 else "bf16")
    ref = R.mppi_solve(pre, dyn, R.COSTS[cost], x0, U0, noise, ctx=ctx, dtype=np.float32)
    assert np.isfinite(res.costs).all()
    np.testing.assert_allclose(res.costs, ref["costs"], rtol=rtol)
    w_own = R.softmin_weights(res.costs.astype(np.float64), 1.0)
    np.testing.assert_allclose(res.weights, w_own, atol=1e-5)


def _shapes():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("gfs", os.path.join(os.path.dirname(__file__), "golden",
                                                                      "gen_fixtures_shapes.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_fa_train_py_humanoid_net_8_heads_7_layers(M):
    """learning/train.py:71-72's FeatureAttentionStatePredictor(30 states, 21 actions, hidden 512, 8 heads, 7 layers;
    51 tokens), the oracle pinned to the reference module by tests/golden/g9_fa_h8l7_fwd.npz: bf16 rollout (K = 16,
    H = 2) vs the bf16-rounding oracle, rtol 2e-2 (seven bf16 layers), quad_est cost (reads x[0:3])."""
    mod = _shapes()
    spec = mod.SHAPES["g9_fa_h8l7_fwd"]
    sd = mod.weights(spec)
    x0 = golden("g9_fa_h8l7_fwd.npz")["x"][0, :30].astype(np.float32)
    _fa_case(M, sd, 30, 21, 8, 1, "quad_est", K=16, H=2, seed=1, x0=x0, ctx=np.array([2.0, 0.0, 1.28]), rtol=2e-2)


@pytest.mark.parametrize("precision", [0, 1])
def test_fa_76_tokens(M, precision):
    """The full humanoid state + action as tokens (55 + 21 = 76, learning/model.py:215): 5 token tiles per
    workgroup.  bf16 at hidden 128, 4 heads (the reference module's example; oracle pinned by
    tests/golden/g9_fa76_fwd.npz), rtol 1e-2 vs the bf16-rounding oracle; exact fp32 at hidden 64, rtol 1e-4.
    humanoid_v3 cost, logged x0."""
    mod = _shapes()
    sd = mod.weights(mod.SHAPES["g9_fa76_fwd"]) if precision else N_fa64()
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][1].astype(np.float32)
    _fa_case(M, sd, 55, 21, 4, precision, "humanoid_v3", K=40, H=3, seed=2, x0=x0, ctx=R.humanoid_context(),
             rtol=1e-2 if precision else 1e-4)


def N_fa64():
    from mppi_hip.nets import synthetic_feature_attention
    return synthetic_feature_attention(55, 21, 64, seed=64)


@pytest.mark.parametrize("D", [128, 512])
def test_fa_8_heads_quadruped(M, D):
    """8 attention heads (head width 16 / 64) at the quadruped's 49 tokens, bf16, K = 24, H = 3, vs the bf16-rounding
    oracle rtol 1e-2 (as test_fa_wide_bf16 for 4 heads)."""
    from mppi_hip.nets import synthetic_feature_attention
    sd = synthetic_feature_attention(37, 12, D, num_heads=8, seed=D + 8)
    _fa_case(M, sd, 37, 12, 8, 1, "quad_est", K=24, H=3, seed=3, ctx=np.array(R.QUAD_GOAL), rtol=1e-2)


def _ca_solve(M, B, K, H, seed=7, cost="humanoid_v3", terminal=0.0, wave="0", fc_ks=None):
    """One CA bf16 solve; wave: MPPI_FC_WAVE (0: off, 1 / 2: the per-wave kernel with 1 / 2 sample tiles per wave, 3:
    its 32x32x16 variant, "1d" / "2d" / "3d": with the dense layer 0 (MPPI_W32_BD=0 at load), "3b": the 112-MFMA
    block-diagonal form 1 (MPPI_W32_BD=1), None: the engine's choice); fc_ks: MPPI_FC_KS for the few-tiles kernel (None: unset)."""
    import os
    if wave is not None and wave[-1] in "db":  # "<ns>d": dense layer 0; "3b": block-diagonal form 1 (default: form 2)
        os.environ["MPPI_W32_BD"] = "0" if wave[-1] == "d" else "1"
        wave = wave[:-1]
    blob, _ = _net(M, "ca")
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][np.arange(B) % 64].astype(np.float32)
    rs = np.random.RandomState(seed)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b) if cost == "humanoid_v3" else R.humanoid_v1_context([0.05 * b, 0.1, 0.0], [-0.05, -0.1, 0.0],
                                                                                 [1.0 + 0.1 * b, 0.2, 1.28])
                    for b in range(B)]).astype(np.float32)
    if wave is not None:
        os.environ["MPPI_FC_WAVE"] = wave
    if fc_ks is not None:
        os.environ["MPPI_FC_KS"] = fc_ks
    try:
        cfg = M.Config.preset("humanoid_v3", K=K, H=H, precision=1, max_batch=B)
        cfg.terminal_weight = terminal
        eng = M.Engine(cfg)
        eng.load_dynamics(*blob).set_cost(cost)
        res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
        eng.close()
    finally:
        os.environ.pop("MPPI_FC_WAVE", None)
        os.environ.pop("MPPI_FC_KS", None)
        os.environ.pop("MPPI_W32_BD", None)
    return res, x0, U0, noise, ctx


def test_config4_24_solves_as_routed(M):
    """24 solves of config #4 (K = 1024, H = 64) = 6 sample tiles per CU, as the engine routes them by itself (the
    per-wave kernel with one sample tile per wave on MI355X): solves 0 and 23 against the bf16-emulating oracle (costs
    rtol 5e-3) and the fp32 oracle's control sequence (atol 2e-2, tie guard as test_config4_full_size).  (The
    layer-pipelined kernel this test also forced in round 3 is an A/B arm of the MPPI_AB_ARMS library only.)"""
    import os
    os.environ.pop("MPPI_FC_WAVE", None)
    blob, stack = _net(M, "ca")
    B = 24
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    rs = np.random.RandomState(45)
    U0 = (0.1 * rs.randn(B, NU, H4)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H4, K4)).astype(np.float32)
    ctx = np.stack([_ctx(b) for b in range(B)])
    eng = M.Engine(M.Config.preset("humanoid_v3", K=K4, H=H4, precision=1, max_batch=B))
    eng.load_dynamics(*blob).set_cost("humanoid_v3")
    res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
    eng.close()
    pre = R.Preset("c4", K=K4, H=H4, lam=1.0, sigma=0.75)
    for b in (0, B - 1):
        ref = R.mppi_solve(pre, _oracle_dyn(stack, "ca", "bf16"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                           ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=5e-3)
        ref32 = R.mppi_solve(pre, _oracle_dyn(stack, "ca", "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                             ctx=ctx[b], dtype=np.float32)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        dw = np.abs(w_own - ref32["weights"])
        atol = 2e-2 + (0.0 if dw.max() < 1e-3 else
                       float(np.max(np.einsum("utk,k->ut", np.abs(noise[b]).astype(np.float64), dw))))
        np.testing.assert_allclose(res.U[b], ref32["U_shifted"], atol=atol)
        np.testing.assert_allclose(res.u0[b], ref32["u0"], atol=atol)


# ------------------------------------------------------------------------------------------ per-wave CA kernel

@pytest.mark.parametrize("ns", ["1", "2", "3", "1d", "2d", "3d", "3b"])
@pytest.mark.parametrize("B,K,H,terminal", [(1, 1024, 13, 0.0), (2, 256, 7, 2.0), (5, 512, 21, 0.0), (3, 64, 3, 1.0)])
def test_wave_kernel_agrees_with_msplit_and_oracle(M, ns, B, K, H, terminal):
    """fc_wave_kernel (kernels_fc_wave.hip: every layer of NS 16-sample tiles in one wave, the weights in LDS, the
    folded LayerNorm's rstd from the Gram matrix of layer 0 before layer 0) forced on (ns "3": its 32x32x16-MFMA
    variant fc_wave32_kernel), on shapes that leave most wave
    slots idle, horizons that end mid-ring (H % (4 / NS) != 0) and a terminal cost.  Costs equal the M-split
    kernel's within 2e-3 (the same bf16 arithmetic up to the rounding points: relu(h + beta' s) rounded to bf16 and
    scaled by rstd after layer 1, instead of relu(h rstd + beta') rounded) and the bf16-emulating oracle's within 5e-3
    on the first and last solve; weights = softmin of the engine's costs."""
    got, x0, U0, noise, ctx = _ca_solve(M, B, K, H, terminal=terminal, wave=ns)
    ref_k, *_ = _ca_solve(M, B, K, H, terminal=terminal)
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got.costs, ref_k.costs, rtol=2e-3)
    _, stack = _net(M, "ca")
    pre = R.Preset("wave", K=K, H=H, lam=1.0, sigma=0.75, terminal_weight=terminal)
    for b in sorted({0, B - 1}):
        ref = R.mppi_solve(pre, _oracle_dyn(stack, "ca", "bf16"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                           ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref["costs"], rtol=5e-3)
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)


@pytest.mark.parametrize("ns", ["1", "2", "3", "1d", "3d", "3b"])
def test_wave_kernel_humanoid_v1(M, ns):
    """The per-wave kernel with the humanoid_v1 cost (the swing foot chosen by the 1-based rollout step, which the
    ring passes) against the M-split kernel, H = 150 across both phase switches."""
    got, *_ = _ca_solve(M, 3, 256, 150, cost="humanoid_v1", wave=ns)
    ref, *_ = _ca_solve(M, 3, 256, 150, cost="humanoid_v1")
    np.testing.assert_allclose(got.costs, ref.costs, rtol=2e-3)


def test_w32_block_diagonal_layer0_differs_from_dense(M):
    """fc_wave32_kernel's block-diagonal layer 0 (mppi_nets.cpp, w32_bd: uncentred bf16 rows, the row mean from the
    statistic MFMAs in the accumulators; form 2, the default, also the qpos rows' bias) is a different rounding of the
    same LayerNorm than the dense centred layer 0 (MPPI_W32_BD=0) and than form 1: costs differ pairwise (each load took
    its own image) and agree within 2e-3."""
    f2, *_ = _ca_solve(M, 4, 512, 16, wave="3")
    f1, *_ = _ca_solve(M, 4, 512, 16, wave="3b")
    dense, *_ = _ca_solve(M, 4, 512, 16, wave="3d")
    assert not np.array_equal(f2.costs, dense.costs) and not np.array_equal(f1.costs, dense.costs)
    assert not np.array_equal(f2.costs, f1.costs)
    np.testing.assert_allclose(f2.costs, dense.costs, rtol=2e-3)
    np.testing.assert_allclose(f1.costs, dense.costs, rtol=2e-3)
    for ns in ("1", "2"):  # the 16x16 per-wave kernel takes form 2 too
        bd16, *_ = _ca_solve(M, 4, 512, 16, wave=ns)
        dense16, *_ = _ca_solve(M, 4, 512, 16, wave=ns + "d")
        assert not np.array_equal(bd16.costs, dense16.costs)
        np.testing.assert_allclose(bd16.costs, dense16.costs, rtol=2e-3)


@pytest.mark.parametrize("ns", ["1", "3"])
def test_wave_kernels_negative_gamma_fall_back_to_dense(M, ns):
    """The block-diagonal layer 0 needs every LayerNorm gamma > 0 (no row negated by the fold, so -mu enters every
    row with the same sign: mppi_nets.cpp).  A CA net with two negative gammas loads the dense layer 0 instead: the
    per-wave kernels (16x16 and 32x32) still match the M-split kernel (2e-3) and the bf16-emulating oracle (5e-3)."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = dict(golden_sd("ca_humanoid_weights.npz"))
    g = np.array(sd["fusion_layer.0.weight"], np.float32).copy()
    g[[3, 200]] *= -1.0
    sd["fusion_layer.0.weight"] = g
    B, K, H = 2, 256, 9
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    rs = np.random.RandomState(47)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b) for b in range(B)])
    costs = {}
    for wave in (ns, "0"):
        os.environ["MPPI_FC_WAVE"] = wave
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=1, max_batch=B))
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost("humanoid_v3")
            costs[wave] = eng.solve(x0, U0, noise=noise, ctx=ctx).costs
            eng.close()
        finally:
            os.environ.pop("MPPI_FC_WAVE", None)
    np.testing.assert_allclose(costs[ns], costs["0"], rtol=2e-3)
    stack = N.ca_fold(sd, 28, 27, 21)
    pre = R.Preset("ng", K=K, H=H, lam=1.0, sigma=0.75)
    for b in range(B):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "bf16"), R.humanoid_v3_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        np.testing.assert_allclose(costs[ns][b], ref, rtol=5e-3)


@pytest.mark.parametrize("cost", ["humanoid_v3", "humanoid_v1"])
def test_split_bf16_wave_kernel_matches_fp32_oracle(M, cost):
    """fc_wave32_x3_kernel (split bf16 per wave, kernels_fc_x3.hip), as routed for 32 solves of K = 1024 (4 wave-tiles
    of 32 per CU, one per SIMD): costs within 1e-4 of the fp32 oracle (the fp32 bar) on the first and last solve, and
    within 1e-4 of the split-bf16 M-split kernel (MPPI_X3_WAVE=0) and of the two-wave kernel forced onto the same
    tiles (MPPI_X3_PAIR=1: fc_wave32_x3p_kernel with half of its waves idle) on every solve; weights = softmin of the
    engine's costs."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    B, K, H = 32, 1024, 12
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    rs = np.random.RandomState(48)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = (np.stack([_ctx(b) for b in range(B)]) if cost == "humanoid_v3" else
           np.stack([R.humanoid_v1_context([0.05 * b, 0.1, 0.0], [-0.05, -0.1, 0.0], [1.0 + 0.1 * b, 0.2, 1.28])
                     for b in range(B)])).astype(np.float32)
    out = {}
    for arm, env in (("wave", {}), ("msplit", {"MPPI_X3_WAVE": "0"}), ("pair", {"MPPI_X3_PAIR": "1"})):
        os.environ.update(env)
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=2, max_batch=B))
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost(cost)
            out[arm] = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True)
            eng.close()
        finally:
            for v in env:
                os.environ.pop(v, None)
    got = out["wave"]
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got.costs, out["msplit"].costs, rtol=1e-4)
    np.testing.assert_allclose(out["pair"].costs, got.costs, rtol=1e-4)
    stack = N.ca_fold(sd, 28, 27, 21)
    pre = R.Preset("x3w", K=K, H=H, lam=1.0, sigma=0.75)
    cfun = R.humanoid_v3_cost if cost == "humanoid_v3" else R.humanoid_v1_cost
    for b in (0, B - 1):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "fp32"), cfun, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref, rtol=1e-4)
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)


@pytest.mark.parametrize("H,two", [(64, True), (65, False)])
def test_split_bf16_layer1_two_products(M, H, two):
    """The split CA's layer 1 with two products (fc_common.h x3_l1_terms: W1_hi a_lo dropped when the engine's probe of
    the loaded net allows it and H <= 64; profiles/r05_x3_error_budget.txt).  34 solves of K = 1024 (the two-wave
    per-wave kernel): at H = 64 the probe of model_cross.pth keeps two products, the routed result differs from the
    three-product form (MPPI_X3_L1_TERMS=3) -- the two-product kernel ran -- and both are within 1e-4 of the fp32
    oracle on the first and last solve; at H = 65 no probe runs and the routed result IS the three-product form, bit
    for bit."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    B, K = 34, 1024
    x0_all = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"]
    x0 = x0_all[np.arange(B) % len(x0_all)].astype(np.float32)
    rs = np.random.RandomState(50)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b) for b in range(B)]).astype(np.float32)
    out = {}
    for arm, env in (("routed", {}), ("three", {"MPPI_X3_L1_TERMS": "3"})):
        os.environ.update(env)
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=2, max_batch=B))
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost("humanoid_v3")
            out[arm] = eng.solve(x0, U0, noise=noise, ctx=ctx)
            out[arm + "_l1"] = eng.x3_layer1()
            eng.close()
        finally:
            for v in env:
                os.environ.pop(v, None)
    assert out["three_l1"] == (3, -1.0)  # forced: no probe
    assert out["routed_l1"][0] == (2 if two else 3), out["routed_l1"]
    if not two:
        assert out["routed_l1"][1] == -1.0  # beyond kX3TwoTermMaxH: no probe
    got, three = out["routed"].costs, out["three"].costs
    assert np.isfinite(got).all()
    if not two:
        np.testing.assert_array_equal(got, three)
        return
    assert not np.array_equal(got, three)
    np.testing.assert_allclose(got, three, rtol=1e-4)
    stack = N.ca_fold(sd, 28, 27, 21)
    cfg = M.Config.preset("humanoid_v3", K=K, H=H)
    pre = R.Preset("x3l1", K=K, H=H, lam=1.0, sigma=0.75, terminal_weight=cfg.terminal_weight)
    for b in (0, B - 1):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        np.testing.assert_allclose(got[b], ref, rtol=1e-4)


def _offset_ca_sd(sd, c=8.0):
    """model_cross.pth with its LayerNorm beta raised by c and layer 1's bias compensated (b1 -= c W1 1): the layer-0
    activations sit ~c above zero, where the net is nearly the same function, but the dropped W1_hi a_lo term of the
    two-product layer 1 grows with them.  CPU emulation (tools/x3_error_budget.py's schemes, 16 logged states, H = 64):
    two products 3.5e-4 from the fp32 oracle, three products 2.0e-6 (model_cross: 4.95e-5 / 1.2e-6)."""
    sd = dict(sd)
    sd["fusion_layer.0.bias"] = sd["fusion_layer.0.bias"] + np.float32(c)
    sd["fusion_layer.2.bias"] = sd["fusion_layer.2.bias"] - np.float32(c) * sd["fusion_layer.2.weight"].sum(1)
    return sd


@pytest.mark.parametrize("B", [64, 8])
@pytest.mark.parametrize("which", ["model_cross", "offset"])
def test_split_layer1_probe_decides_per_net(M, which, B):
    """The two-product layer 1 is a checked property of the LOADED weights (mppi_api.hip x3_probe), not of H alone.
    At config #4's shape (K = 1024, H = 64; B = 64 routes fc_wave32_x3p_kernel, B = 8 the M-split kernels): model_cross.pth keeps two products (probe error <= 7.5e-5, kX3ProbeTol); the offset CA (_offset_ca_sd),
    for which two products break the fp32-accurate bar, gets three -- its forced two-product solve
    (MPPI_X3_L1_TERMS=2) misses the fp32 oracle by > 1e-4 while the engine's own choice stays within 1e-4 on the
    checked solves."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    if which == "offset":
        sd = _offset_ca_sd(sd)
    K, H = K4, H4
    x0_all = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"]
    x0 = x0_all[np.arange(B) % len(x0_all)].astype(np.float32)
    rs = np.random.RandomState(52)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b % 8) for b in range(B)]).astype(np.float32)
    out = {}
    for arm, env in (("engine", {}), ("forced2", {"MPPI_X3_L1_TERMS": "2"})):
        if which == "model_cross" and arm == "forced2":
            continue
        os.environ.update(env)
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=2, max_batch=B))
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost("humanoid_v3")
            res = eng.solve(x0, U0, noise=noise, ctx=ctx)
            out[arm] = (res.costs, eng.x3_layer1(), eng.rollout_kernel(), eng.x3_f16())
            eng.close()
        finally:
            for v in env:
                os.environ.pop(v, None)
    costs, (l1, err), kern = out["engine"][:3]
    f16, f16_err = out["engine"][3]
    assert np.isfinite(costs).all()
    # B = 8: the fp16 form runs fc_rollout_kernel_x3h, the two-product layer 1 fc_rollout_kernel_x3d, three products
    # fc_rollout_kernel_x3w
    assert kern.startswith("fc_wave32_x3p_kernel" if B == 64 else "fc_rollout_kernel_x3h" if f16 else
                           ("fc_rollout_kernel_x3d" if l1 == 2 else "fc_rollout_kernel_x3w")), kern
    if which == "model_cross":
        assert l1 == 2 and 0.0 <= err <= 7.5e-5, (l1, err)
        assert f16 == 1 and 0.0 <= f16_err <= 7.5e-5, (f16, f16_err)
    else:
        assert l1 == 3 and err > 7.5e-5, (l1, err)
        assert (f16 > 0) == (f16_err <= 7.5e-5), (f16, f16_err)  # the fp16 form decided on its own probe error
    # the fp16 form runs whenever its probe allows it (fc_wave32_x3p_kernel at B = 64, fc_rollout_kernel_x3h at 8)
    assert kern.endswith({2: "<f16,l2=1>", 1: "<f16>"}.get(f16, "<l1=2>" if l1 == 2 else "<l1=3>")), kern
    stack = N.ca_fold(sd, 28, 27, 21)
    cfg = M.Config.preset("humanoid_v3", K=K, H=H)
    pre = R.Preset("probe", K=K, H=H, lam=1.0, sigma=0.75, terminal_weight=cfg.terminal_weight)
    worst2 = 0.0
    for b in (0, B - 1):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        np.testing.assert_allclose(costs[b], ref, rtol=1e-4)
        if "forced2" in out:
            worst2 = max(worst2, float(np.max(np.abs(out["forced2"][0][b] - ref) / np.abs(ref))))
    if which == "offset":
        assert out["forced2"][1][0] == 2 and out["forced2"][2].endswith("<l1=2>")  # (a forced L1_TERMS: no fp16 form)
        assert worst2 > 1e-4, f"the offset net was meant to break two products (got {worst2:.2e})"


@pytest.mark.parametrize("B,K,H,cost,terminal,clamp", [
    (8, 1024, 64, "humanoid_v3", 10.0, 0.0),   # the N = 8 shard of config #4 (256 blocks of two groups)
    (16, 1024, 64, "humanoid_v3", 10.0, 0.0),  # the N = 4 shard (two rounds of blocks)
    (3, 64, 17, "humanoid_v3", 10.0, 0.5),     # ragged: cost-ring tail (17 = 2 x 8 + 1), a binding clamp
    (1, 128, 7, "humanoid_v1", 0.0, 0.0),      # a horizon shorter than the ring, the v1 cost, no terminal
    (2, 256, 1, "humanoid_v3", 10.0, 0.0),     # H = 1
])
def test_split_x3d_kernel_matches_x3w_and_oracle(M, B, K, H, cost, terminal, clamp):
    """The split M-split CA rollouts of the few-tiles shards as the engine routes them by itself.  The fp16 form
    (fc_common.h x3_f16_on, allowed by the engine's probe of model_cross.pth) runs fc_rollout_kernel_x3h
    (kernels_fc_x3h.hip: one group per block, two blocks per CU, hi fragments in registers, lo planes in LDS): within
    1e-4 of the fp32 oracle on the first and last solve (src/Humanoid_mppi_v3.jl:128-152), and so are
    fc_rollout_kernel_x3d's fp16 form (MPPI_X3H=0: two groups per block) and fc_wave32_x3p_kernel's (forced onto the
    same solves: MPPI_X3_WAVE=2, MPPI_X3_PAIR=1); among themselves x3d and x3p agree within 2e-5, x3h within 8e-5
    (its layer-0 bias as an fp16 hi / lo pair through the MFMA, its qvel k-step as one product: over 64 steps such
    rounding differences grow to the size of the fp16 form's own error); with two or four 16-sample tiles per wave
    (MPPI_X3H_NS, A/B arms) within 1e-6 of x3h itself (the same arithmetic per tile).  With that form off (MPPI_X3_F16=0) x3d runs the two-product bf16 layer 1, the
    same per-tile arithmetic as fc_rollout_kernel_x3w (MPPI_X3D=0; only the 8-step cost ring reorders each lane's cost
    sums), so costs within 1e-5 of it; weights = softmin of the engine's own costs."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    x0_all = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"]
    x0 = x0_all[np.arange(B) % len(x0_all)].astype(np.float32)
    rs = np.random.RandomState(53 + H)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b % 8) for b in range(B)]).astype(np.float32)
    out = {}
    for arm, env in (("x3h", {}), ("x3h_ns2", {"MPPI_X3H_NS": "2"}), ("x3h_ns4", {"MPPI_X3H_NS": "4"}),
                     ("x3d", {"MPPI_X3H": "0"}), ("x3d_bf16", {"MPPI_X3_F16": "0"}),
                     ("x3w", {"MPPI_X3D": "0", "MPPI_X3_F16": "0"}), ("x3p", {"MPPI_X3_WAVE": "2", "MPPI_X3_PAIR": "1"})):
        os.environ.update(env)
        try:
            cfg = M.Config.preset(cost, K=K, H=H, precision=2, max_batch=B, ctrl_clamp=clamp)
            cfg.terminal_weight = terminal
            eng = M.Engine(cfg)
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost(cost)
            out[arm] = (eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True), eng.rollout_kernel())
            eng.close()
        finally:
            for v in env:
                os.environ.pop(v, None)
    (got, kern), (got_d, kern_d), (got_b, kern_b), (ref_k, kern_w), (got_p, kern_p) = (
        out[a] for a in ("x3h", "x3d", "x3d_bf16", "x3w", "x3p"))
    assert kern == "fc_rollout_kernel_x3h<f16>", kern
    assert kern_d == "fc_rollout_kernel_x3d<f16>", kern_d
    for ns in (2, 4):  # NS tiles per wave (kernels_fc_x3h.hip x3h_ns): the same products, in the same order per tile
        got_n, kern_n = out[f"x3h_ns{ns}"]
        assert kern_n == f"fc_rollout_kernel_x3hw<f16,ns={ns}>", kern_n
        np.testing.assert_allclose(got_n.costs, got.costs, rtol=1e-6)
    assert kern_b == "fc_rollout_kernel_x3d<l1=2>", kern_b
    assert kern_w.startswith("fc_rollout_kernel_x3"), kern_w
    assert kern_p == "fc_wave32_x3p_kernel<f16>", kern_p
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got_b.costs, ref_k.costs, rtol=1e-5)
    assert not np.array_equal(got.costs, got_b.costs)
    stack = N.ca_fold(sd, 28, 27, 21)
    pre = R.Preset("x3d", K=K, H=H, lam=cfg.lambda_, sigma=0.75, ctrl_clamp=clamp, terminal_weight=terminal)
    cfun = R.humanoid_v3_cost if cost == "humanoid_v3" else R.humanoid_v1_cost
    for b in sorted({0, B - 1}):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "fp32"), cfun, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        for arm, res in (("x3h", got), ("x3d", got_d), ("x3p", got_p)):  # every kernel of the fp16 form: the bar
            np.testing.assert_allclose(res.costs[b], ref, rtol=1e-4, err_msg=arm)
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)
    # the kernels among themselves: x3d and x3p differ in summation order and in x3p's one-product qvel k-step (state
    # slots 32..47 of the qvel rows), x3h in its bias rounding and its one-product qvel k-step (slots 32..63)
    np.testing.assert_allclose(got_d.costs, got_p.costs, rtol=2e-5)
    np.testing.assert_allclose(got.costs, got_d.costs, rtol=8e-5)
    np.testing.assert_allclose(got.costs, got_p.costs, rtol=8e-5)


def test_split_bf16_wave_kernel_edges(M):
    """fc_wave32_x3_kernel (kernels_fc_x3.hip) on the edges of its routing and of the horizon loop: K = 992 (31
    wave-tiles per solve, no padding), 34 solves (1054 wave-tiles: just over 4 per CU), an odd horizon H = 7 (the
    2-step cost ring's tail flush), a control clamp that binds (|U + eps| > 0.5 for most samples) and the terminal
    cost.  Costs within 1e-4 of the fp32 oracle on the first and last solve and of the M-split split-bf16 kernel
    (MPPI_X3_WAVE=0) on every solve, and not bitwise equal to the latter (the per-wave kernel ran)."""
    import os
    from mppi_hip.nets import cross_attention_blob
    sd = golden_sd("ca_humanoid_weights.npz")
    B, K, H, clamp = 34, 992, 7, 0.5
    x0_all = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"]
    x0 = x0_all[np.arange(B) % len(x0_all)].astype(np.float32)
    rs = np.random.RandomState(49)
    U0 = (0.1 * rs.randn(B, NU, H)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H, K)).astype(np.float32)
    ctx = np.stack([_ctx(b) for b in range(B)]).astype(np.float32)
    out = {}
    for wave in ("1", "0"):
        os.environ["MPPI_X3_WAVE"] = wave
        try:
            eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=2, max_batch=B, ctrl_clamp=clamp))
            eng.load_dynamics(*cross_attention_blob(sd)).set_cost("humanoid_v3")
            out[wave] = eng.solve(x0, U0, noise=noise, ctx=ctx)
            eng.close()
        finally:
            os.environ.pop("MPPI_X3_WAVE", None)
    got = out["1"]
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got.costs, out["0"].costs, rtol=1e-4)
    assert not np.array_equal(got.costs, out["0"].costs)
    stack = N.ca_fold(sd, 28, 27, 21)
    cfg = M.Config.preset("humanoid_v3", K=K, H=H)
    assert cfg.terminal_weight > 0
    pre = R.Preset("x3e", K=K, H=H, lam=1.0, sigma=0.75, ctrl_clamp=clamp, terminal_weight=cfg.terminal_weight)
    for b in (0, B - 1):
        ref = R.rollout(pre, _oracle_dyn(stack, "ca", "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b], ctx=ctx[b],
                        dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref, rtol=1e-4)


def test_wave_kernel_config4_64_solves(M):
    """BASELINE config #4 as benched on one GPU: 64 solves, K = 1024, H = 64, logged x0, a different real-env context
    per solve -- the batch the engine routes to the per-wave kernel by itself (NS = 2).  Solves 0, 37 and 63 against
    the bf16-emulating oracle (costs rtol 5e-3) and the fp32 oracle's control sequence (atol 2e-2 with the tie guard);
    every solve's weights / U from the engine's own costs."""
    import os
    os.environ.pop("MPPI_FC_WAVE", None)
    blob, stack = _net(M, "ca")
    B = 64
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    rs = np.random.RandomState(46)
    U0 = (0.1 * rs.randn(B, NU, H4)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H4, K4)).astype(np.float32)
    ctx = np.stack([_ctx(b % 8) for b in range(B)])
    eng = M.Engine(M.Config.preset("humanoid_v3", K=K4, H=H4, precision=1, max_batch=B))
    eng.load_dynamics(*blob).set_cost("humanoid_v3")
    res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
    eng.close()
    assert np.isfinite(res.costs).all()
    pre = R.Preset("c4", K=K4, H=H4, lam=1.0, sigma=0.75)
    for b in (0, 37, 63):
        ref = R.mppi_solve(pre, _oracle_dyn(stack, "ca", "bf16"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                           ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(res.costs[b], ref["costs"], rtol=5e-3)
        ref32 = R.mppi_solve(pre, _oracle_dyn(stack, "ca", "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                             ctx=ctx[b], dtype=np.float32)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        dw = np.abs(w_own - ref32["weights"])
        atol = 2e-2 + (0.0 if dw.max() < 1e-3 else
                       float(np.max(np.einsum("utk,k->ut", np.abs(noise[b]).astype(np.float64), dw))))
        np.testing.assert_allclose(res.U[b], ref32["U_shifted"], atol=atol)
        np.testing.assert_allclose(res.u0[b], ref32["u0"], atol=atol)
    for b in range(B):
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)


def _mlp_solve(M, B, K, H, wave, nx=NX, nu=NU, cost="humanoid_v3", terminal=0.0, seed=11, precision=1, env="MPPI_FC_WAVE"):
    """One MLP solve (seeded MLPStatePredictor(nx, nu, 128, 2); bf16, or precision 2: split bf16) with the routing
    variable `env` (MPPI_FC_WAVE, or MPPI_X3M for the split per-wave kernel) set to `wave` (None: the engine's
    choice)."""
    import os
    from mppi_hip.nets import mlp_blob, synthetic_mlp
    sd = synthetic_mlp(nx, nu, seed=0)
    rs = np.random.RandomState(seed)
    if nx == NX:
        x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][np.arange(B) % 64].astype(np.float32)
        ctx = np.stack([_ctx(b % 8) for b in range(B)]).astype(np.float32)
        preset = "humanoid_v3"
    else:
        x0 = (0.2 * rs.randn(B, nx)).astype(np.float32)
        ctx = np.tile(np.array(list(R.QUAD_GOAL) + [0.0] * (8 - len(R.QUAD_GOAL)), np.float32), (B, 1))
        preset = "quad_est"
    U0 = (0.1 * rs.randn(B, nu, H)).astype(np.float32)
    noise = (0.4 * rs.randn(B, nu, H, K)).astype(np.float32)
    os.environ.pop(env, None)
    if wave is not None:
        os.environ[env] = wave
    try:
        cfg = M.Config.preset(preset, K=K, H=H, precision=precision, max_batch=B)
        cfg.terminal_weight = terminal
        eng = M.Engine(cfg)
        eng.load_dynamics(*mlp_blob(sd, nx, nu)).set_cost(cost)
        res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True)
        eng.close()
    finally:
        os.environ.pop(env, None)
    return res, sd, x0, U0, noise, ctx, cfg


@pytest.mark.parametrize("B,K,H,terminal,quad", [(1, 1024, 13, 0.0, False), (2, 256, 7, 2.0, False),
                                                 (3, 48, 3, 1.0, False), (2, 512, 9, 10.0, True)])
@pytest.mark.parametrize("switch", ["MPPI_X3M", "MPPI_X3M32"])
def test_split_mlp_wave_kernel_matches_fp32_oracle(M, switch, B, K, H, terminal, quad):
    """fc_wave_mlp_x3_kernel (kernels_fc_x3m.hip: the split-bf16 MLPStatePredictor(nx, nu, 128, 2) rollout, all 4
    layers of 16 samples in one wave, hi fragments and layers 0 / 3's lo in LDS, the hidden layers' lo from L2)
    forced on (MPPI_X3M=1): the humanoid MLP (55 states, 21 controls, humanoid_v3 with a per-solve context) and the
    quadruped shape (37, 12, quad_est), ragged batches (K = 48: three 16-sample tiles per solve), short horizons, a
    terminal cost.  Costs against the FP32 oracle at rtol 1e-4 (the fp32-accurate bar) and against the M-split split
    kernel (MPPI_X3M=0) at 1e-5; weights = softmin of the engine's own costs.  MPPI_X3M32: fc_wave32_mlp_x3_kernel
    (kernels_fc_x3mp.hip, 32 samples per wave on 32x32x16 MFMAs) forced on the same cases, against the same bars."""
    kw = dict(nx=37, nu=12, cost="quad_est") if quad else {}
    got, sd, x0, U0, noise, ctx, cfg = _mlp_solve(M, B, K, H, "1", terminal=terminal, precision=2, env=switch, **kw)
    ref_k, *_ = _mlp_solve(M, B, K, H, "0", terminal=terminal, precision=2, env=switch, **kw)
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got.costs, ref_k.costs, rtol=1e-5)
    nx = kw.get("nx", NX)
    pre = R.Preset("wmlpx3", K=K, H=H, lam=cfg.lambda_, sigma=cfg.sigma, terminal_weight=terminal)
    for b in sorted({0, B - 1}):
        ref = R.mppi_solve(pre, N.learned_dynamics(N.mlp_stack(sd), nx, precision="fp32"),
                           R.COSTS[kw.get("cost", "humanoid_v3")], x0[b], U0[b], noise[b], ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref["costs"], rtol=1e-4)
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)


@pytest.mark.parametrize("ns", ["1", "2"])
@pytest.mark.parametrize("B,K,H,terminal,quad", [(1, 1024, 13, 0.0, False), (2, 256, 7, 2.0, False),
                                                 (3, 64, 3, 1.0, False), (2, 512, 9, 10.0, True)])
def test_wave_mlp_kernel_agrees_with_msplit_and_oracle(M, ns, B, K, H, terminal, quad):
    """fc_wave_mlp_kernel (kernels_fc_wave.hip: all 4 layers of MLPStatePredictor(nx, nu, 128, 2) for NS tiles in one
    wave, weights in LDS, the controls as layer 0's third k-step) forced on: the humanoid MLP (55 states, 21 controls,
    humanoid_v3 cost with a per-solve real-env context) and the quadruped shape (37, 12, quad_est cost), ragged shapes,
    H % (4 / NS) != 0, a terminal cost.  Costs equal the M-split kernel's within 2e-3 (the same bf16 operands; layer
    0's bias as a bf16 hi / lo pair in the MFMA instead of an fp32 add) and the bf16-emulating oracle's within 5e-3;
    weights = softmin of the engine's costs."""
    kw = dict(nx=37, nu=12, cost="quad_est") if quad else {}
    got, sd, x0, U0, noise, ctx, cfg = _mlp_solve(M, B, K, H, ns, terminal=terminal, **kw)
    ref_k, *_ = _mlp_solve(M, B, K, H, "0", terminal=terminal, **kw)
    assert np.isfinite(got.costs).all()
    np.testing.assert_allclose(got.costs, ref_k.costs, rtol=2e-3)
    nx = kw.get("nx", NX)
    pre = R.Preset("wmlp", K=K, H=H, lam=cfg.lambda_, sigma=cfg.sigma, terminal_weight=terminal)
    for b in sorted({0, B - 1}):
        ref = R.mppi_solve(pre, N.learned_dynamics(N.mlp_stack(sd), nx, precision="bf16"), R.COSTS[kw.get("cost", "humanoid_v3")],
                           x0[b], U0[b], noise[b], ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref["costs"], rtol=5e-3)
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)


def _u_vs_fp32(res_U, res_u0, w_own, ref32, noise_b, atol, key="U_shifted"):
    """U, u0 against the fp32 oracle's control sequence (src/Humanoid_mppi_v3.jl:154-179), with the tie guard of
    SURVEY 8d when the softmin is not well conditioned (the bound sum_k |w_own - w_ref|_k |eps_k| added)."""
    dw = np.abs(w_own - ref32["weights"])
    if dw.max() >= 1e-3:
        atol = atol + float(np.max(np.einsum("utk,k->ut", np.abs(noise_b).astype(np.float64), dw)))
    np.testing.assert_allclose(res_U, ref32[key], atol=atol)
    np.testing.assert_allclose(res_u0, ref32["u0"], atol=atol)
    return dw.max() < 1e-3


def test_wave_mlp_kernel_humanoid_64_solves(M):
    """The humanoid MLP at config #4's batch (64 solves, K = 1024, H = 64), routed to the per-wave kernel by the engine
    itself: solves 0 and 63 against the bf16-emulating oracle (costs rtol 5e-3), and, for this action-sensitive net
    (its U check exercises the dynamics, unlike the CA's), the same best sample as the fp32 oracle and U / u0 against
    the fp32 oracle's control sequence (atol 2e-2, the bf16 bar, with the tie guard)."""
    got, sd, x0, U0, noise, ctx, cfg = _mlp_solve(M, 64, K4, H4, None)
    assert np.isfinite(got.costs).all()
    pre = R.Preset("wmlp64", K=K4, H=H4, lam=cfg.lambda_, sigma=cfg.sigma, terminal_weight=cfg.terminal_weight)
    for b in (0, 63):
        ref = R.mppi_solve(pre, N.learned_dynamics(N.mlp_stack(sd), NX, precision="bf16"), R.humanoid_v3_cost, x0[b],
                           U0[b], noise[b], ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(got.costs[b], ref["costs"], rtol=5e-3)
        ref32 = R.mppi_solve(pre, N.learned_dynamics(N.mlp_stack(sd), NX, precision="fp32"), R.humanoid_v3_cost,
                             x0[b], U0[b], noise[b], ctx=ctx[b], dtype=np.float32)
        assert int(np.argmin(got.costs[b])) == int(np.argmin(ref32["costs"]))
        w_own = R.softmin_weights(got.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(got.weights[b], w_own, atol=1e-5)
        _u_vs_fp32(got.U[b], got.u0[b], w_own, ref32, noise[b], 2e-2, key="U_new")  # (no shift in _mlp_solve)


@pytest.mark.parametrize("net", ["ca", "ca_f16l2x1", "ca_bf16l1", "mlp"])
def test_config4_64_solves_fp32_accurate(M, net):
    """BASELINE config #4 exactly as the default bench line runs it (bench.py: 64 solves, K = 1024, H = 64, logged x0,
    a real-env context per solve, shift on) in the fp32-accurate split mode (precision 2).  The kernel that ran is
    asserted (mppi_rollout_kernel): the CA routes to fc_wave32_x3p_kernel in its fp16 form (fc_common.h x3_f16_on)
    that the engine's probe of model_cross.pth allows (mppi_x3_f16: 1, probe error <= 7.5e-5); ca_f16l2x1 = the opt-in
    one-product last layer (MPPI_X3_F16_L2=1, x3_f16_l2x1; checked at 2e-4: not fp32-accurate on every state);
    ca_bf16l1 = the fp16 form off (MPPI_X3_F16=0): the two-product bf16 layer 1 (mppi_x3_layer1: 2 products, probe
    error <= 7.5e-5); the MLP routes to fc_wave32_mlp_x3_kernel.  Solves 0, 37 and 63 against the FP32 oracle (the reference evaluates the net in fp32
    torch, src/cartpole_mppi_estimator.py:89-93, learning/model.py): costs rtol 1e-4; weights = softmin of the
    engine's own costs (atol 1e-5); U / u0 against the fp32 oracle's control sequence at atol 1e-4 with the tie guard
    (src/Humanoid_mppi_v3.jl:154-179); the MLP's peaked weights (cost gaps of hundreds) must pick the fp32 oracle's
    best sample."""
    import os
    os.environ.pop("MPPI_X3_WAVE", None)
    blob, stack = _net(M, "ca" if net.startswith("ca") else net)
    B = 64
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][:B].astype(np.float32)
    rs = np.random.RandomState(50)
    U0 = (0.1 * rs.randn(B, NU, H4)).astype(np.float32)
    noise = (0.75 * rs.randn(B, NU, H4, K4)).astype(np.float32)
    ctx = np.stack([_ctx(b % 8) for b in range(B)])
    if net == "ca_bf16l1":
        os.environ["MPPI_X3_F16"] = "0"
    if net == "ca_f16l2x1":
        os.environ["MPPI_X3_F16_L2"] = "1"
    try:
        eng = M.Engine(M.Config.preset("humanoid_v3", K=K4, H=H4, precision=2, max_batch=B))
        eng.load_dynamics(*blob).set_cost("humanoid_v3")
        res = eng.solve(x0, U0, noise=noise, ctx=ctx, want_weights=True, shift=True)
        kern, (l1, l1_err), (f16, f16_err) = eng.rollout_kernel(), eng.x3_layer1(), eng.x3_f16()
        eng.close()
    finally:
        os.environ.pop("MPPI_X3_F16", None)
        os.environ.pop("MPPI_X3_F16_L2", None)
    if net == "ca":
        assert kern == "fc_wave32_x3p_kernel<f16>", kern
        assert f16 == 1 and 0.0 <= f16_err <= 7.5e-5, (f16, f16_err)
        assert l1 == 2 and 0.0 <= l1_err <= 7.5e-5, (l1, l1_err)
    elif net == "ca_f16l2x1":
        assert kern == "fc_wave32_x3p_kernel<f16,l2=1>", kern
        assert f16 == 2, f16
    elif net == "ca_bf16l1":
        assert kern == "fc_wave32_x3p_kernel<l1=2>", kern
        assert not f16
        assert l1 == 2 and 0.0 <= l1_err <= 7.5e-5, (l1, l1_err)
    else:
        assert kern == "fc_wave32_mlp_x3_kernel", kern
        assert l1 == 0
    assert np.isfinite(res.costs).all()
    pre = R.Preset("c4", K=K4, H=H4, lam=1.0, sigma=0.75)
    well = 0
    tol = 2e-4 if net == "ca_f16l2x1" else 1e-4
    for b in (0, 37, 63):
        ref32 = R.mppi_solve(pre, _oracle_dyn(stack, net, "fp32"), R.humanoid_v3_cost, x0[b], U0[b], noise[b],
                             ctx=ctx[b], dtype=np.float32)
        np.testing.assert_allclose(res.costs[b], ref32["costs"], rtol=tol)
        w_own = R.softmin_weights(res.costs[b].astype(np.float64), pre.lam)
        np.testing.assert_allclose(res.weights[b], w_own, atol=1e-5)
        well += _u_vs_fp32(res.U[b], res.u0[b], w_own, ref32, noise[b], tol)
        if net == "mlp":
            assert int(np.argmin(res.costs[b])) == int(np.argmin(ref32["costs"]))
    assert well == 3, "the checked solves were expected to be well conditioned"
