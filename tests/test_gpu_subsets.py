"""BASELINE configs #3 and #5 and the D = 512 FeatureAttention net at FULL size (every K and H the bench runs) against
the oracle, through sample subsets.  Needs an MI355X.

The K samples of one solve are independent (src/cartpole_mppi.py:62 loops them one by one; src/Humanoid_mppi_v3.jl:131
threads over them), so the engine runs the whole solve with injected seeded noise and the oracle rolls out only a
subset of the noise columns (the first and last samples and a seeded spread in between): those samples' costs must
match one for one.  The tolerances are the parity bar of tests/test_gpu_parity.py:

  fp32 engine  vs the fp32 oracle:                       costs rtol 1e-4
  bf16 engine  vs the bf16-emulating oracle (weights and every layer input rounded to bf16, fp32 accumulate; the
               LayerNorm folded as the kernel folds it):  costs rtol 5e-3 (fc nets), 1e-2 (FA nets, as test_fa_wide_bf16)

Then the update: the engine's weights are the softmin of its own costs and U is the replace / add update they give
(torch float64 over all K), so the subset checks plus this pin the whole solve.
"""
import numpy as np
import pytest

from conftest import golden, golden_sd
from oracle import mppi_ref as R
from oracle import nets_ref as N

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(gpu_available):
    import mppi_hip
    return mppi_hip


def _subset(K, n, seed):
    """n sample columns of K: the first and last 4 and a seeded spread."""
    rs = np.random.RandomState(seed)
    mid = rs.choice(np.arange(4, K - 4), n - 8, replace=False)
    return np.unique(np.concatenate([np.arange(4), mid, np.arange(K - 4, K)]))


def _check_update(res, pre, U0, noise, lam):
    """weights = softmin(own costs / lambda); U = the update those weights give (replace or add), float64."""
    w_own = R.softmin_weights(res.costs.astype(np.float64), lam)
    np.testing.assert_allclose(res.weights, w_own, atol=1e-5)
    Un = R.update_U(pre, U0.astype(np.float64), noise.astype(np.float64), res.weights.astype(np.float64))
    np.testing.assert_allclose(res.U, Un, atol=2e-5)


@pytest.mark.parametrize("precision", [1, 0, 2])
def test_config3_quad_mlp_full_size_subset(M, precision):
    """Config #3 exactly as benched (bench.py --workload quad_mlp): the quadruped MLPStatePredictor(37, 12, 128, 2)
    trained on the reference's quad_data logs (tests/golden/quad_mlp_trained.npz), x0 a logged state, preset quad_est
    (src/quadruped_mppi_estimator.py:38-41: K = 2048, H = 40, lambda 10, sigma 0.4, replace update), against the
    oracle on 64 of the 2048 samples (:58-95)."""
    K, H, nx, nu = 2048, 40, 37, 12
    sd = golden_sd("quad_mlp_trained.npz", prefix="")
    sd = {k: v for k, v in sd.items() if k.startswith("network.")}
    logs = golden("quad_logs.npz")
    x0 = np.ascontiguousarray(logs["states0"][2::40][0], np.float32)
    rs = np.random.RandomState(31)
    U0 = (0.1 * rs.randn(nu, H)).astype(np.float32)
    noise = (0.4 * rs.randn(nu, H, K)).astype(np.float32)
    eng = M.Engine(M.Config.preset("quad_est", K=K, H=H, precision=precision))
    eng.load_dynamics(*M.mlp_blob(sd, nx, nu)).set_cost("quad_est")
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    eng.close()
    assert np.isfinite(res.costs).all()
    idx = _subset(K, 64, 3)
    pre = R.Preset("c3", K=len(idx), H=H, lam=10.0, sigma=0.4, update="replace")
    prec = "bf16" if precision == 1 else "fp32"
    ref = R.rollout(pre, N.learned_dynamics(N.mlp_stack(sd), nx, precision=prec), R.quad_est_running_cost, x0, U0,
                    noise[:, :, idx], ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    np.testing.assert_allclose(res.costs[idx], ref, rtol=5e-3 if precision == 1 else 1e-4)  # 2: split bf16, fp32 bar
    _check_update(res, R.Preset("c3", K=K, H=H, lam=10.0, sigma=0.4, update="replace"), U0, noise, 10.0)


@pytest.mark.parametrize("layered", [False, True])
def test_fa_d512_full_size_subset(M, layered, monkeypatch):
    """The quadruped FeatureAttention net at hidden 512 (4 heads, 2 layers, 49 tokens; seeded weights, the checkpoint
    is missing) at the config #3 shape (K = 2048, H = 40, bf16, quad_est, replace update): 8 samples against the
    bf16-emulating oracle FA forward (oracle/nets_ref.py::fa_forward_engine), rtol 1e-2."""
    from mppi_hip.nets import feature_attention_blob, synthetic_feature_attention
    K, H, nx, nu = 2048, 40, 37, 12
    sd = synthetic_feature_attention(nx, nu, 512, seed=0)
    rs = np.random.RandomState(32)
    x0 = (0.1 * rs.randn(nx)).astype(np.float32)
    U0 = (0.05 * rs.randn(nu, H)).astype(np.float32)
    noise = (0.4 * rs.randn(nu, H, K)).astype(np.float32)
    if layered:  # the layer-by-layer path (kernels_fa_layered.hip), else the fused fa_rollout_kernel
        monkeypatch.setenv("MPPI_FA_LAYERED", "1")
    eng = M.Engine(M.Config(nx=nx, nu=nu, H=H, K=K, lambda_=10.0, sigma=0.4, precision=1, update_mode=1,
                            shift_fill=0.1, terminal_weight=10.0))
    eng.load_dynamics(*feature_attention_blob(sd, nx, nu, 512)).set_cost("quad_est")
    res = eng.solve(x0, U0, noise=noise, want_weights=True)
    eng.close()
    assert np.isfinite(res.costs).all() and res.costs.std() > 0
    idx = np.array([0, 1, 517, 1024, 1500, 2000, 2046, 2047])
    pre = R.Preset("fa", K=len(idx), H=H, lam=10.0, sigma=0.4, update="replace", terminal_weight=10.0)
    ref = R.rollout(pre, N.fa_dynamics(sd, nx, precision="bf16"), R.quad_est_running_cost, x0, U0, noise[:, :, idx],
                    ctx=np.array([2.0, 0.0, 0.35]), dtype=np.float32)
    np.testing.assert_allclose(res.costs[idx], ref, rtol=1e-2)
    _check_update(res, R.Preset("fa", K=K, H=H, lam=10.0, sigma=0.4, update="replace"), U0, noise, 10.0)


def _bounded_mlp(nx, nu):
    """The seeded humanoid MLPStatePredictor(55, 21, 128, 2) with its output layer scaled by 0.3: over config #5's 128
    steps the unscaled net's rollouts diverge (costs ~2e6), where single bf16 rounding differences are amplified past
    any parity bar; scaled, the rollouts stay bounded (costs ~1.6e4) and the net stays action-sensitive."""
    from mppi_hip.nets import synthetic_mlp
    sd = dict(synthetic_mlp(nx, nu, seed=0))
    sd["network.6.weight"] = (0.3 * sd["network.6.weight"]).astype(np.float32)
    sd["network.6.bias"] = (0.3 * sd["network.6.bias"]).astype(np.float32)
    return sd


@pytest.mark.parametrize("precision", [1, 2])
@pytest.mark.parametrize("net", ["ca", "mlp"])
def test_config5_full_size_subset(M, net, precision):
    """Config #5's solve (K = 8192, H = 128, the humanoid CA surrogate of checkpoints/model_cross.pth; and an
    action-sensitive humanoid MLP at the same shape, _bounded_mlp), one solve with a real-env context: 64 of the 8192
    samples against the oracle (src/Humanoid_mppi_v3.jl:128-170): bf16 (BASELINE config #5's precision) against the
    bf16-emulating oracle, rtol 5e-3; the fp32-accurate split mode (precision 2) against the fp32 oracle, rtol 1e-4."""
    from mppi_hip.nets import cross_attention_blob, mlp_blob
    K, H, nx, nu = 8192, 128, 55, 21
    if net == "ca":
        sd = golden_sd("ca_humanoid_weights.npz")
        blob, stack = cross_attention_blob(sd), N.ca_fold(sd, 28, 27, 21)
        if precision == 1:
            stack = N.ln_fold(stack)
    else:
        sd = _bounded_mlp(nx, nu)
        blob, stack = mlp_blob(sd, nx, nu), N.mlp_stack(sd)
    x0 = golden("g5_ca_humanoid_fwd.npz")["x0_stride20"][7].astype(np.float32)
    rs = np.random.RandomState(33)
    U0 = (0.1 * rs.randn(nu, H)).astype(np.float32)
    noise = (0.75 * rs.randn(nu, H, K)).astype(np.float32)
    ctx = R.humanoid_context(swing_foot_x=0.1, swing_knee_x=0.05, swing_vx=0.2, foot_clearance=0.02,
                             leg_clearance=-0.01)
    eng = M.Engine(M.Config.preset("humanoid_v3", K=K, H=H, precision=precision))
    eng.load_dynamics(*blob).set_cost("humanoid_v3")
    res = eng.solve(x0, U0, noise=noise, ctx=ctx[None], want_weights=True)
    eng.close()
    assert np.isfinite(res.costs).all()
    idx = _subset(K, 64, 5)
    pre = R.Preset("c5", K=len(idx), H=H, lam=1.0, sigma=0.75)
    ref = R.rollout(pre, N.learned_dynamics(stack, nx, precision="bf16" if precision == 1 else "fp32"),
                    R.humanoid_v3_cost, x0, U0, noise[:, :, idx], ctx=ctx, dtype=np.float32)
    np.testing.assert_allclose(res.costs[idx], ref, rtol=5e-3 if precision == 1 else 1e-4)
    _check_update(res, R.Preset("c5", K=K, H=H, lam=1.0, sigma=0.75), U0, noise, 1.0)


def test_split_bf16_scope(M):
    """MPPI_PREC_BF16X3 is built for the register-resident fc shapes (humanoid CA, MLP 128 x 2): a FeatureAttention
    net or another fc shape is refused with MPPI_E_UNSUPPORTED at mppi_load_dynamics, not run at another precision."""
    from mppi_hip import _lib as L
    from mppi_hip.nets import feature_attention_blob, mlp_blob, synthetic_feature_attention, synthetic_mlp
    eng = M.Engine(M.Config(nx=4, nu=1, H=4, K=64, precision=2))
    with pytest.raises(M.MPPIError) as e:
        eng.load_dynamics(*feature_attention_blob(synthetic_feature_attention(4, 1, 64, seed=0), 4, 1, 64))
    assert e.value.code == L.MPPI_E_UNSUPPORTED
    with pytest.raises(M.MPPIError) as e:
        eng.load_dynamics(*mlp_blob(synthetic_mlp(4, 1, hidden_dim=64, seed=0), 4, 1))
    assert e.value.code == L.MPPI_E_UNSUPPORTED
    eng.close()
