"""The compiled CPU restatement (oracle/mppi_cpu.c, the multi-core CPU baseline) against the reference's G7 solve
fixture and the numpy oracle. CPU-only."""
import numpy as np
import pytest

from conftest import golden, golden_sd
from oracle import cpu as C
from oracle import mppi_ref as R
from oracle import nets_ref as N


@pytest.fixture(scope="module", autouse=True)
def _built():
    C.build()


@pytest.mark.parametrize("threads", [1, 4])
def test_c_ca_humanoid_solve_matches_reference_fixture(threads):
    """G7: CrossAttention humanoid solve (K=128, H=16) generated with the reference's learning/model.py."""
    g = golden("g7_ca_humanoid_solve.npz")
    sd = golden_sd("ca_humanoid_weights.npz")
    net = C.FcNet(N.ca_fold(sd, 28, 27, 21))
    r = C.fc_solve(net, 55, 21, "humanoid_v3", g["x0"], g["U0"], g["noise"], lam=float(g["lam"]), ctx=g["ctx"],
                   threads=threads)
    np.testing.assert_allclose(r["costs"], g["costs"], rtol=1e-4)
    np.testing.assert_allclose(r["weights"], g["weights"], atol=1e-4)
    np.testing.assert_allclose(r["U_new"], g["U_new"], atol=1e-4)


@pytest.mark.parametrize("cost,nx,nu,preset", [("quad_est", 37, 12, "quad_est"), ("quad_jl", 37, 12, "quad_mppi_jl"),
                                               ("humanoid_v3", 55, 21, "humanoid_v3")])
def test_c_mlp_solve_matches_numpy_oracle(cost, nx, nu, preset):
    """MLP dynamics (learning/model.py:6-46) with every cost and preset flavour (clamp, eps-norm, replace)."""
    rs = np.random.RandomState(1)
    stack = [dict(W=0.1 * rs.randn(64, nx + nu), b=0.01 * rs.randn(64), ln=None, relu=True),
             dict(W=0.1 * rs.randn(64, 64), b=0.01 * rs.randn(64), ln=None, relu=True),
             dict(W=0.01 * rs.randn(nx, 64), b=0.001 * rs.randn(nx), ln=None, relu=False)]
    pre = R.PRESETS[preset]
    K, H = 75, 9  # K not a multiple of the 16-sample block
    x0 = 0.1 * rs.randn(nx)
    x0[3] = 1.0
    U = 0.2 * rs.randn(nu, H)
    noise = pre.sigma * rs.randn(nu, H, K)
    ctx = R.humanoid_context() if cost == "humanoid_v3" else np.array([2.0, 0.0, 0.35, 0, 0, 0, 0, 0])
    dyn = N.learned_dynamics(stack, nx, precision="fp32")
    ref = R.mppi_solve(pre, dyn, R.COSTS[cost], x0.astype(np.float32), U, noise, ctx=ctx, dtype=np.float32)
    r = C.fc_solve(C.FcNet(stack), nx, nu, cost, x0, U, noise, lam=pre.lam, ctrl_clamp=pre.ctrl_clamp,
                   U_clamp=pre.U_clamp, norm_eps=pre.norm_eps, terminal_weight=pre.terminal_weight,
                   replace=pre.update == "replace", ctx=ctx, threads=3)
    np.testing.assert_allclose(r["costs"], ref["costs"], rtol=2e-5)
    np.testing.assert_allclose(r["U_new"], ref["U_new"], atol=1e-4)  # atol 1e-4 on U (fp32 order)


@pytest.mark.parametrize("x0", [np.zeros(4), np.array([0.0, np.pi, 0.0, 0.0])])
def test_c_cartpole_solve_matches_numpy_oracle(x0):
    K, H = 128, 30  # BASELINE config #1
    noise = R.reference_noise(0, 1, H, K, 1.0)
    U = 0.3 * np.ones((1, H))
    ref = R.mppi_solve(R.Preset("c1", K=K, H=H, lam=1.0, sigma=1.0), R.cartpole_step, R.cartpole_running_cost, x0, U,
                       noise)
    r = C.cartpole_solve(x0, U, noise, threads=4)
    np.testing.assert_allclose(r["costs"], ref["costs"], rtol=1e-12)
    np.testing.assert_allclose(r["weights"], ref["weights"], atol=1e-12)
    np.testing.assert_allclose(r["U_new"], ref["U_new"], atol=1e-12)
