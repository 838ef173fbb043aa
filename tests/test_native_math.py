"""The device math helpers that replace libm in the rollout kernels, built host-only (they are __host__ __device__):
csrc/costs.h::sincos_fast / cos_fast (Cephes sinf/cosf reduction and polynomials, used by the analytic cartpole
dynamics, src/cartpole_mppi.py's mj_step restatement, and the cartpole costs, src/cartpole_mppi.py:44-50 /
src/cartpole_mppi_estimator.py:46-52) against double-precision libm.  CPU only."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def test_sincos_fast_accuracy(tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    exe = str(tmp_path / "trig_check")
    cmd = [HIPCC, "-x", "hip", "--offload-host-only", "-O2", "-std=c++17", f"-I{REPO}/include",
           os.path.join(REPO, "tests", "native", "trig_check.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120, check=True).stdout.split("\n")
    for line in out[:3]:
        lim, es, ec, e1 = (float(v) for v in line.split())
        assert es < 1e-7 and ec < 1e-7, line  # libm float: 3.3e-8; the fp32 parity bar: cost rtol 1e-5
        assert e1 == 0.0  # cos_fast is sincos_fast's cosine
    assert out[3] == "nonfinite 1"  # NaN / inf in -> NaN out (the costs' non-finite guard sees it)
