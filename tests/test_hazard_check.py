"""The split-bf16 M-split kernels issue their MFMAs from inline asm (fc_common.h P<BF16X3>::mma_a / mma_a2: the
fragments read from AGPRs), which hipcc's hazard recognizer does not see into; mma_fence pads every accumulator read.
This CPU test compiles the CA unit to gfx950 assembly with the library's own flags (build.py) and checks, with
tools/mfma_hazard_check.py, that no instruction but a dependent MFMA touches an asm MFMA's destination within 12 wait
states (gfx950 needs 7 after a 4-pass XDL write) -- so a compiler or scheduling change that reintroduced a hazard fails
here instead of as intermittent wrong results on the GPU."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "humanoid_mppi-rl_amd")]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc needed")
@pytest.mark.parametrize("unit,min_kernels", [("kernels_fc_ca.hip", 4), ("kernels_fc_x3d.hip", 4),
                                                 ("kernels_fc_x3h.hip", 4)])
def test_asm_mfma_hazards_padded(tmp_path, unit, min_kernels):
    """kernels_fc_ca.hip: fc_rollout_kernel_x3 / _x3w (two costs x two layer-1 forms); kernels_fc_x3d.hip:
    fc_rollout_kernel_x3d (two costs x the two-product and the fp16 layer 1); kernels_fc_x3h.hip: fc_rollout_kernel_x3h
    (two costs x the two last-layer forms of the fp16 form)."""
    import build as B
    import mfma_hazard_check as H
    src = os.path.join(B.CSRC, unit)
    out = tmp_path / "k.s"
    cmd = [B._hipcc(), "-O3", "-std=c++17", f"--offload-arch={B.ARCH}", "--cuda-device-only", "-S",
           f"-I{B.INCLUDE}", f"-I{B.CSRC}", *B.PER_FILE_FLAGS.get(unit, []), src, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    res = H.check(out.read_text())
    assert len(res) >= min_kernels, [n for n, *_ in res]
    for name, n_mfma, bad in res:
        # x3d: layer 1 only (2 x 16 per wave-step, fp16 form 16; the step loop unrolled by 2 + a tail step); x3 / x3w:
        # every layer
        assert n_mfma >= 48, (name, n_mfma)
        assert bad == 0, f"{name}: {bad} accesses to an asm MFMA's destination within {H.WAIT_STATES} wait states"
