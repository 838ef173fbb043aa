"""Build libmppi_hip.so in-tree (hipcc, gfx950). Usage: python humanoid_mppi-rl_amd/build.py [--force]

Each source compiles to an object in parallel; the shared library links them. The .so lands in
humanoid_mppi-rl_amd/lib/ (git-ignored, but it travels to the GPU box with the repo snapshot).
"""
from __future__ import annotations

import concurrent.futures
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(HERE, "lib", "obj")
LIB = os.path.join(LIBDIR, "libmppi_hip.so")
# MPPI_STAMPS=1 builds the diagnostic variant (in-kernel s_memtime segment stamps) as libmppi_hip_stamps.so
STAMPS = os.environ.get("MPPI_STAMPS", "0") == "1"
if STAMPS:
    LIB = os.path.join(LIBDIR, "libmppi_hip_stamps.so")
    OBJDIR = os.path.join(LIBDIR, "obj_stamps")
# A/B variants: MPPI_VARIANT=<name> MPPI_EXTRA_FLAGS="-DX ..." builds lib/libmppi_hip_<name>.so (own object dir)
VARIANT = os.environ.get("MPPI_VARIANT", "")
EXTRA_FLAGS = os.environ.get("MPPI_EXTRA_FLAGS", "").split()
if VARIANT:
    LIB = os.path.join(LIBDIR, f"libmppi_hip_{VARIANT}.so")
    OBJDIR = os.path.join(LIBDIR, f"obj_{VARIANT}")
ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")
# per-source extra hipcc flags.  -fno-slp-vectorize: the SLP vectorizer packs adjacent f32 VALU ops into v_pk_*_f32,
# which measured slower in these latency- or VALU-bound kernels (CA rollout: 81.6 -> 77.8 us per config #4 launch;
# small-net FA: 760 -> 734 us per cartpole estimator solve; analytic cartpole: 18.3 -> 15.9 us per config #2 solve)
# but faster in others (the MLP rollout of config #3: 37.8 vs 39.7 us; the D = 512 FA kernel), which keep it
PER_FILE_FLAGS: dict[str, list[str]] = {
    "kernels_fc_ca.hip": ["-fno-slp-vectorize"],
    "kernels_fa_small.hip": ["-fno-slp-vectorize"],
    "kernels_fc_pipe.hip": ["-fno-slp-vectorize"],
    "kernels_fc_wave.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    # two sample tiles per wave: MFMA accumulators in VGPRs (the default form put them in AGPRs and copied every
    # result back with v_accvgpr_read before its VALU use, 64 copies per wave-step)
    "kernels_fc_wide.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    "kernels_common.hip": ["-fno-slp-vectorize"],
    # the analytic cartpole's 8-step chunks: the iterative-ILP machine scheduler interleaves the steps' independent
    # work into the dependent chain better (config #2 rollout 13.3 -> 12.9 us, same box, two pairs; max-ilp 13.4)
    "kernels_cartpole.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
}
INCLUDE = os.path.join(os.path.dirname(HERE), "include")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libmppi_hip.so)")


def sources() -> list[str]:
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _deps() -> list[str]:
    return sources() + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [
        os.path.join(INCLUDE, "mppi.h"), os.path.abspath(__file__)]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    hipcc = _hipcc()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", "-Wall", "-Wno-unused-function"]
    if STAMPS:
        flags.append("-DMPPI_STAMPS")
    flags += EXTRA_FLAGS

    def compile_one(src: str) -> str:
        obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
        cmd = [hipcc, *flags, *PER_FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
        if src.endswith(".cpp"):
            cmd = [hipcc, *flags, "-x", "hip", "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr, file=sys.stderr)
        return obj

    jobs = min(8, len(sources()))
    with concurrent.futures.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = LIB + ".tmp"
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs], capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
