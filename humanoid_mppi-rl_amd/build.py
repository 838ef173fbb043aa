"""Build libmppi_hip.so in-tree (hipcc, gfx950). Usage: python humanoid_mppi-rl_amd/build.py [--force]

Each source compiles to an object in parallel; the shared library links them. The .so lands in
humanoid_mppi-rl_amd/lib/ (git-ignored, but it travels to the GPU box with the repo snapshot).
"""
from __future__ import annotations

import concurrent.futures
import hashlib
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
# MPPI_AB_ARMS=1: also compile csrc/ab/ (kernels kept only as A/B arms: the layer-pipelined and the two-tiles-per-wave
# CA rollouts) into lib/libmppi_hip_ab.so (or the MPPI_VARIANT name); the shipped libmppi_hip.so never contains them
AB = os.environ.get("MPPI_AB_ARMS", "0") == "1"
if AB and not VARIANT:
    LIB = os.path.join(LIBDIR, "libmppi_hip_ab.so")
    OBJDIR = os.path.join(LIBDIR, "obj_ab")
ARCH = os.environ.get("MPPI_OFFLOAD_ARCH", "gfx950")
# per-source extra hipcc flags.  -fno-slp-vectorize: the SLP vectorizer packs adjacent f32 VALU ops into v_pk_*_f32,
# which measured slower in these latency- or VALU-bound kernels (CA rollout: 81.6 -> 77.8 us per config #4 launch;
# small-net FA: 760 -> 734 us per cartpole estimator solve; analytic cartpole: 18.3 -> 15.9 us per config #2 solve)
# but faster in others (the MLP rollout of config #3: 37.8 vs 39.7 us; the D = 512 FA kernel), which keep it
PER_FILE_FLAGS: dict[str, list[str]] = {
    "kernels_fc_ca.hip": ["-fno-slp-vectorize"],
    "kernels_fa_small.hip": ["-fno-slp-vectorize"],
    "kernels_fc_pipe.hip": ["-fno-slp-vectorize"],
    # iterative-ILP machine scheduler (round 4, late; same box, two or four pairs each): config #4 headline rollout
    # 346-349 -> 339-345 us, humanoid MLP 333-340 -> 327-332 us, the 32-solve shard 224-226 -> 217-226 us
    "kernels_fc_wave.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form", "-mllvm",
                            "-amdgpu-sched-strategy=iterative-ilp"],
    # two sample tiles per wave: MFMA accumulators in VGPRs (the default form put them in AGPRs and copied every
    # result back with v_accvgpr_read before its VALU use, 64 copies per wave-step)
    "kernels_fc_wide.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    # the split-bf16 per-wave kernel at one wave per SIMD: accumulators in AGPRs (the default form), which frees the
    # 256 ArchVGPRs for the hi / lo activations (config #4, 64 solves: 1298 -> 991 us per rollout, same box), and the
    # iterative-ILP machine scheduler (975 -> 887 us, same box; max-ilp / max-memory-clause 1094-1098 us)
    "kernels_fc_x3.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    # its two-waves-per-SIMD form (round 5): MFMA accumulators wherever the compiler fits them (256 registers per wave)
    "kernels_fc_x3p.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    # the split per-wave MLP kernel (round 5): the same flags as the CA's two-waves-per-SIMD split kernel
    "kernels_fc_x3m.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "kernels_fc_x3mp.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    # the split M-split CA kernel at two waves per SIMD (round 6): accumulators of the compiler's own MFMAs (layers 0
    # and 2) in VGPRs, no v_accvgpr copies (8 solves, same box: 150.5 -> 147.7 us per rollout)
    "kernels_fc_x3d.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    # its fp16 form at one group per block (round 6, late): the same flags
    "kernels_fc_x3h.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"],
    "kernels_common.hip": ["-fno-slp-vectorize"],
    # the analytic cartpole's 8-step chunks: the iterative-ILP machine scheduler interleaves the steps' independent
    # work into the dependent chain better (config #2 rollout 13.3 -> 12.9 us, same box, two pairs; max-ilp 13.4)
    "kernels_cartpole.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
}
# A/B only (variants): MPPI_X3_VGPR=1 builds kernels_fc_x3.hip with its MFMA accumulators in ArchVGPRs too;
# MPPI_AGPR_FORM=<file.hip> builds that file without -amdgpu-mfma-vgpr-form
if VARIANT and os.environ.get("MPPI_X3_VGPR", "0") == "1":
    PER_FILE_FLAGS["kernels_fc_x3.hip"] = ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]
if VARIANT and os.environ.get("MPPI_X3_FLAGS") is not None:  # the split-bf16 unit's flags replaced
    PER_FILE_FLAGS["kernels_fc_x3.hip"] = ["-fno-slp-vectorize"] + os.environ["MPPI_X3_FLAGS"].split()
if VARIANT and os.environ.get("MPPI_FILE_FLAGS"):  # "<file.hip>:<extra flags>" for one unit
    _f, _x = os.environ["MPPI_FILE_FLAGS"].split(":", 1)
    PER_FILE_FLAGS[_f] = PER_FILE_FLAGS.get(_f, []) + _x.split()
if VARIANT and os.environ.get("MPPI_FILE_FLAGS_SET"):  # "<file.hip>:<flags>": one unit's flags replaced
    _f, _x = os.environ["MPPI_FILE_FLAGS_SET"].split(":", 1)
    PER_FILE_FLAGS[_f] = _x.split()
if VARIANT and os.environ.get("MPPI_WAVE_FLAGS"):  # extra flags for kernels_fc_wave.hip only
    PER_FILE_FLAGS["kernels_fc_wave.hip"] = PER_FILE_FLAGS["kernels_fc_wave.hip"] + os.environ["MPPI_WAVE_FLAGS"].split()
if VARIANT and os.environ.get("MPPI_AGPR_FORM"):
    _f = os.environ["MPPI_AGPR_FORM"]
    PER_FILE_FLAGS[_f] = [x for x in PER_FILE_FLAGS.get(_f, []) if x not in ("-mllvm", "-amdgpu-mfma-vgpr-form")]
INCLUDE = os.path.join(os.path.dirname(HERE), "include")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build libmppi_hip.so)")


def sources() -> list[str]:
    src = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    if AB:
        ab = os.path.join(CSRC, "ab")
        src += sorted(os.path.join(ab, f) for f in os.listdir(ab) if f.endswith(".hip"))
    return src


def flag_config() -> str:
    """The effective compile configuration of this build: target, per-source flags (after every MPPI_* variant
    override), extra flags and the STAMPS / AB switches -- what changes the binary besides the sources."""
    per = ";".join(f"{k}={' '.join(v)}" for k, v in sorted(PER_FILE_FLAGS.items()))
    return f"arch={ARCH}|extra={' '.join(EXTRA_FLAGS)}|stamps={int(STAMPS)}|ab={int(AB)}|per={per}"


def source_hash() -> str:
    """SHA-256 over every file of csrc/ (recursive) and include/ (relative path + bytes), this script, and the effective
    compile configuration (flag_config: env-var variant flags included): the build id stamped into the library
    (mppi_build_id), which smoke() compares with the checkout's default build."""
    h = hashlib.sha256()
    h.update(flag_config().encode() + b"\0")
    root = os.path.dirname(HERE)
    files = []
    for top in (CSRC, INCLUDE):
        for d, _, fs in os.walk(top):
            files += [os.path.join(d, f) for f in fs if f.endswith((".hip", ".cpp", ".h"))]
    for f in sorted(files) + [os.path.abspath(__file__)]:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def _id_file() -> str:
    return LIB + ".id"


def up_to_date() -> bool:
    """The library exists and was built from exactly these sources (content hash, not file times: the GPU box
    receives a copy of the tree)."""
    if not (os.path.exists(LIB) and os.path.exists(_id_file())):
        return False
    with open(_id_file()) as f:
        return f.read().strip() == source_hash()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    hipcc = _hipcc()
    bid = source_hash()
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}", "-Wall",
             "-Wno-unused-function"]
    if STAMPS:
        flags.append("-DMPPI_STAMPS")
    if AB:
        flags.append("-DMPPI_AB_ARMS")
    flags += EXTRA_FLAGS

    def compile_one(src: str) -> str:
        obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
        extra = [f'-DMPPI_BUILD_ID="{bid}"'] if os.path.basename(src) == "mppi_api.hip" else []
        cmd = [hipcc, *flags, *extra, *PER_FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
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
    with open(_id_file(), "w") as f:
        f.write(bid + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
