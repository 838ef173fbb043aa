"""ctypes binding of libmppi_hip.so (include/mppi.h). No fallback: if the HIP library is missing the
import of any solve path raises MPPILibraryError."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("MPPI_HIP_LIB", os.path.join(PKG_ROOT, "lib", "libmppi_hip.so"))

# ---- constants (mirror include/mppi.h)
MPPI_OK = 0
MPPI_E_ARG, MPPI_E_HIP, MPPI_E_UNSUPPORTED, MPPI_E_NONFINITE, MPPI_E_STATE = -1, -2, -3, -4, -5
DYN_CARTPOLE, DYN_MLP, DYN_CROSS_ATTN, DYN_FEATURE_ATTN = 1, 2, 3, 4
COST_CARTPOLE, COST_CARTPOLE_EST, COST_HUMANOID_V3, COST_QUAD_JL, COST_QUAD_EST, COST_HUMANOID_V1 = 1, 2, 3, 4, 5, 6
UPDATE_ADD, UPDATE_REPLACE = 0, 1
PREC_FP32, PREC_BF16, PREC_BF16X3 = 0, 1, 2  # BF16X3: fp32-accurate split bf16 (fc nets)
FLAG_SHIFT, FLAG_COLMAJOR, FLAG_DEVICE, FLAG_ASYNC, FLAG_U0_BEFORE, FLAG_RESIDENT_U = 0x1, 0x2, 0x4, 0x8, 0x10, 0x20
FLAG_ENV_STEP, FLAG_SEED_COUNTER, FLAG_CHAIN = 0x40, 0x80, 0x100
CTX_MAX = 8

EXPORTED = ["mppi_preset", "mppi_create", "mppi_destroy", "mppi_load_dynamics", "mppi_set_cost", "mppi_solve",
            "mppi_solve_ex", "mppi_get_U", "mppi_set_U", "mppi_set_stream", "mppi_sync", "mppi_profile",
            "mppi_kernel_time", "mppi_device_buffers", "mppi_last_error", "mppi_abi_version", "mppi_graph_capture",
            "mppi_graph_launch", "mppi_set_seed_counter", "mppi_get_seed_counter", "mppi_graph_capture_traj",
            "mppi_kernel_clock",
            "mppi_kernel_clock_read", "mppi_build_id", "mppi_x3_layer1", "mppi_rollout_kernel", "mppi_x3_f16"]


class MPPIError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[mppi error {code}] {msg}")
        self.code = code


class MPPILibraryError(ImportError):
    pass


class mppi_config(ctypes.Structure):
    _fields_ = [("nx", ctypes.c_int32), ("nu", ctypes.c_int32), ("H", ctypes.c_int32), ("K", ctypes.c_int32),
                ("max_batch", ctypes.c_int32), ("lambda_", ctypes.c_float), ("sigma", ctypes.c_float),
                ("ctrl_clamp", ctypes.c_float), ("U_clamp", ctypes.c_float), ("norm_eps", ctypes.c_float),
                ("shift_fill", ctypes.c_float), ("terminal_weight", ctypes.c_float), ("update_mode", ctypes.c_int32),
                ("precision", ctypes.c_int32), ("reserved", ctypes.c_int32 * 4)]


_fp = ctypes.POINTER(ctypes.c_float)


class mppi_io(ctypes.Structure):
    _fields_ = [("x0", ctypes.c_void_p), ("U", ctypes.c_void_p), ("noise", ctypes.c_void_p), ("costs", ctypes.c_void_p),
                ("weights", ctypes.c_void_p), ("u0", ctypes.c_void_p), ("ctx", ctypes.c_void_p)]


_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libmppi_hip.so (once). Raises MPPILibraryError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise MPPILibraryError(f"libmppi_hip.so not found at {p}: run `python humanoid_mppi-rl_amd/build.py` "
                               "(the MPPI engine has no CPU fallback)")
    lib = ctypes.CDLL(p)
    vp, i32, u64, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "mppi_preset": (i32, [ctypes.c_char_p, ctypes.POINTER(mppi_config)]),
        "mppi_create": (i32, [ctypes.POINTER(mppi_config), i32, ctypes.POINTER(vp)]),
        "mppi_destroy": (None, [vp]),
        "mppi_load_dynamics": (i32, [vp, i32, vp, sz]),
        "mppi_set_cost": (i32, [vp, i32, _fp, i32]),
        "mppi_solve": (i32, [vp, i32, vp, vp, vp, u64, vp, vp, i32]),
        "mppi_solve_ex": (i32, [vp, i32, ctypes.POINTER(mppi_io), u64, i32]),
        "mppi_get_U": (i32, [vp, i32, vp]),
        "mppi_set_U": (i32, [vp, i32, vp]),
        "mppi_set_stream": (i32, [vp, vp]),
        "mppi_sync": (i32, [vp]),
        "mppi_profile": (i32, [vp, i32]),
        "mppi_kernel_time": (i32, [vp, ctypes.c_char_p, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double)]),
        "mppi_device_buffers": (i32, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp)]),
        "mppi_last_error": (ctypes.c_char_p, []),
        "mppi_abi_version": (i32, []),
        "mppi_build_id": (ctypes.c_char_p, []),
        "mppi_graph_capture": (i32, [vp, i32, ctypes.POINTER(mppi_io), u64, i32, i32]),
        "mppi_graph_launch": (i32, [vp, i32]),
        "mppi_graph_capture_traj": (i32, [vp, i32, ctypes.POINTER(mppi_io), u64, i32, i32, vp, vp]),
        "mppi_set_seed_counter": (i32, [vp, u64]),
        "mppi_get_seed_counter": (i32, [vp, ctypes.POINTER(u64)]),
        "mppi_kernel_clock": (i32, [vp, i32]),
        "mppi_x3_layer1": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_float)]),
        "mppi_rollout_kernel": (ctypes.c_char_p, [vp]),
        "mppi_x3_f16": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_float)]),
        "mppi_kernel_clock_read": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_double)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def build_id() -> str:
    """The source hash the loaded library was built from (build.py source_hash)."""
    return load().mppi_build_id().decode()


def check(code: int) -> int:
    if code != MPPI_OK:
        msg = load().mppi_last_error()
        raise MPPIError(code, msg.decode() if msg else "")
    return code


def preset_config(name: str) -> mppi_config:
    cfg = mppi_config()
    check(load().mppi_preset(name.encode(), ctypes.byref(cfg)))
    return cfg
