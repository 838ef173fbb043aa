"""Thin object wrapper over one C-ABI handle (one device, one stream)."""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field, fields

import numpy as np

from . import _lib as L

_KINDS_COST = {"cartpole": L.COST_CARTPOLE, "cartpole_est": L.COST_CARTPOLE_EST, "humanoid_v3": L.COST_HUMANOID_V3,
               "humanoid_v1": L.COST_HUMANOID_V1, "quad_jl": L.COST_QUAD_JL, "quad_est": L.COST_QUAD_EST}


@dataclass
class Config:
    """mppi_config as a dataclass; see include/mppi.h for field meaning."""
    nx: int
    nu: int
    H: int
    K: int
    max_batch: int = 1
    lambda_: float = 1.0
    sigma: float = 1.0
    ctrl_clamp: float = 0.0
    U_clamp: float = 0.0
    norm_eps: float = 0.0
    shift_fill: float = 0.1
    terminal_weight: float = 10.0
    update_mode: int = L.UPDATE_ADD
    precision: int = L.PREC_BF16

    @classmethod
    def preset(cls, name: str, **overrides) -> "Config":
        c = L.preset_config(name)
        kw = {f.name: getattr(c, f.name) for f in fields(cls)}
        kw.update(overrides)
        return cls(**kw)

    def to_c(self) -> L.mppi_config:
        c = L.mppi_config()
        for f in fields(self):
            setattr(c, f.name, getattr(self, f.name))
        return c


def _f32(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if shape is not None and a.shape != tuple(shape):
        a = a.reshape(shape)
    return a


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class SolveResult:
    U: np.ndarray
    costs: np.ndarray | None = None
    weights: np.ndarray | None = None
    u0: np.ndarray | None = None
    status: int = 0


class Engine:
    def __init__(self, config: Config, device: int = 0):
        self.lib = L.load()
        self.config = config
        h = ctypes.c_void_p()
        L.check(self.lib.mppi_create(ctypes.byref(config.to_c()), device, ctypes.byref(h)))
        self._h = h
        self.device = device

    # -- lifecycle
    def close(self):
        if getattr(self, "_h", None):
            self.lib.mppi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- setup
    def load_dynamics(self, kind: int, blob: bytes | None = None):
        if blob is None:
            L.check(self.lib.mppi_load_dynamics(self._h, kind, None, 0))
        else:
            buf = ctypes.create_string_buffer(blob, len(blob))
            L.check(self.lib.mppi_load_dynamics(self._h, kind, buf, len(blob)))
        return self

    def set_cost(self, kind, params=None):
        kind = _KINDS_COST.get(kind, kind)
        if params is None:
            L.check(self.lib.mppi_set_cost(self._h, kind, None, 0))
        else:
            p = _f32(params).ravel()
            L.check(self.lib.mppi_set_cost(self._h, kind, p.ctypes.data_as(L._fp), int(p.size)))
        return self

    # -- host-memory solve
    def solve(self, x0, U, noise=None, seed: int = 0, ctx=None, shift: bool = False, u0_before: bool = False,
              want_costs: bool = True, want_weights: bool = False, colmajor: bool = False,
              raise_nonfinite: bool = False) -> SolveResult:
        """One batched solve. x0 [B,nx] (or [nx]); U [B,nu,H] (or [nu,H]); noise None (device Philox) or
        [B,nu,H,K] (or [nu,H,K]). Returns the updated (and optionally shifted) U plus diagnostics."""
        c = self.config
        single = np.ndim(x0) == 1
        x0 = _f32(x0).reshape(-1, c.nx)
        B = x0.shape[0]
        Uo = _f32(U).reshape(B, c.H, c.nu) if colmajor else _f32(U).reshape(B, c.nu, c.H)
        Uo = Uo.copy()
        nz = None
        if noise is not None:
            nz = _f32(noise).reshape(B, c.K, c.H, c.nu) if colmajor else _f32(noise).reshape(B, c.nu, c.H, c.K)
        cx = None if ctx is None else _f32(ctx).reshape(B, L.CTX_MAX)
        costs = np.empty((B, c.K), np.float32) if want_costs else None
        weights = np.empty((B, c.K), np.float32) if want_weights else None
        u0 = np.empty((B, c.nu), np.float32)
        io = L.mppi_io(_ptr(x0), _ptr(Uo), _ptr(nz), _ptr(costs), _ptr(weights), _ptr(u0), _ptr(cx))
        flags = (L.FLAG_SHIFT if shift else 0) | (L.FLAG_U0_BEFORE if u0_before else 0) | (
            L.FLAG_COLMAJOR if colmajor else 0)
        rc = self.lib.mppi_solve_ex(self._h, B, ctypes.byref(io), ctypes.c_uint64(seed), flags)
        if rc != L.MPPI_E_NONFINITE or raise_nonfinite:
            L.check(rc)
        sq = (lambda a: a[0]) if single else (lambda a: a)
        return SolveResult(U=sq(Uo), costs=None if costs is None else sq(costs),
                           weights=None if weights is None else sq(weights), u0=sq(u0), status=rc)

    # -- device-memory solve (pointers are integers, e.g. torch tensor .data_ptr())
    def solve_device(self, B: int, x0_ptr: int, U_ptr: int | None = None, noise_ptr: int | None = None, seed: int = 0,
                     costs_ptr: int | None = None, u0_ptr: int | None = None, ctx_ptr: int | None = None,
                     weights_ptr: int | None = None, shift: bool = False, resident_U: bool = False,
                     asynchronous: bool = True, env_step: bool = False, seed_counter: bool = False,
                     chain: bool = False) -> int:
        """env_step: advance x0 in place by one dynamics step with u0 (MPPI_FLAG_ENV_STEP);
        seed_counter: noise key = seed + the handle's device counter (MPPI_FLAG_SEED_COUNTER);
        chain: a chained solve (MPPI_FLAG_CHAIN: the previous chained solve's reduce generated this one's noise;
        2 launches, bitwise equal to plain counter solves)."""
        io = L.mppi_io(x0_ptr, U_ptr, noise_ptr, costs_ptr, weights_ptr, u0_ptr, ctx_ptr)
        flags = self._dev_flags(shift, resident_U, env_step) | (L.FLAG_ASYNC if asynchronous else 0) | (
            L.FLAG_SEED_COUNTER if seed_counter else 0) | (L.FLAG_CHAIN if chain else 0)
        return L.check(self.lib.mppi_solve_ex(self._h, B, ctypes.byref(io), ctypes.c_uint64(seed), flags))

    @staticmethod
    def _dev_flags(shift, resident_U, env_step):
        return L.FLAG_DEVICE | (L.FLAG_SHIFT if shift else 0) | (L.FLAG_RESIDENT_U if resident_U else 0) | (
            L.FLAG_ENV_STEP if env_step else 0)

    # -- receding-horizon stream as one hipGraph (mppi_graph_capture / mppi_graph_launch)
    def graph_capture(self, B: int, n_solves: int, x0_ptr: int, U_ptr: int | None = None, u0_ptr: int | None = None,
                      ctx_ptr: int | None = None, costs_ptr: int | None = None, seed: int = 0, shift: bool = True,
                      resident_U: bool = False, env_step: bool = True):
        return self.graph_capture_traj(B, n_solves, x0_ptr, U_ptr, u0_ptr, ctx_ptr, costs_ptr, seed, shift,
                                       resident_U, env_step)

    def graph_capture_traj(self, B: int, n_solves: int, x0_ptr: int, U_ptr: int | None = None,
                           u0_ptr: int | None = None, ctx_ptr: int | None = None, costs_ptr: int | None = None,
                           seed: int = 0, shift: bool = True, resident_U: bool = False, env_step: bool = True,
                           traj_x_ptr: int | None = None, traj_u_ptr: int | None = None):
        """Capture n_solves chained solves; with traj_*_ptr (device [n][B][nx] / [n][B][nu]) the env steps log
        the (state, control) trajectory."""
        io = L.mppi_io(x0_ptr, U_ptr, None, costs_ptr, None, u0_ptr, ctx_ptr)
        self._graph_io = io  # the graph holds these device pointers
        flags = self._dev_flags(shift, resident_U, env_step)
        L.check(self.lib.mppi_graph_capture_traj(self._h, B, ctypes.byref(io), ctypes.c_uint64(seed), flags,
                                                 n_solves, traj_x_ptr, traj_u_ptr))
        return self

    def graph_launch(self, sync: bool = False) -> int:
        return L.check(self.lib.mppi_graph_launch(self._h, int(sync)))

    def set_seed_counter(self, value: int = 0):
        L.check(self.lib.mppi_set_seed_counter(self._h, ctypes.c_uint64(value)))

    def get_seed_counter(self) -> int:
        """The device noise-key counter after every enqueued solve (waits for the stream): with get_U, the warm-start
        state of a receding-horizon stream (checkpoint / resume)."""
        v = ctypes.c_uint64(0)
        L.check(self.lib.mppi_get_seed_counter(self._h, ctypes.byref(v)))
        return int(v.value)

    def x3_layer1(self) -> tuple[int, float]:
        """(products, probe_rel_err) of the split CA's layer 1 (mppi_x3_layer1): 2 or 3 once the first solve's probe
        ran (0 otherwise or not a split CA), and the probe's max relative cost difference between the two forms (-1: no
        probe ran)."""
        n, e = ctypes.c_int(), ctypes.c_float()
        L.check(self.lib.mppi_x3_layer1(self._h, ctypes.byref(n), ctypes.byref(e)))
        return n.value, float(e.value)

    def x3_f16(self) -> tuple[int, float]:
        """(form, probe_rel_err) of the split CA's fp16 form (mppi_x3_f16): 2 = on with the one-product last layer, 1 =
        on with the two-product one, 0 = off for this handle's horizon; and the probe's max relative cost difference
        between the form in effect and three products (-1: no probe ran)."""
        n, e = ctypes.c_int(), ctypes.c_float()
        L.check(self.lib.mppi_x3_f16(self._h, ctypes.byref(n), ctypes.byref(e)))
        return int(n.value), float(e.value)

    def rollout_kernel(self) -> str:
        """The kernel the last solve's rollout was routed to (mppi_rollout_kernel)."""
        return (self.lib.mppi_rollout_kernel(self._h) or b"").decode()

    def set_stream(self, stream_handle: int | None):
        L.check(self.lib.mppi_set_stream(self._h, stream_handle))

    def sync(self):
        L.check(self.lib.mppi_sync(self._h))

    def get_U(self, B: int = 1) -> np.ndarray:
        out = np.empty((B, self.config.nu, self.config.H), np.float32)
        L.check(self.lib.mppi_get_U(self._h, B, _ptr(out)))
        return out

    def set_U(self, U, B: int | None = None):
        U = _f32(U).reshape(-1, self.config.nu, self.config.H)
        L.check(self.lib.mppi_set_U(self._h, U.shape[0] if B is None else B, _ptr(U)))

    def profile(self, enable: bool = True):
        L.check(self.lib.mppi_profile(self._h, int(enable)))

    def kernel_time(self, name: str) -> tuple[int, float]:
        n, ms = ctypes.c_int(), ctypes.c_double()
        L.check(self.lib.mppi_kernel_time(self._h, name.encode(), ctypes.byref(n), ctypes.byref(ms)))
        return n.value, ms.value

    def kernel_clock(self, enable: bool = True):
        """Reset and (re)start the rollout launch clock (mppi_kernel_clock): device wall-clock stamps of every
        rollout launch enqueued or captured from now on, read with kernel_clock_read()."""
        L.check(self.lib.mppi_kernel_clock(self._h, int(enable)))

    def kernel_clock_read(self) -> tuple[int, float, float]:
        """(launches, total_us, max_us) of the stamped rollout launches since the last reset."""
        n, tot, mx = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        L.check(self.lib.mppi_kernel_clock_read(self._h, ctypes.byref(n), ctypes.byref(tot), ctypes.byref(mx)))
        return n.value, tot.value, mx.value

    def device_buffers(self) -> dict:
        dU, du0, dc = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        L.check(self.lib.mppi_device_buffers(self._h, ctypes.byref(dU), ctypes.byref(du0), ctypes.byref(dc)))
        return dict(U=dU.value, u0=du0.value, costs=dc.value)
