"""ctypes binding + build recipe of oracle/mppi_cpu.c — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The compiled multi-core CPU restatement of the MPPI solve (see mppi_cpu.c's header). Imported only by tests/,
bench.py's cpu_baseline leg and __graft_entry__.build() (which compiles it); never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "mppi_cpu.c")
LIB = os.path.join(HERE, "lib", "libmppi_cpu.so")
MAXL = 8
COSTS = {"cartpole": 1, "cartpole_est": 2, "humanoid_v3": 3, "quad_jl": 4, "quad_est": 5}


def build(force: bool = False) -> str:
    """gcc -O3 -fopenmp; x86-64-v3 (AVX2 + FMA) so the .so built here runs on the GPU box's host CPU too."""
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = ["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-Wall", "-o", tmp, SRC, "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gcc failed for {SRC}:\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


class _Net(ctypes.Structure):
    _fields_ = [("nl", ctypes.c_int), ("dims", ctypes.c_int * (MAXL + 1)),
                ("W", ctypes.c_void_p * MAXL), ("b", ctypes.c_void_p * MAXL),
                ("lng", ctypes.c_void_p * MAXL), ("lnb", ctypes.c_void_p * MAXL), ("relu", ctypes.c_int * MAXL)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        _lib.mppi_cpu_fc_solve.argtypes = [ctypes.POINTER(_Net), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int, P, P,
                                           ctypes.c_int]
        _lib.mppi_cpu_cartpole_solve.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, ctypes.c_double,
                                                 ctypes.c_double, ctypes.c_int, P, P, ctypes.c_int]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class FcNet:
    """An fc stack (oracle/nets_ref.py format: dicts W, b, ln, relu) held as fp32 arrays for the C solver."""

    def __init__(self, stack: list):
        if len(stack) > MAXL:
            raise ValueError("too many layers")
        self._keep = []
        n = _Net()
        n.nl = len(stack)
        n.dims[0] = np.asarray(stack[0]["W"]).shape[1]
        for l, L in enumerate(stack):
            if L.get("lnfold") is not None:
                raise ValueError("pass the unfolded stack (LayerNorm as ln=(gamma, beta))")
            W = np.ascontiguousarray(L["W"], np.float32)
            b = np.ascontiguousarray(L["b"], np.float32)
            n.dims[l + 1] = W.shape[0]
            n.W[l], n.b[l] = W.ctypes.data, b.ctypes.data
            self._keep += [W, b]
            if L.get("ln") is not None:
                g, be = (np.ascontiguousarray(a, np.float32) for a in L["ln"])
                n.lng[l], n.lnb[l] = g.ctypes.data, be.ctypes.data
                self._keep += [g, be]
            n.relu[l] = 1 if L["relu"] else 0
        self.net = n


def fc_solve(net: FcNet, nx: int, nu: int, cost: str, x0, U, noise, lam: float, ctrl_clamp: float = 0.0,
             U_clamp: float = 0.0, norm_eps: float = 0.0, terminal_weight: float = 10.0, replace: bool = False,
             ctx=None, threads: int = 1) -> dict:
    """One learned-dynamics solve; U [nu][H] (not modified), noise [nu][H][K]. Returns costs, weights, U_new."""
    lib = _load()
    noise = np.ascontiguousarray(noise, np.float32)
    _, H, K = noise.shape
    Un = np.ascontiguousarray(U, np.float32).copy()
    costs = np.empty(K, np.float32)
    w = np.empty(K, np.float32)
    x0 = np.ascontiguousarray(x0, np.float32)
    cx = np.ascontiguousarray(np.zeros(8) if ctx is None else ctx, np.float32)
    rc = lib.mppi_cpu_fc_solve(ctypes.byref(net.net), nx, nu, K, H, COSTS[cost], _p(cx), _p(x0), _p(Un), _p(noise),
                               lam, ctrl_clamp, U_clamp, norm_eps, terminal_weight, 1 if replace else 0, _p(costs),
                               _p(w), threads)
    if rc != 0:
        raise RuntimeError(f"mppi_cpu_fc_solve returned {rc}")
    return dict(costs=costs, weights=w, U_new=Un)


def cartpole_solve(x0, U, noise, lam: float = 1.0, terminal_weight: float = 10.0, replace: bool = False,
                   threads: int = 1) -> dict:
    """One analytic-cartpole solve (fp64); U [1][H] (not modified), noise [1][H][K]."""
    lib = _load()
    noise = np.ascontiguousarray(noise, np.float64)
    _, H, K = noise.shape
    Un = np.ascontiguousarray(U, np.float64).reshape(-1).copy()
    costs = np.empty(K)
    w = np.empty(K)
    x0 = np.ascontiguousarray(x0, np.float64)
    rc = lib.mppi_cpu_cartpole_solve(K, H, _p(x0), _p(Un), _p(noise), lam, terminal_weight, 1 if replace else 0,
                                     _p(costs), _p(w), threads)
    if rc != 0:
        raise RuntimeError(f"mppi_cpu_cartpole_solve returned {rc}")
    return dict(costs=costs, weights=w, U_new=Un.reshape(1, H))


def _median_solve_s(fn, n: int, warm: int, budget_s: float) -> tuple[float, int]:
    """Median wall time of up to n calls after `warm` warm-ups (median of 20 after 3), within budget_s."""
    import time

    for _ in range(warm):
        fn()
    ts = []
    t_end = time.perf_counter() + budget_s
    while len(ts) < n and (not ts or time.perf_counter() < t_end):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), len(ts)


def time_fc_baseline(stack: list, nx: int, nu: int, cost: str, x0, K: int, H: int, sigma: float, lam: float,
                     ctx=None, threads: int = 1, n: int = 20, warm: int = 3, budget_s: float = 20.0, **kw) -> dict:
    """CPU baseline: full learned-dynamics solves of this shape on `threads` cores (the noise draw excluded, as on
    the GPU side, where it is one fused kernel; the reference draws it with randn on one core)."""
    net = FcNet(stack)
    noise = (sigma * np.random.RandomState(0).randn(nu, H, K)).astype(np.float32)
    U = np.zeros((nu, H), np.float32)
    s, cnt = _median_solve_s(lambda: fc_solve(net, nx, nu, cost, x0, U, noise, lam=lam, ctx=ctx, threads=threads,
                                              **kw), n, warm, budget_s)
    return dict(value=K * H / s, ms_per_solve=s * 1e3, solves=cnt)


def time_cartpole_baseline(x0, K: int, H: int, threads: int = 1, n: int = 20, warm: int = 3,
                           budget_s: float = 20.0) -> dict:
    noise = np.random.RandomState(0).randn(1, H, K)
    U = np.zeros((1, H))
    s, cnt = _median_solve_s(lambda: cartpole_solve(x0, U, noise, threads=threads), n, warm, budget_s)
    return dict(value=K * H / s, ms_per_solve=s * 1e3, solves=cnt)
