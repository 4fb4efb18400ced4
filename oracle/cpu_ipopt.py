"""CPU RESTATEMENT -- TEST INFRASTRUCTURE AND CPU BASELINE ONLY. NOT THE PRODUCT.

ctypes binding of ``oracle/libnmpc_cpu.so`` (``oracle/cpu_ipopt.cpp``, built by
``oracle/Makefile`` / ``__graft_entry__.build()``): the compiled C++/OpenMP
restatement of the same IPOPT algorithm as ``oracle/nmpc_oracle.py`` with a
Riccati Newton step (BASELINE.md plan 2: "CPU
restatement, not CasADi").  Only ``tests/`` and ``bench.py``'s ``cpu_baseline``
leg use it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import nmpc_oracle as orc

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnmpc_cpu.so")
MAXOBS = 16


class CpuProblem(C.Structure):
    _fields_ = [("N", C.c_int32), ("model", C.c_int32), ("n_obs", C.c_int32), ("np", C.c_int32),
                ("w1_pidx", C.c_int32), ("w2_pidx", C.c_int32),
                ("T", C.c_double), ("w1", C.c_double), ("w2", C.c_double), ("vfov", C.c_double),
                ("hfov", C.c_double), ("obs_x", C.c_double * MAXOBS), ("obs_y", C.c_double * MAXOBS),
                ("obs_rsum", C.c_double * MAXOBS), ("obs_x_pidx", C.c_int32 * MAXOBS),
                ("obs_y_pidx", C.c_int32 * MAXOBS)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):  # the checker is built on demand (not part of the product build)
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.dirname(LIB_PATH)], check=False)
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle` or python __graft_entry__.py")
        L = C.CDLL(LIB_PATH)
        L.nmpc_cpu_option_names.restype = C.c_char_p
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        L.nmpc_cpu_solve_batch.argtypes = [C.POINTER(CpuProblem), dp, C.c_int64, dp, dp, dp, dp, dp, dp,
                                           dp, dp, dp, dp, dp, ip, ip, C.c_int, dp]
        L.nmpc_cpu_closed_loop.argtypes = [C.POINTER(CpuProblem), dp, C.c_int64, C.c_int32, dp, dp, dp, dp, dp, dp,
                                           C.c_double, C.c_double, dp, C.c_double, C.c_int, ip, ip, dp, dp, ip, dp,
                                           dp, dp]
        _lib = L
    return _lib


def problem_struct(prob: orc.Problem) -> CpuProblem:
    if prob.n_obs > MAXOBS:
        raise ValueError(f"at most {MAXOBS} obstacles")
    c = CpuProblem()
    c.N, c.model, c.n_obs, c.np = prob.N, 1 if prob.model == "uav5" else 0, prob.n_obs, prob.np_
    c.w1_pidx, c.w2_pidx = prob.w1_pidx, prob.w2_pidx
    c.T, c.w1, c.w2, c.vfov, c.hfov = prob.T, prob.w1, prob.w2, prob.vfov, prob.hfov
    for j in range(prob.n_obs):
        c.obs_x[j], c.obs_y[j], c.obs_rsum[j] = prob.obs_x[j], prob.obs_y[j], prob.obs_rsum[j]
        c.obs_x_pidx[j], c.obs_y_pidx[j] = int(prob.obs_x_pidx[j]), int(prob.obs_y_pidx[j])
    return c


def options_array(opts=None) -> np.ndarray:
    """IPOPT_DEFAULTS overridden by opts, in the library's option order."""
    o = dict(orc.IPOPT_DEFAULTS)
    for k, v in (opts or {}).items():
        if k not in o:
            raise KeyError(f"unknown IPOPT option {k}")
        o[k] = v
    names = lib().nmpc_cpu_option_names().decode().split(",")
    missing = set(o) - set(names)
    if missing:
        raise KeyError(f"options not restated by the C++ solver: {sorted(missing)}")
    return np.array([float(o[k]) for k in names], dtype=np.float64)


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _f64(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a if shape is None else a.reshape(shape)


def solve_batch(prob, W0, P, lbx, ubx, lbg, ubg, opts=None, threads=0):
    """B independent solves; W0 (B, nw), P (B, np).  Returns a dict like the oracle's
    result (x, f, g, lam_x, lam_g, status, iter), batched, plus each solve's wall time
    (solve_s, seconds)."""
    W0 = _f64(W0)
    P = _f64(P)
    B = W0.shape[0]
    nw, m = prob.nw, prob.ng
    out = {"x": np.empty((B, nw)), "f": np.empty(B), "g": np.empty((B, m)), "lam_x": np.empty((B, nw)),
           "lam_g": np.empty((B, m)), "status": np.empty(B, np.int32), "iter": np.empty(B, np.int32),
           "solve_s": np.zeros(B)}
    cp = problem_struct(prob)
    oa = options_array(opts)
    bl = [_f64(b) for b in (lbx, ubx, lbg, ubg)]
    rc = lib().nmpc_cpu_solve_batch(C.byref(cp), _p(oa), B, _p(W0), _p(P), *[_p(b) for b in bl], _p(out["x"]),
                                    _p(out["f"]), _p(out["g"]), _p(out["lam_x"]), _p(out["lam_g"]),
                                    _i(out["status"]), _i(out["iter"]), int(threads), _p(out["solve_s"]))
    if rc != 0:
        raise RuntimeError(f"nmpc_cpu_solve_batch failed ({rc})")
    return out


def closed_loop(prob, P0, K, lbx, ubx, lbg, ubg, opts=None, vt=12.0, wt=0.01, p_step=None, budget_s=0.0,
                threads=0, W0=None):
    """K warm-started MPC steps per scenario (solve + shift_timestep; obstacle
    parameters advanced by p_step[k] (K, np) after step k), from p0 rows and the warm
    starts W0 (B, nw; None: w = 0).  Stops starting new steps after budget_s seconds (0:
    no limit).  Returns status / iter (B, K), u0 (B, K, nu), f (B, K), steps (B,),
    solve_s (B, K): each solve's wall time in seconds, and p / w (B, np) / (B, nw): the
    state after each scenario's last step, from which the loop continues."""
    P0 = _f64(P0)
    ps = None if p_step is None else _f64(p_step, (K, prob.np_))
    B = P0.shape[0]
    w0 = None if W0 is None else _f64(W0, (B, prob.nw))
    out = {"status": np.full((B, K), -1000, np.int32), "iter": np.zeros((B, K), np.int32),
           "u0": np.full((B, K, prob.nu), np.nan), "f": np.full((B, K), np.nan), "steps": np.zeros(B, np.int32),
           "solve_s": np.full((B, K), np.nan), "p": np.empty((B, prob.np_)), "w": np.empty((B, prob.nw))}
    cp = problem_struct(prob)
    oa = options_array(opts)
    bl = [_f64(b) for b in (lbx, ubx, lbg, ubg)]
    rc = lib().nmpc_cpu_closed_loop(C.byref(cp), _p(oa), B, int(K), _p(P0), None if w0 is None else _p(w0),
                                    *[_p(b) for b in bl], float(vt), float(wt), None if ps is None else _p(ps),
                                    float(budget_s), int(threads), _i(out["status"]), _i(out["iter"]),
                                    _p(out["u0"]), _p(out["f"]), _i(out["steps"]), _p(out["solve_s"]),
                                    _p(out["p"]), _p(out["w"]))
    if rc != 0:
        raise RuntimeError(f"nmpc_cpu_closed_loop failed ({rc})")
    return out
