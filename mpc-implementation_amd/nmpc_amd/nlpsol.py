"""``nlpsol``-compatible front end over the C-ABI.

Mirrors the reference's operator interface for the hot path:

    solver = ca.nlpsol('solver', 'ipopt', nlp_prob, opts)       Python/NMPC_TT.py:267
    sol = solver(x0=..., lbx=..., ubx=..., lbg=..., ubg=..., p=...)   :358-365
    u = ca.reshape(sol['x'], n_controls, N)                     :367

``nlpsol(name, 'ipopt', spec, opts)`` takes a :class:`ProblemSpec` instead of a
symbolic dict (there is no CasADi here) and the same ``opts`` dict
(``{'ipopt': {...}, 'print_time': 0}``).  The returned :class:`Solver` is
called with the same keyword arguments.  Each argument may be one column
((n,), (n,1)) or a batch of columns ((n,B), CasADi's ``Function.map``
horzcat convention); bounds given as one column are shared by the batch.
Results come back as numpy arrays shaped (n,1) for one scenario or (n,B),
so ``np.reshape(sol['x'], (6, N), order='F')`` is ``ca.reshape``.

Errors follow CasADi: a dimension mismatch raises; non-convergence does not
(it is reported by ``solver.stats()``, which the reference never reads --
SURVEY F8).  All arithmetic runs in the HIP library; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Any

import numpy as np

from . import _lib
from .spec import ProblemSpec

RETURN_STATUS = {
    0: "Solve_Succeeded", 1: "Solved_To_Acceptable_Level", 2: "Infeasible_Problem_Detected",
    3: "Search_Direction_Becomes_Too_Small", 4: "Diverging_Iterates",
    -1: "Maximum_Iterations_Exceeded", -2: "Restoration_Failed", -3: "Error_In_Step_Computation",
    -11: "Invalid_Problem_Definition", -13: "Invalid_Number_Detected",
    -102: "Insufficient_Memory",  # NMPC_STATUS_EQ_UNRESERVED: equality rows, no reserve_equality(B)
}
_SUCCESS = (0, 1)
NOT_RUN = -1000  # NMPC_STATUS_NOT_RUN: a closed-loop step the scheduler never ran
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int32)


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(_DP)


def make_options(opts: dict | None) -> _lib.Options:
    """IPOPT option dict (CasADi ``opts['ipopt']``) -> C options struct."""
    o = _lib.default_options()
    if not opts:
        return o
    ip = dict(opts.get("ipopt", {}))
    if "linear_solver_fp32" in ip or "reserved0" in ip:
        raise ValueError("use the nlpsol option linear_solver_precision='single' (not an IPOPT option)")
    for k, v in ip.items():
        name = _lib.IPOPT_ALIASES.get(k, k)
        if name == "warm_start_init_point":
            if v != "no":
                raise ValueError("only warm_start_init_point='no' (IPOPT default: lam_x0/lam_g0 unused) "
                                 "is supported")
            continue
        if name in ("print_level", "print_timing_statistics", "sb", "linear_solver", "hessian_approximation",
                    "mu_strategy", "nlp_scaling_method", "fixed_variable_treatment"):
            if name == "hessian_approximation" and v != "exact":
                raise ValueError("only hessian_approximation='exact' is supported")
            if name == "mu_strategy" and v != "monotone":
                raise ValueError("only mu_strategy='monotone' (IPOPT default) is supported")
            if name == "nlp_scaling_method" and v != "gradient-based":
                raise ValueError("only nlp_scaling_method='gradient-based' (IPOPT default) is supported")
            if name == "fixed_variable_treatment" and v != "make_parameter":
                raise ValueError("only fixed_variable_treatment='make_parameter' (IPOPT default) is supported")
            continue  # output / linear-solver choices do not change the iterates here
        if not hasattr(o, name):
            raise ValueError(f"unsupported IPOPT option {k!r}")
        setattr(o, name, type(getattr(o, name))(v))
    for k in opts:
        if k not in ("ipopt", "print_time", "verbose", "expand", "error_on_fail", "linear_solver_precision"):
            raise ValueError(f"unsupported nlpsol option {k!r}")
    prec = opts.get("linear_solver_precision", "double")
    if prec not in ("double", "single"):
        raise ValueError("linear_solver_precision must be 'double' or 'single'")
    o.linear_solver_fp32 = 1 if prec == "single" else 0
    return o


class Solver:
    """Callable returned by :func:`nlpsol`; one handle (and GPU) per instance."""

    def __init__(self, name: str, spec: ProblemSpec, opts: dict | None = None):
        spec.validate()
        self.name = name
        self.spec = spec
        self.error_on_fail = bool((opts or {}).get("error_on_fail", False))
        L = _lib.lib()
        d = _lib.Desc()
        d.model = 1 if spec.model == "uav5" else 0
        d.N, d.np, d.n_obs = spec.N, spec.np, spec.n_obs
        d.T, d.w1, d.w2, d.vfov, d.hfov = spec.T, spec.w1, spec.w2, spec.vfov, spec.hfov
        for j, ob in enumerate(spec.obstacles):
            d.obs_x[j], d.obs_y[j], d.obs_rsum[j] = ob.x, ob.y, ob.r
            d.obs_x_pidx[j], d.obs_y_pidx[j] = ob.x_pidx, ob.y_pidx
        d.opts = make_options(opts)
        d.w1_pidx, d.w2_pidx = spec.w1_pidx, spec.w2_pidx
        self.max_iter = int(d.opts.max_iter)
        h = C.c_void_p()
        _lib.check(L.nmpc_create(C.byref(d), C.byref(h)))
        self._h = h
        self._stats: dict[str, Any] = {}
        self.nw, self.ng, self.np, self.nX = spec.nw, spec.ng, spec.np, spec.nX

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib().nmpc_destroy(h)
            except Exception:
                pass
            self._h = None

    # ---- argument normalisation (CasADi DM column / matrix semantics)
    def _arg(self, v, n: int, default: float, name: str):
        if v is None:
            return np.full((1, n), default), 0
        a = np.asarray(v, dtype=np.float64)
        if a.ndim == 0:
            a = np.full((n,), float(a))
        if a.ndim == 1:
            if a.shape[0] != n:
                raise ValueError(f"{name}: expected length {n}, got {a.shape[0]}")
            return np.ascontiguousarray(a.reshape(1, n)), 0
        if a.ndim == 2:
            if a.shape[0] != n:
                raise ValueError(f"{name}: expected {n} rows, got shape {a.shape}")
            cols = np.ascontiguousarray(a.T)  # (B, n): each scenario contiguous
            if cols.shape[0] == 1:
                return cols, 0
            return cols, n
        raise ValueError(f"{name}: expected a vector or an (n,B) matrix")

    def __call__(self, x0=None, lbx=None, ubx=None, lbg=None, ubg=None, p=None, lam_x0=None, lam_g0=None):
        # lam_x0 / lam_g0 are accepted and, exactly as IPOPT does under its default
        # warm_start_init_point='no' (the reference sets no warm-start option,
        # Python/NMPC_TT.py:257-265), not used: the multipliers are initialised by
        # IPOPT's own rules (bound_mult_init_val, least-squares y).  Their shapes are
        # still checked as CasADi checks them.
        for name, v, n in (("lam_x0", lam_x0, self.nw), ("lam_g0", lam_g0, self.ng)):
            if v is not None:
                self._arg(v, n, 0.0, name)
        args = {}
        B = 1
        for name, v, n, dflt in (("x0", x0, self.nw, 0.0), ("lbx", lbx, self.nw, -np.inf),
                                 ("ubx", ubx, self.nw, np.inf), ("lbg", lbg, self.ng, -np.inf),
                                 ("ubg", ubg, self.ng, np.inf), ("p", p, self.np, 0.0)):
            a, ld = self._arg(v, n, dflt, name)
            if ld:
                if B not in (1, a.shape[0]):
                    raise ValueError(f"{name}: batch size {a.shape[0]} does not match {B}")
                B = a.shape[0]
            args[name] = (a, ld)
        out = self.solve_batch(B, **{k: v for k, v in args.items()})
        single = B == 1
        res = {}
        for k in ("x", "g", "lam_x", "lam_g", "lam_p", "X"):
            arr = out[k].T  # (n, B)
            res[k] = arr if not single else arr.reshape(-1, 1)
        res["f"] = out["f"].reshape(1, B) if not single else out["f"].reshape(1, 1)
        st = out["status"]
        self._stats = {
            "return_status": RETURN_STATUS.get(int(st[0]), str(int(st[0]))) if single
            else [RETURN_STATUS.get(int(s), str(int(s))) for s in st],
            "success": bool(st[0] in _SUCCESS) if single else [bool(s in _SUCCESS) for s in st],
            "iter_count": int(out["iters"][0]) if single else out["iters"].copy(),
            "status_code": st.copy(),
        }
        if self.error_on_fail and not np.all(np.isin(st, _SUCCESS)):
            raise RuntimeError(f"nlpsol '{self.name}' failed: {self._stats['return_status']}")
        return res

    def solve_batch(self, B: int, x0, lbx, ubx, lbg, ubg, p):
        """Arrays as (B or 1, n) C-contiguous + leading dim (0 = broadcast)."""
        L = _lib.lib()
        out = {
            "x": np.empty((B, self.nw)), "g": np.empty((B, self.ng)), "lam_x": np.empty((B, self.nw)),
            "lam_g": np.empty((B, self.ng)), "lam_p": np.empty((B, self.np)), "X": np.empty((B, self.nX)),
            "f": np.empty(B),
            "status": np.empty(B, dtype=np.int32), "iters": np.empty(B, dtype=np.int32),
        }
        ins = []
        for a, ld in (x0, lbx, ubx, lbg, ubg, p):
            ins += [_dptr(a), ld]
        _lib.check(L.nmpc_solve_batch(
            self._h, B, *ins, _dptr(out["x"]), _dptr(out["f"]), _dptr(out["g"]), _dptr(out["lam_x"]),
            _dptr(out["lam_g"]), _dptr(out["lam_p"]), _dptr(out["X"]), out["status"].ctypes.data_as(_IP),
            out["iters"].ctypes.data_as(_IP)))
        return out

    def solve_device(self, x0, lbx, ubx, lbg, ubg, p, out: dict, stream=None):
        """Device path: torch CUDA float64 tensors, scenario-major (B, n) or shared (n,).

        ``out`` holds preallocated device tensors x (B,nw) [required], f (B,),
        g (B,ng), lam_x (B,nw), lam_g (B,ng), lam_p (B,np), X (B,nX), status/iters (B,) int32
        (optional).  Enqueued on ``stream`` (torch stream; default = current); never
        synchronises the host.  Batches with equality rows (lbg == ubg) need
        ``reserve_equality(B)`` first, otherwise every scenario reports status -102
        (Insufficient_Memory) with NaN x and f.
        """
        import torch  # plumbing only: device memory and streams

        L = _lib.lib()
        B = out["x"].shape[0]

        def dv(t, n):
            assert t.dtype == torch.float64 and t.is_cuda and t.is_contiguous()
            if t.dim() == 1:
                assert t.shape[0] == n
                return C.c_void_p(t.data_ptr()), 0
            assert t.shape == (B, n), (tuple(t.shape), (B, n))
            return C.c_void_p(t.data_ptr()), n

        ins = []
        for t, n in ((x0, self.nw), (lbx, self.nw), (ubx, self.nw), (lbg, self.ng), (ubg, self.ng), (p, self.np)):
            ins += list(dv(t, n))

        def op(k):
            t = out.get(k)
            return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)

        if stream is None:
            stream = torch.cuda.current_stream()
        _lib.check(L.nmpc_solve_batch_dev(self._h, B, *ins, op("x"), op("f"), op("g"), op("lam_x"),
                                          op("lam_g"), op("lam_p"), op("X"), op("status"), op("iters"),
                                          C.c_void_p(stream.cuda_stream)))

    def shift_device(self, p, u_sol, w_out, v_t, w_t, stream=None):
        """Closed-loop shift on device (Python/NMPC_TT.py:13-30), see nmpc_shift_dev."""
        import torch

        L = _lib.lib()
        B = u_sol.shape[0]
        if stream is None:
            stream = torch.cuda.current_stream()
        _lib.check(L.nmpc_shift_dev(self._h, B, C.c_void_p(p.data_ptr()), p.shape[1],
                                    C.c_void_p(u_sol.data_ptr()), C.c_void_p(w_out.data_ptr()),
                                    C.c_void_p(v_t.data_ptr()), C.c_void_p(w_t.data_ptr()),
                                    C.c_void_p(stream.cuda_stream)))

    def closed_loop_device(self, K: int, lbx, ubx, lbg, ubg, p, w, v_t, w_t, hist: dict | None = None,
                           stream=None, p_step=None, order=None, check: bool = True, _validate_order: bool = True):
        """K closed-loop MPC steps per scenario in one launch (see nmpc_closed_loop_dev).

        p (B,np) and w (B,nw) are advanced in place.  Target controls v_t, w_t:
        (B,) per scenario, (1,) shared, (K,1) one schedule for all scenarios
        (targets.schedule), or (K,B).  ``hist`` may hold device tensors
        u (K,B,6), x (K,B,8), f (K,B), fov (K,B), status/iters (K,B) int32.
        ``p_step`` (K,np), optional: added to p[11:] after each step (moving
        obstacles, targets.obstacle_steps).
        ``order`` (B,) int32 device tensor, optional: dispatch order, a permutation
        of range(B) (schedule.longest_first); results do not depend on it.  Validated
        (ValueError) when ``check`` is set; with ``check=False`` a non-permutation is
        reported by check_closed_loop instead.
        ``check`` (default): synchronise and raise unless every scenario completed its K
        steps (check_closed_loop); pass False to stay asynchronous and call
        check_closed_loop later.
        ``_validate_order=False`` (tests only) hands a non-permutation to the device, whose
        completion guard must then report the scenarios it leaves unrun.
        """
        import torch

        L = _lib.lib()
        B = w.shape[0]
        hist = hist or {}

        def dv(t, n):
            assert t.dtype == torch.float64 and t.is_cuda and t.is_contiguous()
            if t.dim() == 1:
                assert t.shape[0] == n
                return C.c_void_p(t.data_ptr()), 0
            assert t.shape == (B, n), (tuple(t.shape), (B, n))
            return C.c_void_p(t.data_ptr()), n

        ins = []
        for t, n in ((lbx, self.nw), (ubx, self.nw), (lbg, self.ng), (ubg, self.ng)):
            ins += list(dv(t, n))
        assert p.shape == (B, self.np) and p.is_contiguous() and p.dtype == torch.float64
        assert w.shape == (B, self.nw) and w.is_contiguous() and w.dtype == torch.float64
        assert v_t.shape == w_t.shape and v_t.dtype == torch.float64 and w_t.dtype == torch.float64
        assert v_t.is_contiguous() and w_t.is_contiguous() and v_t.is_cuda and w_t.is_cuda
        if v_t.dim() == 2:
            assert v_t.shape[0] == K and v_t.shape[1] in (1, B), tuple(v_t.shape)
            ld_tk, ld_tb = v_t.shape[1], (1 if v_t.shape[1] == B and B > 1 else 0)
        else:
            assert v_t.dim() == 1 and v_t.shape[0] in (1, B), tuple(v_t.shape)
            ld_tk, ld_tb = 0, (1 if v_t.shape[0] == B and B > 1 else 0)
        for t, shp, dt in (("u", (K, B, 6), torch.float64), ("x", (K, B, 8), torch.float64),
                           ("f", (K, B), torch.float64), ("fov", (K, B), torch.float64),
                           ("status", (K, B), torch.int32), ("iters", (K, B), torch.int32)):
            if hist.get(t) is not None:
                assert tuple(hist[t].shape) == shp and hist[t].dtype == dt and hist[t].is_contiguous(), t

        def op(k):
            t = hist.get(k)
            return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)

        ps_ld = 0
        if p_step is not None:
            assert p_step.dtype == torch.float64 and p_step.is_cuda and p_step.is_contiguous()
            assert tuple(p_step.shape) == (K, self.np), (tuple(p_step.shape), (K, self.np))
            ps_ld = self.np
        if order is not None:
            assert order.dtype == torch.int32 and order.is_cuda and order.is_contiguous()
            assert tuple(order.shape) == (B,), tuple(order.shape)
            # a dispatch order must be a permutation: a duplicate would run one scenario
            # on two waves at once (the completion check would still flag the missing one).
            # Checked on the synchronous path only: the check reads the device tensor back,
            # and check=False promises no host synchronisation (the device completion guard
            # reports a scenario a bad order leaves unrun)
            if check and _validate_order and not torch.equal(torch.sort(order).values,
                                                   torch.arange(B, dtype=torch.int32, device=order.device)):
                raise ValueError("order must be a permutation of range(B)")
        if stream is None:
            stream = torch.cuda.current_stream()
        _lib.check(L.nmpc_closed_loop_dev(self._h, B, K, *ins, C.c_void_p(p.data_ptr()), self.np,
                                          C.c_void_p(w.data_ptr()), C.c_void_p(v_t.data_ptr()),
                                          C.c_void_p(w_t.data_ptr()), ld_tk, ld_tb,
                                          C.c_void_p(p_step.data_ptr() if p_step is not None else 0), ps_ld,
                                          op("u"), op("x"),
                                          op("f"), op("fov"), op("status"), op("iters"),
                                          C.c_void_p(order.data_ptr() if order is not None else 0),
                                          C.c_void_p(stream.cuda_stream)))
        if check:
            self.check_closed_loop(B, K)

    def reserve_equality(self, B: int):
        """Allocate the equality class's device workspace for B scenarios (nmpc_reserve_eq):
        the device entry points (solve_device, closed_loop_device) never allocate it
        themselves, so that they never synchronise the host.  The host-array call
        (``solver(...)``) allocates it on demand."""
        _lib.check(_lib.lib().nmpc_reserve_eq(self._h, int(B)))

    def set_trace(self, enable: bool):
        _lib.check(_lib.lib().nmpc_set_trace(self._h, int(enable)))

    def read_trace(self, B: int) -> np.ndarray:
        buf = np.zeros((B, self.max_iter + 3, _lib.TRACE_FIELDS))
        _lib.check(_lib.lib().nmpc_read_trace(self._h, B, _dptr(buf)))
        return buf

    def closed_loop_info(self):
        """Scheduling of the last closed_loop_device launch (nmpc_closed_loop_info;
        synchronises the stream that launch was enqueued on before reading its flags)."""
        pol, res, err, wav, done = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        _lib.check(_lib.lib().nmpc_closed_loop_info(self._h, C.byref(pol), C.byref(res), C.byref(err),
                                                    C.byref(wav), C.byref(done)))
        return {"policy": ("step_queues" if pol.value == 1 else "per_scenario"), "resident_waves": res.value,
                "launched_waves": wav.value, "scheduler_error": err.value, "steps_done": done.value}

    def check_closed_loop(self, B: int, K: int):
        """Raise if the last closed-loop launch did not run every (scenario, step)."""
        info = self.closed_loop_info()
        if info["scheduler_error"] & 4:
            raise _lib.NmpcError("closed loop not run: the batch has equality rows (lbg == ubg) and the "
                                 "equality workspace is not reserved (Solver.reserve_equality(B)); the steps "
                                 f"carry status {_lib.EQ_UNRESERVED}")
        if info["scheduler_error"] != 0 or info["steps_done"] != B * K:
            raise _lib.NmpcError(f"closed loop incomplete: {info['steps_done']} of {B * K} steps run, "
                                 f"scheduler_error={info['scheduler_error']} (unrun steps carry status "
                                 f"{NOT_RUN} in the history)")
        return info

    def closed_loop_times(self, B: int, K: int):
        """Diagnostics (NMPC_STEP_TIMES set before the launch): (K, B, 3) uint64 --
        start / end s_memrealtime stamps (100 MHz) of every step and the running wave."""
        out = np.zeros((K, B, 3), dtype=np.uint64)
        _lib.check(_lib.lib().nmpc_closed_loop_times(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), out.size))
        return out

    def kernel_info(self):
        lds, tps = C.c_int32(), C.c_int32()
        _lib.check(_lib.lib().nmpc_kernel_info(self._h, C.byref(lds), C.byref(tps)))
        return {"lds_bytes": lds.value, "threads_per_scenario": tps.value}

    def memory_info(self):
        """Device workspace the handle holds: the problem class's, and the equality class's
        (allocated only once a batch with equality rows was solved); per-scenario sizes."""
        v = [C.c_int64() for _ in range(4)]
        _lib.check(_lib.lib().nmpc_memory_info(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("ws_bytes", "ws_eq_bytes", "ws_per_scenario", "ws_eq_per_scenario"), (x.value for x in v)))

    def stats(self) -> dict:
        return dict(self._stats)


def nlpsol(name: str, plugin: str, spec: ProblemSpec, opts: dict | None = None) -> Solver:
    """``ca.nlpsol(name, 'ipopt', nlp_prob, opts)`` for the NMPC_TT problem family."""
    if plugin != "ipopt":
        raise ValueError(f"only the 'ipopt' plugin is provided (got {plugin!r})")
    return Solver(name, spec, opts)
