"""ctypes binding of the C-ABI in include/nmpc_amd.h (libnmpc_amd.so).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if the shared object is missing or fails to load, every
entry point raises -- the product never silently runs on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os

MAX_OBS = 16
MAX_N = 63
TRACE_FIELDS = 12
EQ_UNRESERVED = -102  # NMPC_STATUS_EQ_UNRESERVED (IPOPT Insufficient_Memory)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnmpc_amd.so")
# diagnostics only: NMPC_LIB=<path> loads e.g. the -DNMPC_STAMPS phase-timer build
if os.environ.get("NMPC_LIB"):
    LIB_PATH = os.environ["NMPC_LIB"]

# every symbol include/nmpc_amd.h declares (checked by tests/test_capi.py)
EXPORTS = (
    "nmpc_default_options", "nmpc_create", "nmpc_destroy", "nmpc_dims",
    "nmpc_solve_batch", "nmpc_solve_batch_dev", "nmpc_set_trace", "nmpc_read_trace",
    "nmpc_shift_dev", "nmpc_closed_loop_dev", "nmpc_closed_loop_info", "nmpc_last_error", "nmpc_kernel_info",
    "nmpc_build_id", "nmpc_closed_loop_times", "nmpc_memory_info", "nmpc_reserve_eq",
)

_OPT_INT = ("max_iter", "acceptable_iter", "max_soc", "max_soft_resto_iters",
            "watchdog_shortened_iter_trigger", "watchdog_trial_iter_max", "linear_solver_fp32", "reserved0")
_OPT_DBL = (
    "tol", "acceptable_tol", "acceptable_obj_change_tol", "acceptable_dual_inf_tol",
    "acceptable_constr_viol_tol", "acceptable_compl_inf_tol",
    "dual_inf_tol", "constr_viol_tol", "compl_inf_tol",
    "mu_init", "kappa_mu", "theta_mu", "barrier_tol_factor", "tau_min",
    "bound_push", "bound_frac", "slack_bound_push", "slack_bound_frac", "bound_relax_factor",
    "bound_mult_init_val", "constr_mult_init_max",
    "nlp_scaling_max_gradient", "nlp_scaling_min_value", "kappa_d", "kappa_sigma", "s_max",
    "theta_max_fact", "theta_min_fact", "gamma_theta", "gamma_phi", "delta", "s_theta", "s_phi", "eta_phi",
    "alpha_red_factor", "alpha_min_frac", "kappa_soc", "obj_max_inc",
    "first_hessian_perturbation", "min_hessian_perturbation", "max_hessian_perturbation",
    "perturb_inc_fact_first", "perturb_inc_fact", "perturb_dec_fact",
    "tiny_step_tol", "soft_resto_pderror_reduction_factor",
    "resto_penalty_parameter", "resto_proximity_weight", "required_infeasibility_reduction",
    "bound_mult_reset_threshold", "constr_mult_reset_threshold",
)
# IPOPT's option names for the fields whose C name differs
IPOPT_ALIASES = {
    "mu_linear_decrease_factor": "kappa_mu",
    "mu_superlinear_decrease_power": "theta_mu",
    "delta_xs_init": "first_hessian_perturbation",
}


class Options(C.Structure):
    _fields_ = [(n, C.c_int32) for n in _OPT_INT] + [(n, C.c_double) for n in _OPT_DBL]


class Desc(C.Structure):
    _fields_ = [
        ("model", C.c_int32), ("N", C.c_int32), ("np", C.c_int32), ("n_obs", C.c_int32),
        ("T", C.c_double), ("w1", C.c_double), ("w2", C.c_double),
        ("vfov", C.c_double), ("hfov", C.c_double),
        ("obs_x", C.c_double * MAX_OBS), ("obs_y", C.c_double * MAX_OBS),
        ("obs_rsum", C.c_double * MAX_OBS),
        ("obs_x_pidx", C.c_int32 * MAX_OBS), ("obs_y_pidx", C.c_int32 * MAX_OBS),
        ("opts", Options),
        ("w1_pidx", C.c_int32), ("w2_pidx", C.c_int32),
    ]


class NmpcError(RuntimeError):
    """A non-zero return code of the C-ABI (invalid argument or HIP failure)."""


_lib = None


def lib():
    """Load libnmpc_amd.so (raises if it is absent: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built; run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    L = C.CDLL(LIB_PATH)
    dp, i64, i32p, vp = C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_int32), C.c_void_p
    L.nmpc_default_options.argtypes = [C.POINTER(Options)]
    L.nmpc_default_options.restype = None
    L.nmpc_create.argtypes = [C.POINTER(Desc), C.POINTER(vp)]
    L.nmpc_destroy.argtypes = [vp]
    L.nmpc_dims.argtypes = [vp, i32p, i32p, i32p, i32p]
    args = [vp, C.c_int32] + [dp, i64] * 6 + [dp] * 7 + [i32p, i32p]
    L.nmpc_solve_batch.argtypes = args
    L.nmpc_solve_batch_dev.argtypes = [vp, C.c_int32] + [vp, i64] * 6 + [vp] * 7 + [vp, vp, vp]
    L.nmpc_set_trace.argtypes = [vp, C.c_int32]
    L.nmpc_read_trace.argtypes = [vp, C.c_int32, dp]
    L.nmpc_shift_dev.argtypes = [vp, C.c_int32, vp, i64, vp, vp, vp, vp, vp]
    L.nmpc_closed_loop_dev.argtypes = ([vp, C.c_int32, C.c_int32] + [vp, i64] * 4 + [vp, i64] + [vp] * 3
                                       + [i64, i64] + [vp, i64] + [vp] * 8)
    L.nmpc_last_error.argtypes = []
    L.nmpc_last_error.restype = C.c_char_p
    L.nmpc_closed_loop_times.argtypes = [vp, C.POINTER(C.c_uint64), i64]
    L.nmpc_build_id.argtypes = []
    L.nmpc_build_id.restype = C.c_char_p
    L.nmpc_kernel_info.argtypes = [vp, i32p, i32p]
    L.nmpc_memory_info.argtypes = [vp] + [C.POINTER(C.c_int64)] * 4
    if hasattr(L, "nmpc_reserve_eq") or not os.environ.get("NMPC_LIB"):  # (an older diagnostic build may lack it)
        L.nmpc_reserve_eq.argtypes = [vp, C.c_int32]
    L.nmpc_closed_loop_info.argtypes = [vp, i32p, i32p, i32p, i32p, C.POINTER(C.c_int64)]
    for n in EXPORTS:
        if n not in ("nmpc_default_options", "nmpc_last_error", "nmpc_build_id") and hasattr(L, n):
            getattr(L, n).restype = C.c_int
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        msg = lib().nmpc_last_error()
        raise NmpcError(f"nmpc C-ABI error {rc}: {msg.decode() if msg else ''}")


def default_options() -> Options:
    o = Options()
    lib().nmpc_default_options(C.byref(o))
    return o
