"""Equality rows (lbg == ubg) on the GPU against the oracle.

IPOPT treats a row with lbg == ubg as c(x) = g(x) - g_l = 0 (no slack, no bound
relaxation) and solves the augmented Newton system with an inertia test on it.  The
kernel adds such rows through the Schur complement of that system; the
oracle (oracle/nmpc_oracle.py) factors the augmented system densely.  Two cases:

(i)  feasible: z at one stage pinned to a reachable height (the free optimum's + 1 m);
(ii) the reference's own bound vectors run at N != 15 (Python/NMPC_TT.py:271-291, SURVEY
     F3): the rows past index 128 stay lbg = ubg = 0, an infeasible NLP that both end in
     the restoration phase.

Tolerance (north star): x within 1e-6 (1 + |x|) where both converge; statuses equal.
"""
import numpy as np
import pytest

from oracle import nmpc_oracle as orc
from tests.test_oracle import _pinned_z_problem, reference_bounds_literal

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / (1.0 + np.abs(np.asarray(b)))))


def _gpu_solve(layout, N, T, x0, lbx, ubx, lbg, ubg, P):
    from nmpc_amd import nlpsol, make_spec, REFERENCE_OPTS
    solver = nlpsol("solver", "ipopt", make_spec(layout, N=N, T=T), REFERENCE_OPTS)
    sol = solver(x0=x0, lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P)
    return sol, solver.stats()


@pytest.mark.parametrize("b", [0, 1, 2])
def test_pinned_height_matches_oracle(b):
    prob, p, lbx, ubx, lbg, ubg, row = _pinned_z_problem(b)
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    sol, st = _gpu_solve("race_track_2", 8, 0.2, np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    status = int(st["status_code"][0]) if np.ndim(st["status_code"]) else int(st["status_code"])
    print(f"scenario {b}: GPU status {status} iters {st['iter_count']}, oracle {ref['status']} {ref['iter']}")
    assert status == ref["status"] == orc.SOLVE_SUCCEEDED
    assert _rel(sol["x"].ravel(), ref["x"]) <= TOL
    assert abs(float(sol["g"].ravel()[row]) - lbg[row]) <= 1e-6
    assert _rel(sol["lam_g"].ravel()[row], ref["lam_g"][row]) <= 1e-5


@pytest.mark.parametrize("N", [16, 17])
def test_reference_bounds_at_n_not_15_match_oracle(N):
    lbx, ubx, lbg, ubg = reference_bounds_literal(N)
    prob = orc.make_problem("nmpc_tt", N=N, T=1.0)
    p = np.array([90, 150, 80, 0, 0, 0, 0, 0, 100, 150, 0.0])  # Python/NMPC_TT.py:57-58,316-339
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    sol, st = _gpu_solve("nmpc_tt", N, 1.0, np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    status = int(np.ravel(st["status_code"])[0])
    print(f"N={N}: {int(np.sum(lbg == ubg))} equality rows; GPU status {status} iters {st['iter_count']}, "
          f"oracle {ref['status']} {ref['iter']}")
    assert status == ref["status"]
    if status in (0, 1):
        assert _rel(sol["x"].ravel(), ref["x"]) <= TOL


def test_too_many_equality_rows_is_invalid_problem():
    # more than NMPC_MEQ (16) equality rows: Invalid_Problem_Definition (-11), documented
    lbx, ubx, lbg, ubg = reference_bounds_literal(20)  # 40 equality rows
    prob = orc.make_problem("nmpc_tt", N=20, T=1.0)
    p = np.array([90, 150, 80, 0, 0, 0, 0, 0, 100, 150, 0.0])
    _, st = _gpu_solve("nmpc_tt", 20, 1.0, np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    assert int(np.ravel(st["status_code"])[0]) == -11
