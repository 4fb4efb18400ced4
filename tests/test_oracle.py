"""CPU tests: the oracle against committed golden vectors.

* derivs_*.npz: SymPy-differentiated restatement of the reference NLP
  (tests/golden/gen_golden.py) -- pins F, grad F, g, J and the Lagrangian
  Hessian of oracle/nmpc_oracle.py's hand-derived derivatives.
* solutions_*.npz: the oracle's own converged solutions (regression pin) with
  SciPy SLSQP's objective as an independent-solver cross-check.
* The reference's literal N=15 bound vectors (Python/NMPC_TT.py:269-306,
  Python/10_obstacles.py:314-366) pin the generalised bounds generator.

IPOPT itself is absent here, so parity with IPOPT is unpinned.
"""
import glob
import math
import os

import numpy as np
import pytest

from oracle import nmpc_oracle as orc

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _prob_from(z):
    obs = z["obs"]
    return orc.Problem(N=int(z["N"]), T=float(z["T"]), obs_x=obs[:, 0], obs_y=obs[:, 1], obs_rsum=obs[:, 2],
                       obs_y_pidx=z["ypidx"], np_=int(z["npar"]))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "derivs_*.npz"))))
def test_derivatives_vs_sympy(path):
    z = np.load(path)
    prob = _prob_from(z)
    for i in range(len(z["w"])):
        ev = orc.SSEval(prob, z["w"][i], z["p"][i])
        assert ev.F == pytest.approx(float(z["F"][i]), rel=1e-12, abs=1e-9)
        np.testing.assert_allclose(ev.g, z["g"][i], rtol=1e-12, atol=1e-9)
        sc = np.max(np.abs(z["grad"][i]))
        np.testing.assert_allclose(ev.gradF, z["grad"][i], rtol=0, atol=1e-10 * sc)
        sj = np.max(np.abs(z["J"][i]))
        np.testing.assert_allclose(ev.J, z["J"][i], rtol=0, atol=1e-11 * sj)
        W = ev.hessian(float(z["of"][i]), z["lam"][i])
        sw = np.max(np.abs(z["W"][i]))
        np.testing.assert_allclose(W, z["W"][i], rtol=0, atol=1e-9 * sw)


def test_derivatives_finite_difference():
    prob = orc.make_problem("race_track_2", N=6, T=0.2)
    lbx, ubx, _, _ = orc.bounds(prob)
    rng = np.random.default_rng(3)
    w = rng.uniform(lbx, ubx)
    p = np.array([300.0, 400, 100, 0.05, 0.3, 0.1, -0.1, 0.3, 330, 420, 0.2])
    ev = orc.SSEval(prob, w, p)
    h = 1e-6
    E = np.eye(prob.nw)
    g_fd = np.array([(orc.objective(prob, w + h * e, p) - orc.objective(prob, w - h * e, p)) / (2 * h) for e in E])
    np.testing.assert_allclose(ev.gradF, g_fd, rtol=0, atol=1e-6 * np.max(np.abs(g_fd)))


def _ref_bounds_n15(m_rows, n_obs):
    """The reference's literal slice assignments for N=15 (F3/F4)."""
    N = 15
    nrow = m_rows * (N + 1)
    stop = 128 if m_rows == 8 else 240
    lbg = np.zeros(m_rows * (N + 1)) if m_rows == 15 else np.zeros(8 * (N + 1))
    ubg = np.zeros_like(lbg)
    lbg[0:stop:m_rows] = 75; ubg[0:stop:m_rows] = 150
    lbg[1:stop:m_rows] = -0.2618; ubg[1:stop:m_rows] = 0.2618
    lbg[2:stop:m_rows] = -math.pi / 6; ubg[2:stop:m_rows] = math.pi / 6
    lbg[3:stop:m_rows] = -math.pi / 6; ubg[3:stop:m_rows] = math.pi / 6
    lbg[4:stop:m_rows] = -math.pi / 2; ubg[4:stop:m_rows] = math.pi / 2
    for j in range(5, 5 + n_obs):
        lbg[j:stop:m_rows] = -np.inf
        ubg[j:stop:m_rows] = 0
    lbx = np.zeros(6 * N); ubx = np.zeros(6 * N)
    for j, (lo, hi) in enumerate([(14, 30), (-math.pi / 30, math.pi / 30), (-math.pi / 21, math.pi / 21),
                                  (-math.pi / 30, math.pi / 30), (-math.pi / 30, math.pi / 30),
                                  (-math.pi / 30, math.pi / 30)]):
        lbx[j:6 * N:6] = lo; ubx[j:6 * N:6] = hi
    assert len(lbg) == nrow
    return lbx, ubx, lbg, ubg


@pytest.mark.parametrize("layout,m_rows", [("nmpc_tt", 8), ("10_obstacles", 15)])
def test_bounds_reproduce_reference_n15(layout, m_rows):
    prob = orc.make_problem(layout, N=15, T=1.0)
    got = orc.bounds(prob)
    want = _ref_bounds_n15(m_rows, prob.n_obs)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


def test_bounds_general_n_stays_feasible():
    # the reference's strides leave lbg=ubg=0 past stage 15; ours do not
    prob = orc.make_problem("race_track_2", N=20, T=0.2)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    assert len(lbg) == prob.ng == 15 * 21
    assert np.all(lbg < ubg)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "solutions_*.npz"))))
def test_oracle_solutions_regression(path):
    z = np.load(path)
    layout = str(z["layout"])
    prob = orc.make_problem(layout, N=int(z["N"]), T=float(z["T"]))
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    solver = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    for i in range(min(3, len(z["p"]))):
        r = solver.solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, z["p"][i])
        assert r["status"] == int(z["status"][i])
        assert r["iter"] == int(z["iter"][i])
        np.testing.assert_allclose(r["x"], z["x"][i], rtol=1e-9, atol=1e-9)
        if r["status"] == 0:
            # independent solver (SciPy SLSQP from the same point) finds no better objective
            assert z["slsqp_f"][i] >= r["f"] - 1e-6 * (1 + abs(r["f"]))


def test_oracle_kkt_certificate():
    z = np.load(os.path.join(GOLD, "solutions_race_track_2_n10.npz"))
    prob = orc.make_problem("race_track_2", N=int(z["N"]), T=float(z["T"]))
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    for i in range(len(z["p"])):
        if z["status"][i] != 0:
            continue
        ev = orc.SSEval(prob, z["x"][i], z["p"][i])
        stat = ev.gradF + ev.J.T @ z["lam_g"][i] + z["lam_x"][i]
        assert np.max(np.abs(stat)) <= 1e-6 * (1 + np.max(np.abs(ev.gradF)))
        assert np.all(ev.g <= ubg + 1e-6) and np.all(ev.g >= lbg - 1e-6)
        # complementarity: multipliers vanish away from the bounds
        act_u = ubg - ev.g
        act_l = ev.g - lbg
        lam = z["lam_g"][i]
        assert np.max(np.abs(np.where(lam > 0, lam * act_u, 0))) < 1e-6
        assert np.max(np.abs(np.where(lam < 0, lam * np.where(np.isfinite(act_l), act_l, 0), 0))) < 1e-6


def test_closed_loop_shift_matches_reference_formula():
    # Python/NMPC_TT.py:13-30 on a hand-computed case
    prob = orc.make_problem(None, N=3, T=1.0)
    x0 = np.array([90.0, 150, 80, 0, 0, 0, 0, 0])
    u = np.tile(np.array([[20.0], [0.01], [0.02], [0.0], [0.0], [0.0]]), (1, 3))
    u[0, 1] = 21.0
    xs = np.array([100.0, 150, 0.0])
    x1, u1, xs1 = orc.shift_timestep(prob, x0, u, xs)
    np.testing.assert_allclose(x1[:3], [110.0, 150, 80])
    np.testing.assert_allclose(x1[3:5], [0.01, 0.02])
    assert u1[0, 0] == 21.0 and u1[0, 2] == 20.0
    np.testing.assert_allclose(xs1, [112.0, 150.0, 0.01])


def test_no_gimbal_model_functions_and_bounds():
    """No-gimbal variant (MATLAB/Dynamic Obstacles/NMPC_TT.m): 5-state kinematics
    (:37-38), distance cost (:102-105), rows [z, theta] (:129-134) and the
    script's literal N=15 bound vectors (:140-149)."""
    import math
    prob5 = orc.make_problem(None, N=15, T=0.2, model="uav5")
    lbx, ubx, lbg, ubg = orc.bounds(prob5)
    assert len(lbx) == 45 and len(lbg) == 32
    np.testing.assert_array_equal(lbg[0::2], 75.0)
    np.testing.assert_array_equal(ubg[0::2], 150.0)
    np.testing.assert_array_equal(lbg[1::2], -0.2618)
    np.testing.assert_array_equal(ubg[1::2], 0.2618)
    np.testing.assert_array_equal(lbx[0::3], 14.0)
    np.testing.assert_array_equal(ubx[1::3], math.pi / 30)
    np.testing.assert_array_equal(ubx[2::3], math.pi / 21)
    rng = np.random.default_rng(3)
    w5 = rng.uniform(lbx, ubx)
    p5 = np.array([90.0, 150.0, 80.0, 0.05, 0.3, 100.0, 150.0, 0.0])
    # literal restatement of the MATLAB rollout / objective / g
    X = np.zeros((5, 16))
    X[:, 0] = p5[:5]
    U = w5.reshape(15, 3).T
    F = 0.0
    for k in range(15):
        th, ps, v = X[3, k], X[4, k], U[0, k]
        X[:, k + 1] = X[:, k] + 0.2 * np.array([v * math.cos(ps) * math.cos(th), v * math.sin(ps) * math.cos(th),
                                                v * math.sin(th), U[1, k], U[2, k]])
        F += math.sqrt((X[0, k] - p5[5]) ** 2 + (X[1, k] - p5[6]) ** 2)
    assert abs(orc.objective(prob5, w5, p5) - F) <= 1e-12 * F
    np.testing.assert_allclose(orc.constraints(prob5, w5, p5), X[2:4].T.ravel(), rtol=1e-14)
    # derivatives: finite differences of the literal functions
    ev = orc.SSEval(prob5, w5, p5)
    h = 1e-6
    for j in (0, 7, 20, 44):
        e = np.zeros(45)
        e[j] = h
        fd = (orc.objective(prob5, w5 + e, p5) - orc.objective(prob5, w5 - e, p5)) / (2 * h)
        assert abs(ev.gradF[j] - fd) <= 1e-6 * (1 + abs(fd))
        fdg = (orc.constraints(prob5, w5 + e, p5) - orc.constraints(prob5, w5 - e, p5)) / (2 * h)
        np.testing.assert_allclose(ev.J[:, j], fdg, atol=1e-6)


def _pinned_z_problem(b, dz=1.0, k=6):
    """Race Track 2 layout, N = 8: z at stage k pinned (lbg == ubg) to the free optimum's
    height + dz, a reachable target (|dz| is within a few steps' climb)."""
    from nmpc_amd import make_spec, draw_scenarios
    prob = orc.make_problem("race_track_2", N=8, T=0.2)
    p = draw_scenarios(make_spec("race_track_2", N=8, T=0.2), 4, seed=11)[b]
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    r0 = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    X0 = orc.rollout(prob, np.reshape(r0["x"], (6, prob.N), order="F"), p[:8])
    row = k * prob.m
    lbg, ubg = lbg.copy(), ubg.copy()
    lbg[row] = ubg[row] = X0[2, k] + dz
    return prob, p, lbx, ubx, lbg, ubg, row


@pytest.mark.parametrize("b", [0, 1, 2])
def test_equality_row_solved_as_ipopt_does(b):
    """lbg == ubg: c(x) = 0 through the augmented system (Schur complement, Haynsworth
    inertia test).  Checked against SciPy SLSQP's objective on the same NLP and by the KKT
    certificate of the returned point."""
    from scipy.optimize import minimize
    prob, p, lbx, ubx, lbg, ubg, row = _pinned_z_problem(b)
    r = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    assert r["status"] == orc.SOLVE_SUCCEEDED
    g = orc.constraints(prob, r["x"], p)
    assert abs(g[row] - lbg[row]) <= 1e-6
    ineq = np.isfinite(lbg) & (lbg != ubg), np.isfinite(ubg) & (lbg != ubg)
    cons = [{"type": "eq", "fun": lambda w: orc.constraints(prob, w, p)[row] - lbg[row]},
            {"type": "ineq", "fun": lambda w: np.concatenate([(orc.constraints(prob, w, p) - lbg)[ineq[0]],
                                                             (ubg - orc.constraints(prob, w, p))[ineq[1]]])}]
    sl = minimize(lambda w: orc.objective(prob, w, p), r["x"], method="SLSQP", bounds=list(zip(lbx, ubx)),
                  constraints=cons, options={"maxiter": 500, "ftol": 1e-12})
    assert sl.success and r["f"] <= sl.fun + 1e-6 * (1 + abs(sl.fun))
    # stationarity with the returned multipliers (CasADi's sign convention)
    ev = orc.SSEval(prob, r["x"], p)
    res = ev.gradF + ev.J.T @ r["lam_g"] + r["lam_x"]
    assert np.max(np.abs(res)) <= 1e-5 * (1 + np.max(np.abs(ev.gradF)))


@pytest.mark.parametrize("N,n_eq", [(16, 8), (20, 40)])
def test_reference_bounds_at_n_not_15_are_equality_rows(N, n_eq):
    """Python/NMPC_TT.py:271-291 run at N != 15 leaves the rows past index 128
    at lbg = ubg = 0 (z = 0, theta = 0, ... and every obstacle row active): equality rows of
    an infeasible NLP.  IPOPT's path for it -- restoration, then Infeasible_Problem_Detected
    -- is restated; the kernel test (tests/test_gpu_equality.py) compares with this."""
    lbx, ubx, lbg, ubg = reference_bounds_literal(N)
    assert int(np.sum(lbg == ubg)) == n_eq
    prob = orc.make_problem("nmpc_tt", N=N, T=1.0)
    p = np.array([90, 150, 80, 0, 0, 0, 0, 0, 100, 150, 0.0])  # Python/NMPC_TT.py:57-58,316-339
    r = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    assert r["status"] == orc.INFEASIBLE_PROBLEM_DETECTED


def reference_bounds_literal(N, m_rows=8, n_obs=3, stop=128):
    """Python/NMPC_TT.py:269-306 verbatim for any N: lbg/ubg sized n_states_u*(N+1), the
    row slices hard-coded to stop at 128 (F3), lbx/ubx sliced with N."""
    lbg = np.zeros(m_rows * (N + 1))
    ubg = np.zeros_like(lbg)
    lbg[0:stop:m_rows] = 75; ubg[0:stop:m_rows] = 150
    lbg[1:stop:m_rows] = -0.2618; ubg[1:stop:m_rows] = 0.2618
    lbg[2:stop:m_rows] = -math.pi / 6; ubg[2:stop:m_rows] = math.pi / 6
    lbg[3:stop:m_rows] = -math.pi / 6; ubg[3:stop:m_rows] = math.pi / 6
    lbg[4:stop:m_rows] = -math.pi / 2; ubg[4:stop:m_rows] = math.pi / 2
    for j in range(5, 5 + n_obs):
        lbg[j:stop:m_rows] = -np.inf
        ubg[j:stop:m_rows] = 0
    lbx = np.zeros(6 * N); ubx = np.zeros(6 * N)
    for j, (lo, hi) in enumerate([(14, 30), (-math.pi / 30, math.pi / 30), (-math.pi / 21, math.pi / 21),
                                  (-math.pi / 30, math.pi / 30), (-math.pi / 30, math.pi / 30),
                                  (-math.pi / 30, math.pi / 30)]):
        lbx[j:6 * N:6] = lo; ubx[j:6 * N:6] = hi
    return lbx, ubx, lbg, ubg


def test_oracle_records_restoration_checks():
    """The oracle's convergence-check record (the parity tests' termination margins) holds
    the restoration NLP's own checks too (resto=True), as the kernel's trace does (negative
    error in fields 8..11): an Infeasible_Problem_Detected step of the 10_obstacles.py run
    ends on such a check, converged (scaled NLP error at or below tol)."""
    import os
    import sys
    GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, GOLD)
    from gen_reference_runs import run_problem, warm_start
    z = np.load(os.path.join(GOLD, "ref_run_10_obstacles.npz"))
    prob = run_problem("10_obstacles")
    ipo = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    tol = orc.REFERENCE_OPTS.get("tol", orc.IPOPT_DEFAULTS["tol"])
    k = int(np.flatnonzero(z["status"] == orc.INFEASIBLE_PROBLEM_DETECTED)[0])
    w = warm_start(z["x"][k - 1]) if k > 0 else np.zeros(prob.nw)
    r = ipo.solve(w, z["lbx"], z["ubx"], z["lbg"], z["ubg"], z["p"][k], trace=True)
    res = [c for c in ipo.chk if c.get("resto")]
    assert r["status"] == orc.INFEASIBLE_PROBLEM_DETECTED and r["iter"] == z["iter"][k]
    assert res and res[-1]["it"] == r["iter"] and res[-1]["err"] <= tol
    assert all(c["err"] > tol for c in res[:-1] if c["it"] < r["iter"] - 1) or len(res) == 1
