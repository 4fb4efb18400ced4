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


@pytest.mark.parametrize("N", [16, 17, 20, 25])
def test_reference_bounds_at_n_not_15_match_oracle(N):
    """8, 16, 40 and 80 equality rows: the Schur step holds up to 128 (lane l owns rows l and
    l + 64 of S), so the kernel returns the oracle's status, not -11."""
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


def test_more_than_128_equality_rows_is_invalid_problem():
    # more than NMPC_MEQ (128) equality rows: Invalid_Problem_Definition (-11), documented
    lbx, ubx, lbg, ubg = reference_bounds_literal(32)  # 136 equality rows
    prob = orc.make_problem("nmpc_tt", N=32, T=1.0)
    p = np.array([90, 150, 80, 0, 0, 0, 0, 0, 100, 150, 0.0])
    _, st = _gpu_solve("nmpc_tt", 32, 1.0, np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
    assert int(np.ravel(st["status_code"])[0]) == -11


def test_mixed_batch_with_per_scenario_bounds_matches_oracle():
    """Per-scenario bounds (ld_lbg > 0): scenario 0 has a pinned row, scenario 1 none.  The
    batch runs on the equality class (the device flag is batch-wide), whose path for a
    scenario without equality rows is the ordinary one: both match the oracle."""
    prob, p0, lbx, ubx, lbg0, ubg0, row = _pinned_z_problem(0)
    _, p1, _, _, lbg1, ubg1, _ = _pinned_z_problem(1)
    lbg1, ubg1 = orc.bounds(prob)[2:]
    P = np.stack([p0, p1], axis=1)
    LG, UG = np.stack([lbg0, lbg1], axis=1), np.stack([ubg0, ubg1], axis=1)
    sol, st = _gpu_solve("race_track_2", 8, 0.2, np.zeros((prob.nw, 2)), lbx, ubx, LG, UG, P)
    for b, (lg, ug, p) in enumerate(((lbg0, ubg0, p0), (lbg1, ubg1, p1))):
        ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS).solve(np.zeros(prob.nw), lbx, ubx, lg, ug, p)
        print(f"scenario {b}: GPU {int(st['status_code'][b])} / {int(st['iter_count'][b])} iterations, "
              f"oracle {ref['status']} / {ref['iter']}")
        assert int(st["status_code"][b]) == ref["status"]
        assert _rel(sol["x"][:, b], ref["x"]) <= TOL


def test_fp32_leg_rejects_equality_rows():
    # the fp32 Riccati leg has no equality class: Invalid_Problem_Definition (-11)
    from nmpc_amd import nlpsol, make_spec, REFERENCE_OPTS
    prob, p, lbx, ubx, lbg, ubg, row = _pinned_z_problem(0)
    s = nlpsol("solver", "ipopt", make_spec("race_track_2", N=8, T=0.2),
               dict(REFERENCE_OPTS, linear_solver_precision="single"))
    s(x0=np.zeros(prob.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=p)
    assert int(np.ravel(s.stats()["status_code"])[0]) == -11


@pytest.mark.parametrize("extra", [0, 173])
def test_equality_rows_closed_loop_matches_per_step_launches(extra):
    """nmpc_closed_loop_dev with an equality row in the shared bounds runs the equality
    class's closed-loop kernels (one workgroup per scenario, and -- with more scenarios than
    the problem class's resident waves -- the step queues); its histories equal K rounds of
    solve_batch_dev + shift_dev, which run the equality class's solve kernel."""
    import torch
    from nmpc_amd import nlpsol, make_spec, draw_scenarios, REFERENCE_OPTS
    spec = make_spec("race_track_2", N=8, T=0.2)
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    f64 = dict(dtype=torch.float64, device="cuda")
    lbx, ubx, lbg, ubg = (np.array(v, float) for v in spec.bounds())
    if extra:
        P0 = draw_scenarios(spec, 8, seed=5)
        s.closed_loop_device(1, *[torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)], torch.tensor(P0, **f64),
                             torch.zeros(8, spec.nw, **f64),
                             torch.full((8,), 12.0, **f64), torch.full((8,), 0.01, **f64))
        torch.cuda.synchronize()
    B = (s.closed_loop_info()["resident_waves"] + extra) if extra else 48
    K = 3
    P = draw_scenarios(spec, B, seed=21)
    # per-scenario bounds (ld_lbg = ng): z at stage 6 pinned 0.5 m above the scenario's start
    LG, UG = np.tile(lbg, (B, 1)), np.tile(ubg, (B, 1))
    LG[:, 6 * spec.m] = UG[:, 6 * spec.m] = P[:, 2] + 0.5
    bnd = [torch.tensor(lbx, **f64), torch.tensor(ubx, **f64), torch.tensor(LG, **f64), torch.tensor(UG, **f64)]
    vt, wt = torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64)
    p1, w1 = torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64)
    out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
           "status": torch.empty(B, dtype=torch.int32, device="cuda"),
           "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
    ref = {"u": [], "f": [], "status": [], "iters": []}
    s.reserve_equality(B)  # the device entry points never allocate it themselves
    for _ in range(K):
        s.solve_device(w1, *bnd, p1, out)
        ref["u"].append(out["x"][:, :6].clone())
        for k in ("f", "status", "iters"):
            ref[k].append(out[k].clone())
        s.shift_device(p1, out["x"], w1, vt, wt)
    p2, w2 = torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda"),
            "iters": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p2, w2, vt, wt, hist)
    torch.cuda.synchronize()
    info = s.closed_loop_info()
    assert info["policy"] == ("step_queues" if extra else "per_scenario")
    st = hist["status"].cpu().numpy()
    print(f"B={B}: statuses {dict(zip(*np.unique(st, return_counts=True)))}")
    assert np.any(st == 0)
    for k in ("status", "iters"):
        np.testing.assert_array_equal(hist[k].cpu().numpy(), torch.stack(ref[k]).cpu().numpy(), err_msg=k)
    for k in ("u", "f"):
        assert _rel(hist[k].cpu().numpy(), torch.stack(ref[k]).cpu().numpy()) <= 1e-12, k


def _pinned_z_draw(b, dz, k, n=32):
    """Race Track 2 layout, N = 8, scenario b of `n` draws (seed 11): z at stage k pinned
    to the start height + dz (lbg == ubg)."""
    from nmpc_amd import make_spec, draw_scenarios
    prob = orc.make_problem("race_track_2", N=8, T=0.2)
    p = draw_scenarios(make_spec("race_track_2", N=8, T=0.2), n, seed=11)[b]
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    lbg, ubg = lbg.copy(), ubg.copy()
    lbg[k * prob.m] = ubg[k * prob.m] = p[2] + dz
    return prob, p, lbx, ubx, lbg, ubg


# (b, dz, k), the last iteration compared, the watchdog trial iteration left out (see below)
WD_CASES = [((1, 3.0, 2), 20, 15), ((1, 8.0, 4), 25, 20), ((16, 3.0, 6), 27, 19), ((28, 8.0, 6), 36, 32)]


@pytest.mark.parametrize("case,last,skip", WD_CASES)
def test_watchdog_stop_with_equality_rows_matches_oracle(case, last, skip):
    """The watchdog procedure (BacktrackingLineSearch::StartWatchDog / StopWatchDog) on a
    problem with an equality row.  After StopWatchDog the line search runs on the STORED
    step, whose equality-multiplier component dy_c must come back with it (IPOPT keeps the
    whole step in the watchdog's stored point; the kernel's weqy buffer): a stale dy_c
    changes y_c, hence the Lagrangian Hessian of every later iteration.

    These pinned heights are out of reach: the main phase shortens its steps, the watchdog
    starts and is stopped, y_c grows to 1e7..1e12 and the condensed Hessian's condition
    number to ~1e21.  There, on the last watchdog trial iteration before a stop (`skip`),
    the oracle's dense eigenvalue count finds negative eigenvalues of size ~1e4 that are
    rounding noise at that conditioning (the stage-wise Riccati pivots of the kernel and of
    the compiled restatement find none), so the inertia corrections differ -- but that
    trial iterate is discarded by StopWatchDog, and from the restored point on the runs
    agree again.  Compared, per main-phase iteration up to `last` (the compiled
    restatement agrees with the oracle over the same window, measured): the scaled
    objective (1e-9 relative) and the line-search trial count; and the oracle's stops fall
    inside the window."""
    b, dz, k = case
    prob, p, lbx, ubx, lbg, ubg = _pinned_z_draw(b, dz, k)
    ipo = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    ref = ipo.solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p, trace=True)
    stops = [i for i in ipo.wd_stop_its if i <= last]
    # the window exercises StopWatchDog, and the left-out trial iteration is the one it discards
    assert stops and (skip + 1) in ipo.wd_stop_its, ipo.wd_stop_its
    from nmpc_amd import nlpsol, make_spec, REFERENCE_OPTS
    s = nlpsol("solver", "ipopt", make_spec("race_track_2", N=8, T=0.2), REFERENCE_OPTS)
    s.set_trace(True)
    try:
        s(x0=np.zeros(prob.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=p)
        tr = s.read_trace(1)[0]
    finally:
        s.set_trace(False)
    st = s.stats()
    rows = {t["iter"]: t for t in ref["trace"] if not t.get("resto")}
    bad = []
    for it in range(1, last + 1):
        if it == skip:
            continue
        o, g = rows[it], tr[it - 1]
        assert int(g[0]) == it
        if not (abs(g[2] - o["f"]) <= 1e-9 * (1 + abs(o["f"])) and int(g[7]) == o["ls"]):
            bad.append((it, g[2], o["f"], int(g[7]), o["ls"]))
    print(f"{case}: watchdog stops at {ipo.wd_stop_its}; iterations 1..{last} compared (without {skip}); "
          f"GPU status {int(np.ravel(st['status_code'])[0])} / {int(np.ravel(st['iter_count'])[0])} iterations, "
          f"oracle {ref['status']} / {ref['iter']}; mismatches {bad}")
    assert not bad


def test_equality_workspace_is_allocated_lazily():
    """The equality class's workspace (~840 KB per scenario: global rows up to N = 63 and the
    128 x 128 Schur storage) is allocated only when asked for; a config-3 handle whose batches
    have none holds its class's ~120 KB per scenario only.
    Device-pointer batches never allocate it (they never synchronise the host): without it a
    batch with equality rows reports NMPC_STATUS_EQ_UNRESERVED (-102) per scenario with NaN x
    and f, and a closed loop raises (scheduler_error bit 4); after reserve_equality(B) it
    is solved, and a batch without equality rows gives bitwise the same results either way.
    The host-array call allocates it on demand, and an equality batch through the device path
    equals the host path's solve of it."""
    import torch
    from nmpc_amd import nlpsol, config_spec, draw_scenarios, make_spec, REFERENCE_OPTS
    from nmpc_amd._lib import NmpcError, EQ_UNRESERVED

    f64 = dict(dtype=torch.float64, device="cuda")
    spec = config_spec(3)
    s3 = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    B = 256
    P = draw_scenarios(spec, B, seed=1003)
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    hist = {"status": torch.empty(2, B, dtype=torch.int32, device="cuda")}
    s3.closed_loop_device(2, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64),
                          torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64), hist)
    torch.cuda.synchronize()
    mi = s3.memory_info()
    print(mi)
    assert mi["ws_eq_bytes"] == 0 and mi["ws_bytes"] == B * mi["ws_per_scenario"]
    assert mi["ws_per_scenario"] <= 130_000 < mi["ws_eq_per_scenario"]

    prob, p, lbx, ubx, lbg, ubg, row = _pinned_z_problem(0)
    spec8 = make_spec("race_track_2", N=8, T=0.2)
    s = nlpsol("solver", "ipopt", spec8, REFERENCE_OPTS)
    Bs = 3
    pd = torch.tensor(np.tile(p, (Bs, 1)), **f64)
    x0 = torch.zeros(Bs, prob.nw, **f64)

    def dev_solve(lg, ug):
        out = {"x": torch.empty(Bs, prob.nw, **f64), "f": torch.empty(Bs, **f64),
               "status": torch.empty(Bs, dtype=torch.int32, device="cuda"),
               "iters": torch.empty(Bs, dtype=torch.int32, device="cuda")}
        b = [torch.tensor(v, **f64) for v in (lbx, ubx, lg, ug)]
        s.solve_device(x0, *b, pd, out)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in out.items()}

    lbg0, ubg0 = orc.bounds(prob)[2:]
    a1 = dev_solve(lbg0, ubg0)                      # no equality row: the class alone
    assert s.memory_info()["ws_eq_bytes"] == 0
    e0 = dev_solve(lbg, ubg)                        # equality rows, nothing reserved: not solved
    assert s.memory_info()["ws_eq_bytes"] == 0
    assert np.all(e0["status"] == EQ_UNRESERVED) and np.all(np.isnan(e0["x"])) and np.all(np.isnan(e0["f"]))
    # the closed loop reports it too (and raises on the synchronous path)
    hq = {"status": torch.empty(2, Bs, dtype=torch.int32, device="cuda")}
    bq = [torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)]
    with pytest.raises(NmpcError, match="reserve_equality"):
        s.closed_loop_device(2, *bq, pd.clone(), x0.clone(), torch.full((Bs,), 12.0, **f64),
                             torch.full((Bs,), 0.01, **f64), hq)
    assert np.all(hq["status"].cpu().numpy() == EQ_UNRESERVED)
    s.reserve_equality(Bs)
    assert s.memory_info()["ws_eq_bytes"] == Bs * s.memory_info()["ws_eq_per_scenario"]
    e1 = dev_solve(lbg, ubg)                        # equality rows: the equality class
    a2 = dev_solve(lbg0, ubg0)                      # the gated pair, decided on the device
    for k in a1:
        np.testing.assert_array_equal(a1[k], a2[k])
    h = s(x0=np.zeros(prob.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=p)
    assert int(e1["status"][0]) == int(np.ravel(s.stats()["status_code"])[0]) == orc.SOLVE_SUCCEEDED
    np.testing.assert_array_equal(e1["x"][0], h["x"].ravel())
    # the host-array call allocates the workspace on demand
    s2 = nlpsol("solver", "ipopt", spec8, REFERENCE_OPTS)
    h2 = s2(x0=np.zeros(prob.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=p)
    assert s2.memory_info()["ws_eq_bytes"] == s2.memory_info()["ws_eq_per_scenario"]
    np.testing.assert_array_equal(h2["x"], h["x"])
    assert abs(float(h["g"].ravel()[row]) - lbg[row]) <= 1e-6
