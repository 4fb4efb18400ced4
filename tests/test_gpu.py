"""GPU parity tests: the HIP solver (through the C-ABI) against the CPU oracle
(oracle/nmpc_oracle.py, dense single-shooting IPOPT restatement) and the
committed golden solutions.

Tolerance (BASELINE.json north star): trajectories within 1e-6 relative
error, |a-b| <= 1e-6 (1+|b|), for scenarios both solvers converge on.  In
practice the two agree iteration for iteration (same status, same iteration
count, ~1e-14 differences), which is also asserted where it is robust.
"""
import glob
import os

import numpy as np
import pytest

from oracle import nmpc_oracle as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-6


def _rel(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / (1.0 + np.abs(np.asarray(b)))))


def _solver(spec, opts=None, **kw):
    from nmpc_amd import nlpsol, REFERENCE_OPTS

    return nlpsol("solver", "ipopt", spec, REFERENCE_OPTS if opts is None else opts)


def _oracle(layout, N, T, dynamic=False):
    prob = orc.make_problem(layout, N=N, T=T, dynamic=dynamic)
    return prob, orc.IpoptDense(prob, orc.REFERENCE_OPTS)


@pytest.mark.parametrize("layout,N,T,B,seed", [
    ("race_track_2", 20, 0.2, 4, 1003),   # config 3 family
    (None, 20, 0.2, 3, 1002),             # config 2 family (no obstacles)
    ("nmpc_tt", 15, 1.0, 2, 1001),        # Python/NMPC_TT.py as written (T=1, NLP scaling active)
    ("10_obstacles", 15, 0.2, 3, 1004),   # Python/10_obstacles.py layout
    ("race_track_2", 8, 0.2, 3, 7),
])
def test_parity_with_oracle(layout, N, T, B, seed):
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec(layout, N=N, T=T)
    P = draw_scenarios(spec, B, seed=seed)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    st = s.stats()
    prob, ref = _oracle(layout, N, T)
    for b in range(B):
        r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b])
        assert st["status_code"][b] == r["status"], (b, st["status_code"][b], r["status"])
        assert abs(int(st["iter_count"][b]) - r["iter"]) <= 2
        if r["status"] == 0:
            assert _rel(sol["x"][:, b], r["x"]) <= TOL
            assert _rel(sol["X"][:, b], r["X"].T.ravel()) <= TOL
            assert _rel(sol["f"][0, b], r["f"]) <= TOL
            assert _rel(sol["g"][:, b], r["g"]) <= TOL


def test_iteration_traces_match_oracle():
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("race_track_2", N=20, T=0.2)
    P = draw_scenarios(spec, 2, seed=1003)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    s.set_trace(True)
    s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    tr = s.read_trace(2)
    _, ref = _oracle("race_track_2", 20, 0.2)
    for b in range(2):
        r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b], trace=True)
        for k in range(min(8, len(r["trace"]))):
            o = r["trace"][k]
            g = tr[b, k]
            assert g[1] == pytest.approx(o["mu"], rel=1e-12)
            assert g[2] == pytest.approx(o["f"], rel=1e-10)
            assert g[5] == pytest.approx(o["alpha_p"], rel=1e-8, abs=1e-12)
            assert g[7] == o["ls"]


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "solutions_*.npz"))))
def test_golden_solutions(path):
    from nmpc_amd import make_spec

    z = np.load(path)
    spec = make_spec(str(z["layout"]), N=int(z["N"]), T=float(z["T"]))
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=z["p"].T)
    st = s.stats()
    for b in range(len(z["p"])):
        assert st["status_code"][b] == z["status"][b]
        if z["status"][b] == 0:
            assert _rel(sol["x"][:, b], z["x"][b]) <= TOL
            assert _rel(sol["f"][0, b], z["f"][b]) <= TOL
            assert _rel(sol["lam_g"][:, b], z["lam_g"][b]) <= 1e-4


def test_dynamic_obstacles_parity():
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("dynamic", N=12, T=0.2, dynamic=True)
    P = draw_scenarios(spec, 3, seed=1005)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    _, ref = _oracle("dynamic", 12, 0.2, dynamic=True)
    for b in range(3):
        r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b])
        assert s.stats()["status_code"][b] == r["status"]
        if r["status"] == 0:
            assert _rel(sol["x"][:, b], r["x"]) <= TOL


def test_single_scenario_shapes_and_broadcast_bounds():
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("race_track_2", N=10, T=0.2)
    P = draw_scenarios(spec, 3, seed=5)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    one = s(x0=np.zeros((spec.nw, 1)), lbx=lbx[:, None], ubx=ubx[:, None], lbg=lbg, ubg=ubg, p=P[1][:, None])
    assert one["x"].shape == (spec.nw, 1) and one["f"].shape == (1, 1) and one["g"].shape == (spec.ng, 1)
    assert isinstance(s.stats()["return_status"], str)
    u = np.reshape(one["x"], (6, spec.N), order="F")  # ca.reshape(sol['x'], 6, N)
    assert u.shape == (6, spec.N)
    # per-scenario (batched) bounds give bitwise the same result as broadcast bounds
    rep = lambda v: np.repeat(v[:, None], 3, axis=1)
    a = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    b = s(x0=np.zeros((spec.nw, 3)), lbx=rep(lbx), ubx=rep(ubx), lbg=rep(lbg), ubg=rep(ubg), p=P.T)
    np.testing.assert_array_equal(a["x"], b["x"])
    np.testing.assert_array_equal(a["x"][:, 1:2], one["x"])
    with pytest.raises(ValueError):
        s(x0=np.zeros(spec.nw + 1), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P[0])


def test_invalid_inputs_reported_per_scenario():
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("race_track_2", N=6, T=0.2)
    P = draw_scenarios(spec, 4, seed=8)
    lbx, ubx, lbg, ubg = spec.bounds()
    LB = np.repeat(lbx[:, None], 4, 1); UB = np.repeat(ubx[:, None], 4, 1)
    LG = np.repeat(lbg[:, None], 4, 1); UG = np.repeat(ubg[:, None], 4, 1)
    Pt = P.T.copy()
    LB[3, 0] = UB[3, 0] + 1.0          # lbx > ubx -> Invalid_Problem_Definition
    LG[0, 1] = UG[0, 1] + 1.0          # lbg > ubg -> Invalid_Problem_Definition
    Pt[2, 2] = np.nan                  # NaN in p -> Invalid_Number_Detected
    s = _solver(spec)
    s(x0=np.zeros(spec.nw), lbx=LB, ubx=UB, lbg=LG, ubg=UG, p=Pt)
    sc = s.stats()["status_code"]
    assert sc[0] == -11 and sc[1] == -11
    assert sc[2] == -13
    assert sc[3] in (0, 1)             # untouched scenario unaffected by its neighbours


def test_empty_batch_is_noop():
    import ctypes as C
    from nmpc_amd import _lib, make_spec

    s = _solver(make_spec(None, N=4, T=0.2))
    assert _lib.lib().nmpc_solve_batch(s._h, 0, *([None, 0] * 6), *([None] * 7), None, None) == 0


@pytest.mark.parametrize("N,layout", [(1, "race_track_2"), (63, None)])
def test_horizon_limits(N, layout):
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec(layout, N=N, T=0.2)
    P = draw_scenarios(spec, 1, seed=3)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    _, ref = _oracle(layout, N, 0.2)
    r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[0])
    assert s.stats()["status_code"][0] == r["status"]
    if r["status"] == 0:
        assert _rel(sol["x"][:, 0], r["x"]) <= TOL


def test_max_obstacles_and_infinite_bounds():
    from nmpc_amd import spec as S
    from nmpc_amd import draw_scenarios

    rng = np.random.default_rng(0)
    obs = tuple(S.Obstacle(float(x), float(y), 40.0) for x, y in rng.uniform(-300, 1500, (16, 2)))
    spec = S.ProblemSpec(N=10, T=0.2, obstacles=obs).validate()
    P = draw_scenarios(spec, 2, seed=4)
    lbx, ubx, lbg, ubg = spec.bounds()
    lbx = lbx.copy(); ubg = ubg.copy()
    lbx[1::6] = -np.inf                 # no lower bound on omega_2u
    ubg[5::spec.m] = np.inf             # first obstacle row free
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    prob = orc.Problem(N=10, T=0.2, obs_x=[o.x for o in obs], obs_y=[o.y for o in obs],
                       obs_rsum=[o.r for o in obs])
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    for b in range(2):
        r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b])
        assert s.stats()["status_code"][b] == r["status"]
        if r["status"] == 0:
            assert _rel(sol["x"][:, b], r["x"]) <= TOL


def test_full_size_properties():
    """BASELINE config 3 at full size (4096 scenarios): determinism,
    batch-position invariance, KKT certificate on a sample, status set."""
    from nmpc_amd import config_spec, draw_scenarios

    spec = config_spec(3)
    B = 4096
    P = draw_scenarios(spec, B, seed=1003)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    a = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    sa = s.stats()["status_code"].copy()
    b = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    np.testing.assert_array_equal(a["x"], b["x"])
    assert set(np.unique(sa)) <= {0, 1, 2, -1, -2, 3}
    assert np.mean(sa == 0) > 0.95
    one = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P[1234])
    np.testing.assert_array_equal(one["x"][:, 0], a["x"][:, 1234])
    prob = orc.make_problem("race_track_2", N=spec.N, T=spec.T)
    idx = np.flatnonzero(sa == 0)[:: max(1, int(np.sum(sa == 0)) // 16)][:16]
    for i in idx:
        ev = orc.SSEval(prob, a["x"][:, i], P[i])
        stat = ev.gradF + ev.J.T @ a["lam_g"][:, i] + a["lam_x"][:, i]
        assert np.max(np.abs(stat)) <= 1e-6 * (1 + np.max(np.abs(ev.gradF)))
        # Solve_Succeeded means a constraint violation <= constr_viol_tol = 1e-4 (IPOPT's
        # unscaled test) against the bounds relaxed by bound_relax_factor = 1e-8
        viol = max(float(np.max(ev.g - ubg)), float(np.max(lbg - ev.g)), 0.0)
        print(f"scenario {i}: max bound violation {viol:.3e}")
        assert viol <= 1e-4


def test_device_path_matches_host_path():
    import torch
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("race_track_2", N=20, T=0.2)
    B = 8
    P = draw_scenarios(spec, B, seed=11)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    h = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    f64 = dict(dtype=torch.float64, device="cuda")
    out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
           "status": torch.empty(B, dtype=torch.int32, device="cuda"),
           "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
    s.solve_device(torch.zeros(B, spec.nw, **f64), torch.tensor(lbx, **f64), torch.tensor(ubx, **f64),
                   torch.tensor(lbg, **f64), torch.tensor(ubg, **f64), torch.tensor(P, **f64), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["x"].cpu().numpy(), h["x"].T)
    np.testing.assert_array_equal(out["status"].cpu().numpy(), s.stats()["status_code"])


def test_dev_entry_points_do_not_synchronise():
    """nmpc_solve_batch_dev and nmpc_closed_loop_dev only enqueue work (include/nmpc_amd.h:
    "returns without synchronising").  Enqueued on a side stream behind a kernel that spins for
    ~1 s, each call returns while that kernel still runs: the stream is still busy
    (Stream.query() is False) and the call took a small fraction of the spin.  The handle is a
    config-3 one without the equality workspace, the case whose bounds scan once read the
    device flag back (round 5): the rows are now scanned on the device and the class pair is
    gated by the flag with no host round trip.  The results equal an unobstructed run's."""
    import time
    import torch
    from nmpc_amd import config_spec

    spec = config_spec(3)
    s = _solver(spec)
    B, K = 64, 2
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, seed=31)
    f64 = dict(dtype=torch.float64, device="cuda")
    st = torch.cuda.Stream()

    def outs():
        return {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
                "status": torch.empty(B, dtype=torch.int32, device="cuda"),
                "iters": torch.empty(B, dtype=torch.int32, device="cuda")}

    def hists():
        return {"u": torch.empty(K, B, 6, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}

    w0, p0 = torch.zeros(B, spec.nw, **f64), torch.tensor(P, **f64)
    # unobstructed runs first: they also size the workspace and the scheduler state (an
    # allocation may synchronise; a sized handle only enqueues)
    ref_o, ref_h = outs(), hists()
    s.solve_device(w0, *bnd, p0, ref_o, stream=st)
    s.closed_loop_device(K, *bnd, p0.clone(), w0.clone(), vt, wt, ref_h, stream=st, check=False)
    torch.cuda.synchronize()
    assert s.memory_info()["ws_eq_bytes"] == 0
    # calibrate the spin kernel (torch.cuda._sleep: clock cycles) to ~1 s
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record(st); torch.cuda._sleep(1 << 24); e1.record(st)
    torch.cuda.synchronize()
    per_cycle_ms = e0.elapsed_time(e1) / (1 << 24)
    cycles = int(min(max(1000.0 / max(per_cycle_ms, 1e-12), float(1 << 24)), float(1 << 36)))
    for what in ("solve", "closed_loop"):
        o, hh = outs(), hists()
        pc, wc = p0.clone(), w0.clone()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            e0.record(st)
            torch.cuda._sleep(cycles)
            e1.record(st)
        t0 = time.perf_counter()
        if what == "solve":
            s.solve_device(w0, *bnd, p0, o, stream=st)
        else:
            s.closed_loop_device(K, *bnd, pc, wc, vt, wt, hh, stream=st, check=False)
        call_ms = (time.perf_counter() - t0) * 1e3
        busy = not st.query()
        torch.cuda.synchronize()
        spin_ms = e0.elapsed_time(e1)
        print(f"{what}: call {call_ms:.2f} ms, spin {spin_ms:.0f} ms, stream busy after the call: {busy}")
        assert spin_ms > 300.0
        assert busy and call_ms < 0.25 * spin_ms, (what, call_ms, spin_ms)
        if what == "solve":
            for k in o:
                np.testing.assert_array_equal(o[k].cpu().numpy(), ref_o[k].cpu().numpy(), err_msg=k)
        else:
            s.check_closed_loop(B, K)
            for k in hh:
                np.testing.assert_array_equal(hh[k].cpu().numpy(), ref_h[k].cpu().numpy(), err_msg=k)


def test_speculative_restoration_pairs_are_bitwise_neutral(monkeypatch):
    """The restoration line search of the LDS-row class forms each new trial together with
    the next backtracking trial (Solver::kSpec: rollout2 / eval_fg2 on lanes 32 + k, the
    second trial's X, rows and objective parked in lam, dms and spec_f), and a later
    from_pair acceptance -- possibly after a failed second-order correction in between --
    takes that parked trial.  Against a handle whose trials are all formed alone
    (NMPC_NO_SPEC=1 at nmpc_create, Params::nospec), the bench's whole config-3 workload
    (4,096 scenarios x 20 closed-loop steps from u = 0: the restoration-heavy chains that
    bound the launch, with their SOC blocks) gives bitwise the same histories."""
    import torch
    from nmpc_amd import config_spec

    spec = config_spec(3)
    B, K = 4096, 20
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, seed=1003)
    f64 = dict(dtype=torch.float64, device="cuda")

    def run():
        s = _solver(spec)
        hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
                "status": torch.empty(K, B, dtype=torch.int32, device="cuda"),
                "iters": torch.empty(K, B, dtype=torch.int32, device="cuda")}
        p, w = torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64)
        s.closed_loop_device(K, *bnd, p, w, vt, wt, hist)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in hist.items()}, p.cpu().numpy(), w.cpu().numpy()

    a, pa, wa = run()
    monkeypatch.setenv("NMPC_NO_SPEC", "1")
    b, pb, wb = run()
    st = a["status"]
    print(f"iterations {int(a['iters'].sum())}, max_iter steps {int((st == -1).sum())}, "
          f"infeasible {int((st == 2).sum())}")
    assert int((st == -1).sum()) > 100  # restoration-heavy max_iter steps are in the workload
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    np.testing.assert_array_equal(pa, pb)
    np.testing.assert_array_equal(wa, wb)


def test_shift_kernel_matches_reference_shift():
    import torch
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec("race_track_2", N=20, T=0.2)
    B = 5
    P = draw_scenarios(spec, B, seed=12)
    rng = np.random.default_rng(1)
    lbx, ubx, _, _ = spec.bounds()
    U = rng.uniform(lbx, ubx, (B, spec.nw))
    s = _solver(spec)
    f64 = dict(dtype=torch.float64, device="cuda")
    p = torch.tensor(P, **f64)
    w = torch.empty(B, spec.nw, **f64)
    s.shift_device(p, torch.tensor(U, **f64), w, torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64))
    torch.cuda.synchronize()
    prob = orc.make_problem("race_track_2", N=20, T=0.2)
    for b in range(B):
        u = U[b].reshape(spec.N, 6).T
        x1, u1, xs1 = orc.shift_timestep(prob, P[b, :8], u, P[b, 8:11])
        np.testing.assert_allclose(p[b, :8].cpu().numpy(), x1, rtol=1e-15, atol=1e-12)
        np.testing.assert_allclose(p[b, 8:11].cpu().numpy(), xs1, rtol=1e-15, atol=1e-12)
        np.testing.assert_array_equal(w[b].cpu().numpy(), u1.T.ravel())


def _closed_loop_inputs(spec, B, seed):
    import torch
    from nmpc_amd import draw_scenarios

    f64 = dict(dtype=torch.float64, device="cuda")
    P = draw_scenarios(spec, B, seed=seed)
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    return P, bnd, torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64)


def test_closed_loop_kernel_matches_per_step_launches():
    """nmpc_closed_loop_dev (K steps in one launch) == K x (solve_batch_dev + shift_dev)."""
    import torch
    from nmpc_amd import make_spec

    spec = make_spec("race_track_2", N=20, T=0.2)
    B, K = 96, 4
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 1003)
    f64 = dict(dtype=torch.float64, device="cuda")
    s = _solver(spec)
    # per-step launches
    p1 = torch.tensor(P, **f64)
    w1 = torch.zeros(B, spec.nw, **f64)
    out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
           "status": torch.empty(B, dtype=torch.int32, device="cuda"),
           "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
    ref = {"u": [], "x": [], "f": [], "status": [], "iters": []}
    for _ in range(K):
        ref["x"].append(p1[:, :8].clone())
        s.solve_device(w1, *bnd, p1, out)
        ref["u"].append(out["x"][:, :6].clone())
        for k in ("f", "status", "iters"):
            ref[k].append(out[k].clone())
        s.shift_device(p1, out["x"], w1, vt, wt)
    # one launch
    p2 = torch.tensor(P, **f64)
    w2 = torch.zeros(B, spec.nw, **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "x": torch.empty(K, B, 8, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda"),
            "iters": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p2, w2, vt, wt, hist)
    torch.cuda.synchronize()
    for k in ("status", "iters"):
        np.testing.assert_array_equal(hist[k].cpu().numpy(), torch.stack(ref[k]).cpu().numpy(), err_msg=k)
    for k in ("u", "x", "f"):
        a, b_ = hist[k].cpu().numpy(), torch.stack(ref[k]).cpu().numpy()
        assert _rel(a, b_) <= 1e-12, (k, _rel(a, b_))
    assert _rel(p2.cpu().numpy(), p1.cpu().numpy()) <= 1e-12
    assert _rel(w2.cpu().numpy(), w1.cpu().numpy()) <= 1e-12


def test_closed_loop_dispatch_order_does_not_change_results():
    """nmpc_closed_loop_dev with a dispatch order (schedule.longest_first of the
    previous launch's iterations, then a random permutation) gives bitwise the
    results of index-order dispatch; entries outside [0,B) are skipped."""
    import torch
    from nmpc_amd import make_spec
    from nmpc_amd.schedule import longest_first

    spec = make_spec("race_track_2", N=20, T=0.2)
    B, K = 80, 3
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 1003)
    f64 = dict(dtype=torch.float64, device="cuda")
    s = _solver(spec)

    def run(order, validate=True):
        p = torch.tensor(P, **f64)
        w = torch.zeros(B, spec.nw, **f64)
        hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
                "status": torch.full((K, B), 99, dtype=torch.int32, device="cuda"),
                "iters": torch.full((K, B), -1, dtype=torch.int32, device="cuda")}
        s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, order=order, check=validate, _validate_order=validate)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in hist.items()}, p.cpu().numpy(), w.cpu().numpy()

    ref, p_ref, w_ref = run(None)
    g = torch.Generator().manual_seed(5)
    for order in (longest_first(torch.tensor(ref["iters"], device="cuda")),
                  torch.randperm(B, generator=g).to(torch.int32).cuda()):
        got, p_got, w_got = run(order)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        np.testing.assert_array_equal(p_got, p_ref)
        np.testing.assert_array_equal(w_got, w_ref)
    # out-of-range entries (not a permutation: nlpsol refuses it; here handed to the device
    # directly): those workgroups do nothing, the named scenarios still run, and the
    # completion guard marks the two scenarios left unrun and reports the launch
    from nmpc_amd.nlpsol import NOT_RUN
    bad = torch.arange(B, dtype=torch.int32, device="cuda")
    bad[1] = B + 7
    bad[2] = -3
    with pytest.raises(ValueError, match="permutation"):
        run(bad)
    got, _, _ = run(bad, validate=False)
    assert (got["iters"][:, 1:3] == NOT_RUN).all() and (got["status"][:, 1:3] == NOT_RUN).all()
    np.testing.assert_array_equal(got["iters"][:, 3:], ref["iters"][:, 3:])
    info = s.closed_loop_info()
    assert info["scheduler_error"] & 2 and info["steps_done"] == (B - 2) * K


def test_closed_loop_step_queues_match_per_scenario_dispatch():
    """More scenarios than resident waves: nmpc_closed_loop_dev runs the step-queue
    scheduler (persistent waves claim (scenario, step) pairs, lowest step first, each
    scenario pinned to one XCD).  Results are bitwise those of one workgroup per
    scenario (NMPC_CLOSED_LOOP=static), with and without a dispatch order, and no wave
    reports a scheduler wait error."""
    import torch
    from nmpc_amd import make_spec

    spec = make_spec("race_track_2", N=20, T=0.2)
    s = _solver(spec)
    f64 = dict(dtype=torch.float64, device="cuda")
    K = 3
    # learn the resident-wave count with a small launch, then exceed it
    P0, bnd, vt0, wt0 = _closed_loop_inputs(spec, 8, 5)
    s.closed_loop_device(1, *bnd, torch.tensor(P0, **f64), torch.zeros(8, spec.nw, **f64), vt0, wt0)
    torch.cuda.synchronize()
    res = s.closed_loop_info()["resident_waves"]
    assert res >= 8
    B = res + 173
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 1003)

    def run(order=None):
        p = torch.tensor(P, **f64)
        w = torch.zeros(B, spec.nw, **f64)
        hist = {"u": torch.empty(K, B, 6, **f64), "x": torch.empty(K, B, 8, **f64), "f": torch.empty(K, B, **f64),
                "fov": torch.empty(K, B, **f64),
                "status": torch.full((K, B), 99, dtype=torch.int32, device="cuda"),
                "iters": torch.full((K, B), -1, dtype=torch.int32, device="cuda")}
        s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, order=order)
        torch.cuda.synchronize()
        return {k: v.cpu().numpy() for k, v in hist.items()}, p.cpu().numpy(), w.cpu().numpy()

    os.environ["NMPC_CLOSED_LOOP"] = "static"
    try:
        ref, p_ref, w_ref = run()
        assert s.closed_loop_info()["policy"] == "per_scenario"
    finally:
        del os.environ["NMPC_CLOSED_LOOP"]
    g = torch.Generator().manual_seed(9)
    for order in (None, torch.randperm(B, generator=g).to(torch.int32).cuda()):
        got, p_got, w_got = run(order)
        info = s.closed_loop_info()
        assert info["policy"] == "step_queues" and info["scheduler_error"] == 0, info
        assert info["steps_done"] == B * K and info["launched_waves"] == res, info
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        np.testing.assert_array_equal(p_got, p_ref)
        np.testing.assert_array_equal(w_got, w_ref)


def test_closed_loop_parity_with_oracle_loop():
    """The fused closed loop against the oracle's own solve + shift_timestep loop
    (Python/NMPC_TT.py:348-402 restated) under a target schedule that changes
    mid-run (Python/10_obstacles.py:28-31, iterations 298..300): same statuses,
    applied controls, states and FOV-centre errors (:397-400,433-437)."""
    import torch
    from nmpc_amd import make_spec
    from nmpc_amd.targets import schedule

    spec = make_spec("race_track_2", N=10, T=0.2)
    B, K = 3, 3
    P, bnd, _, _ = _closed_loop_inputs(spec, B, 21)
    f64 = dict(dtype=torch.float64, device="cuda")
    vs, ws = schedule("10_obstacles", 298, K)
    assert ws[1] == 0.0 and ws[2] != 0.0
    vt, wt = torch.tensor(vs, **f64).reshape(K, 1), torch.tensor(ws, **f64).reshape(K, 1)
    s = _solver(spec)
    p = torch.tensor(P, **f64)
    w = torch.zeros(B, spec.nw, **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "x": torch.empty(K, B, 8, **f64),
            "fov": torch.empty(K, B, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p, w, vt, wt, hist)
    torch.cuda.synchronize()
    prob, ref = _oracle("race_track_2", 10, 0.2)
    lbx, ubx, lbg, ubg = spec.bounds()
    for b in range(B):
        x0, xs, u0 = P[b, :8].copy(), P[b, 8:11].copy(), np.zeros(spec.nw)
        for k in range(K):
            np.testing.assert_allclose(hist["x"][k, b].cpu().numpy(), x0, rtol=1e-9, atol=1e-9)
            r = ref.solve(u0, lbx, ubx, lbg, ubg, np.concatenate([x0, xs]))
            assert int(hist["status"][k, b]) == r["status"], (b, k)
            if r["status"] != 0:
                break
            assert _rel(hist["u"][k, b].cpu().numpy(), r["x"][:6]) <= TOL
            x1, u1, xs1 = orc.shift_timestep(prob, x0, r["x"].reshape(spec.N, 6).T, xs, con_t=(vs[k], ws[k]))
            xe, ye = orc.fov_centre(x1)
            fov = np.hypot(xe - xs[0], ye - xs[1])
            assert abs(float(hist["fov"][k, b]) - fov) <= 1e-6 * (1 + fov), (b, k)
            x0, u0, xs = x1, u1.T.ravel(), xs1


def test_restoration_phase_against_oracle():
    """Solves whose filter line search fails (captured from the config-3 closed
    loop; tests/golden/gen_resto_cases.py) go through the feasibility restoration
    phase.  Checked against the oracle: identical main iterations up to the
    failure, restoration entered at the same iteration with the same restoration
    barrier parameter mu_R = max(mu, |d - s|_inf) and a matching first restoration
    step.  Past that point restoration compares theta values near rounding level
    (it starts feasible for its own constraints), so outcomes are only required to
    be valid terminal states; agreement of the final status is reported."""
    from nmpc_amd import make_spec

    G = np.load(os.path.join(GOLD, "resto_cases.npz"))
    B = G["w"].shape[0]
    spec = make_spec("race_track_2", N=20, T=0.2)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    s.set_trace(True)
    s(x0=G["w"].T, lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=G["p"].T)
    st = s.stats()["status_code"]
    tr = s.read_trace(B)
    agree = 0
    for b in range(B):
        fr = int(G["first_resto"][b])
        ref = G["trace"][b]
        assert fr > 1, "fixture without a restoration phase"
        for i in range(fr - 1):  # main iterations before restoration
            assert tr[b, i, 7] >= 0
            assert abs(tr[b, i, 3] - ref[i, 2]) <= 1e-7 * (1 + abs(ref[i, 2])), (b, i, tr[b, i, 3], ref[i, 2])
            assert abs(tr[b, i, 5] - ref[i, 3]) <= 1e-6 * (1 + abs(ref[i, 3])), (b, i)
        i = fr - 1  # first restoration iteration
        assert tr[b, i, 7] < 0, (b, "GPU did not enter restoration at the oracle's iteration")
        assert abs(tr[b, i, 1] - ref[i, 1]) <= 1e-9 * ref[i, 1], (b, tr[b, i, 1], ref[i, 1])
        # theta_R is a residual of O(theta) quantities: rounding-level differences
        # relative to the last main-iteration theta
        th_main = ref[fr - 2, 2]
        assert abs(tr[b, i, 3] - ref[i, 2]) <= 1e-2 * abs(ref[i, 2]) + 1e-10 * (1 + th_main), (b, tr[b, i, 3], ref[i, 2])
        assert int(st[b]) in (0, 1, 2, -1, -2), int(st[b])
        agree += int(st[b]) == int(G["status"][b])
    print(f"restoration cases: final status agrees with the oracle on {agree}/{B}")
    assert agree >= B - 1  # 15/16 at the last run: one case decided at rounding level (docstring)


def test_weights_from_p_match_oracle_and_constant_solver():
    """Batched weight sweep (the RL replay rebuilds nlpsol per
    (w1, w2), MATLAB/Race Track 1/MPC.m:1,127): weights read from p per scenario."""
    from nmpc_amd import make_spec, draw_scenarios

    spec_w = make_spec("race_track_2", N=10, T=0.2, weights_in_p=True)
    spec_c = make_spec("race_track_2", N=10, T=0.2)
    B = 4
    P = draw_scenarios(spec_c, B, seed=31)
    W = np.array([[1.0, 2.0], [0.5, 3.0], [2.0, 0.5], [1.0, 2.0]])
    Pw = np.hstack([P, W])
    lbx, ubx, lbg, ubg = spec_c.bounds()
    sw = _solver(spec_w)
    sol_w = sw(x0=np.zeros(spec_w.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=Pw.T)
    sc = _solver(spec_c)
    sol_c = sc(x0=np.zeros(spec_c.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    # weight pair (1, 2) is the reference's constant setting (Python/NMPC_TT.py:204-205)
    for b in (0, 3):
        np.testing.assert_array_equal(sol_w["x"][:, b], sol_c["x"][:, b])
    prob = orc.make_problem("race_track_2", N=10, T=0.2)
    prob.w1_pidx, prob.w2_pidx, prob.np_ = 11, 12, 13
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    st = sw.stats()["status_code"]
    for b in (1, 2):
        r = ref.solve(np.zeros(spec_w.nw), lbx, ubx, lbg, ubg, Pw[b])
        assert int(st[b]) == r["status"]
        if r["status"] == 0:
            assert _rel(sol_w["x"][:, b], r["x"]) <= TOL
            assert abs(sol_w["f"][0, b] - r["f"]) <= TOL * (1 + abs(r["f"]))


def test_closed_loop_moving_obstacles_match_oracle_loop():
    """Device closed loop with the dynamic-obstacle parameter schedule of
    MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:211-230 (obstacle 2
    starts moving after iteration 100) against the oracle's loop."""
    import torch
    from nmpc_amd import make_spec
    from nmpc_amd.targets import obstacle_steps

    spec = make_spec("dynamic", N=10, T=0.2, dynamic=True)
    B, K, it0 = 3, 3, 100
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 41)
    f64 = dict(dtype=torch.float64, device="cuda")
    dp = obstacle_steps(it0, K, spec.np)
    assert dp[0].sum() == 0 and dp[1, 12] == -1.0  # window opens after iteration 100
    s = _solver(spec)
    p = torch.tensor(P, **f64)
    w = torch.zeros(B, spec.nw, **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, p_step=torch.tensor(dp, **f64))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(p[:, 11:].cpu().numpy(), P[:, 11:] + dp.sum(0)[11:])
    prob, ref = _oracle("dynamic", 10, 0.2, dynamic=True)
    lbx, ubx, lbg, ubg = spec.bounds()
    for b in range(B):
        pk, u0 = P[b].copy(), np.zeros(spec.nw)
        for k in range(K):
            r = ref.solve(u0, lbx, ubx, lbg, ubg, pk)
            assert int(hist["status"][k, b]) == r["status"], (b, k)
            if r["status"] != 0:
                break
            assert _rel(hist["u"][k, b].cpu().numpy(), r["x"][:6]) <= TOL
            x1, u1, xs1 = orc.shift_timestep(prob, pk[:8], r["x"].reshape(spec.N, 6).T, pk[8:11])
            pk = np.concatenate([x1, xs1, pk[11:] + dp[k, 11:]])
            u0 = u1.T.ravel()


@pytest.mark.parametrize("layout,N,seed", [(None, 10, 1001), ("10_obstacles", 15, 77)])
def test_no_gimbal_model_parity(layout, N, seed):
    """No-gimbal variant (MATLAB/Dynamic Obstacles/NMPC_TT.m) run on the
    gimbal kernel with the gimbal controls/states absent, against the oracle's
    dense IPOPT on the true 3N-variable problem."""
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec(layout, N=N, T=0.2, model="uav5")
    assert (spec.nw, spec.m, spec.np) == (3 * N, 2 + spec.n_obs, 8)
    B = 4
    P = draw_scenarios(spec, B, seed=seed)
    lbx, ubx, lbg, ubg = spec.bounds()
    s = _solver(spec)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    assert sol["x"].shape == (3 * N, B) and sol["X"].shape == (5 * (N + 1), B)
    st, its = s.stats()["status_code"], s.stats()["iter_count"]
    prob = orc.make_problem(layout, N=N, T=0.2, model="uav5")
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    for b in range(B):
        r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b])
        assert int(st[b]) == r["status"], (b, st[b], r["status"])
        assert abs(int(its[b]) - r["iter"]) <= 2
        if r["status"] == 0:
            assert _rel(sol["x"][:, b], r["x"]) <= TOL
            assert _rel(sol["X"][:, b], r["X"].T.ravel()) <= TOL
            assert abs(sol["f"][0, b] - r["f"]) <= TOL * (1 + abs(r["f"]))


def test_no_gimbal_shift_matches_oracle():
    """nmpc_shift_dev on the no-gimbal model: MATLAB/Dynamic Obstacles/shift1.m
    (x0 <- x0 + T f5(x0, u0), u shifted by one stage of 3 controls, target
    unicycle step with con_t = [15; 0.12]) against the oracle's shift_timestep."""
    import torch
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec(None, N=10, T=0.2, model="uav5")
    prob = orc.make_problem(None, N=10, T=0.2, model="uav5")
    B = 5
    rng = np.random.default_rng(3)
    P = draw_scenarios(spec, B, seed=11)
    lbx, ubx, _, _ = spec.bounds()
    U = lbx + (ubx - lbx) * rng.random((B, spec.nw))
    f64 = dict(dtype=torch.float64, device="cuda")
    p, u = torch.tensor(P, **f64), torch.tensor(U, **f64)
    w = torch.zeros(B, spec.nw, **f64)
    s = _solver(spec)
    s.shift_device(p, u, w, torch.full((B,), 15.0, **f64), torch.full((B,), 0.12, **f64))
    torch.cuda.synchronize()
    for b in range(B):
        x1, u1, xs1 = orc.shift_timestep(prob, P[b, :5], U[b].reshape(10, 3).T, P[b, 5:8], con_t=(15.0, 0.12))
        assert _rel(p[b, :5].cpu().numpy(), x1) <= 1e-14
        assert _rel(p[b, 5:8].cpu().numpy(), xs1) <= 1e-14
        np.testing.assert_array_equal(w[b].cpu().numpy(), u1.T.ravel())


def test_no_gimbal_closed_loop_matches_oracle_loop():
    """The fused closed loop on the no-gimbal model (MATLAB/Dynamic Obstacles/NMPC_TT.m
    main loop :150-183 with shift1.m) against the oracle's solve + shift loop on the
    true 3N-variable problem: statuses, applied controls, states and the FOV-centre
    error, which without gimbal angles is the UAV-target ground distance."""
    import torch
    from nmpc_amd import make_spec

    N, B, K = 10, 3, 3
    spec = make_spec(None, N=N, T=0.2, model="uav5")
    P, bnd, _, _ = _closed_loop_inputs(spec, B, 1001)
    f64 = dict(dtype=torch.float64, device="cuda")
    vt, wt = torch.full((B,), 15.0, **f64), torch.full((B,), 0.12, **f64)
    s = _solver(spec)
    p = torch.tensor(P, **f64)
    w = torch.zeros(B, spec.nw, **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "x": torch.empty(K, B, 8, **f64),
            "fov": torch.empty(K, B, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p, w, vt, wt, hist)
    torch.cuda.synchronize()
    prob = orc.make_problem(None, N=N, T=0.2, model="uav5")
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    lbx, ubx, lbg, ubg = spec.bounds()
    H = {k: v.cpu().numpy() for k, v in hist.items()}
    checked = 0
    for b in range(B):
        x0, xs, u0 = P[b, :5].copy(), P[b, 5:8].copy(), np.zeros(spec.nw)
        for k in range(K):
            np.testing.assert_allclose(H["x"][k, b, :5], x0, rtol=1e-9, atol=1e-9)
            assert (H["x"][k, b, 5:] == 0).all() and (H["u"][k, b, 3:] == 0).all()
            r = ref.solve(u0, lbx, ubx, lbg, ubg, np.concatenate([x0, xs]))
            assert int(H["status"][k, b]) == r["status"], (b, k)
            if r["status"] != 0:
                break
            assert _rel(H["u"][k, b, :3], r["x"][:3]) <= TOL
            x1, u1, xs1 = orc.shift_timestep(prob, x0, r["x"].reshape(N, 3).T, xs, con_t=(15.0, 0.12))
            d = np.hypot(x1[0] - xs[0], x1[1] - xs[1])
            assert abs(H["fov"][k, b] - d) <= 1e-6 * (1 + d), (b, k, H["fov"][k, b], d)
            x0, u0, xs = x1, u1.T.ravel(), xs1
            checked += 1
    assert checked >= B




def test_no_gimbal_closed_loop_per_scenario_bounds():
    """Per-scenario (B, 3N) bounds for the no-gimbal model's closed loop (the caller
    layout's stride is 3N): accepted, and bitwise equal to the shared-bound run."""
    import torch
    from nmpc_amd import make_spec

    N, B, K = 10, 4, 2
    spec = make_spec(None, N=N, T=0.2, model="uav5")
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 1001)
    f64 = dict(dtype=torch.float64, device="cuda")
    s = _solver(spec)
    outs = []
    for per in (False, True):
        b = [t.expand(B, -1).contiguous() if per else t for t in bnd]
        p = torch.tensor(P, **f64)
        w = torch.zeros(B, spec.nw, **f64)
        hist = {"u": torch.empty(K, B, 6, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
        s.closed_loop_device(K, *b, p, w, vt, wt, hist)
        outs.append({k: v.cpu().numpy() for k, v in hist.items()} | {"w": w.cpu().numpy()})
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_step_queue_guard_reports_unrun_scenarios():
    """If the XCD sets were not all served (a partitioned device, a CU-masked stream),
    the step queues would leave scenarios unrun.  NMPC_SCHED_TEST_ONE_SET forces that
    (only the waves on XCD 0 run, so sets 1..7 have no wave): the launch must raise,
    never return garbage, and
    the unrun steps carry NMPC_STATUS_NOT_RUN and NaN in the histories."""
    import torch
    from nmpc_amd import make_spec
    from nmpc_amd._lib import NmpcError
    from nmpc_amd.nlpsol import NOT_RUN

    spec = make_spec("race_track_2", N=6, T=0.2)
    s = _solver(spec)
    f64 = dict(dtype=torch.float64, device="cuda")
    P0, bnd, vt0, wt0 = _closed_loop_inputs(spec, 8, 5)
    s.closed_loop_device(1, *bnd, torch.tensor(P0, **f64), torch.zeros(8, spec.nw, **f64), vt0, wt0)
    B, K = s.closed_loop_info()["resident_waves"] + 64, 2
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 11)
    hist = {"u": torch.zeros(K, B, 6, **f64), "f": torch.zeros(K, B, **f64), "x": torch.zeros(K, B, 8, **f64),
            "fov": torch.zeros(K, B, **f64), "iters": torch.full((K, B), 99, dtype=torch.int32, device="cuda"),
            "status": torch.full((K, B), 99, dtype=torch.int32, device="cuda")}
    os.environ["NMPC_SCHED_TEST_ONE_SET"] = "1"
    try:
        with pytest.raises(NmpcError, match="closed loop incomplete"):
            s.closed_loop_device(K, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64), vt, wt, hist)
    finally:
        del os.environ["NMPC_SCHED_TEST_ONE_SET"]
    info = s.closed_loop_info()
    assert info["policy"] == "step_queues" and info["scheduler_error"] & 2
    st = hist["status"].cpu().numpy()
    pos = np.arange(B)  # dispatch position = scenario index (no order): set = position mod 8
    assert np.all(st[:, pos % 8 != 0] == NOT_RUN)
    assert np.all(st[:, pos % 8 == 0] != NOT_RUN) and np.all(st != 99)
    assert np.isnan(hist["f"].cpu().numpy()[:, pos % 8 != 0]).all()
    # every history of an unrun step is marked, none is left uninitialised
    assert np.isnan(hist["fov"].cpu().numpy()[:, pos % 8 != 0]).all()
    assert np.isnan(hist["x"].cpu().numpy()[:, pos % 8 != 0]).all()
    assert np.isnan(hist["u"].cpu().numpy()[:, pos % 8 != 0]).all()
    assert np.all(hist["iters"].cpu().numpy()[:, pos % 8 != 0] == NOT_RUN)
    assert info["steps_done"] == K * int((pos % 8 == 0).sum())


@pytest.mark.parametrize("policy", ["step_queues", "per_scenario"])
def test_closed_loop_check_on_a_side_stream(policy):
    """check=True on a non-blocking torch stream: nmpc_closed_loop_info synchronises the
    launch's own stream before reading the completion flags, so the check sees this
    launch (not the previous one) under both policies; the one-workgroup-per-scenario
    policy is counted by the same check kernel."""
    import torch
    from nmpc_amd import make_spec

    spec = make_spec("race_track_2", N=6, T=0.2)
    s = _solver(spec)
    f64 = dict(dtype=torch.float64, device="cuda")
    P0, bnd, vt0, wt0 = _closed_loop_inputs(spec, 8, 5)
    s.closed_loop_device(1, *bnd, torch.tensor(P0, **f64), torch.zeros(8, spec.nw, **f64), vt0, wt0)
    B = s.closed_loop_info()["resident_waves"] + 64 if policy == "step_queues" else 96
    K = 3
    P, bnd, vt, wt = _closed_loop_inputs(spec, B, 21)
    res = []
    for use_side in (False, True):
        hist = {"status": torch.full((K, B), 99, dtype=torch.int32, device="cuda")}
        p, w = torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64)
        torch.cuda.synchronize()
        if use_side:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, stream=st, check=True)
            st.synchronize()
        else:
            s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, check=True)
        info = s.closed_loop_info()
        assert info["policy"] == policy and info["steps_done"] == B * K and info["scheduler_error"] == 0
        res.append(hist["status"].cpu().numpy())
    np.testing.assert_array_equal(res[0], res[1])
    with pytest.raises(ValueError, match="permutation"):
        order = torch.zeros(B, dtype=torch.int32, device="cuda")  # every entry the same scenario
        s.closed_loop_device(K, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64), vt, wt, order=order)


@pytest.mark.parametrize("layout,N,dyn,model,weights", [("race_track_2", 12, False, "uav8g", False),
                                                         ("dynamic", 10, True, "uav8g", False),
                                                         ("race_track_2", 10, False, "uav8g", True),
                                                         ("10_obstacles", 8, False, "uav5", False)])
def test_lam_p_matches_oracle_finite_differences(layout, N, dyn, model, weights):
    """lam_p = -grad_p (f + lam_g' g) at the returned x (CasADi nlpsol's output; the
    reference never reads it): x0 through the adjoint of the rollout, the target through
    the stage costs, moving-obstacle coordinates and cost weights taken from p --
    against central differences of the oracle's objective / constraints at the GPU's
    own (x, lam_g).  Parity unpinned against CasADi itself (not installed); the sign
    follows CasADi's convention grad f + J_g' lam_g + lam_x = 0 extended to p."""
    from nmpc_amd import make_spec, draw_scenarios

    spec = make_spec(layout, N=N, T=0.2, dynamic=dyn, model=model, weights_in_p=weights)
    P = draw_scenarios(make_spec(layout, N=N, T=0.2, dynamic=dyn, model=model), 4, seed=21)
    prob = orc.make_problem(layout, N=N, T=0.2, dynamic=dyn, model=model)
    if weights:
        P = np.hstack([P, np.array([[1.0, 2.0], [0.5, 3.0], [2.0, 0.5], [1.5, 1.0]])])
        prob.w1_pidx, prob.w2_pidx, prob.np_ = P.shape[1] - 2, P.shape[1] - 1, P.shape[1]
    s = _solver(spec)
    lbx, ubx, lbg, ubg = spec.bounds()
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    st = s.stats()["status_code"]
    checked = 0
    for b in range(4):
        if st[b] not in (0, 1):
            continue
        ref = orc.lam_p(prob, sol["x"][:, b], P[b], sol["lam_g"][:, b])
        got = sol["lam_p"][:, b]
        scale = 1.0 + np.abs(ref).max()
        assert np.all(np.abs(got - ref) <= 1e-5 * scale), (b, got, ref)
        checked += 1
    assert checked >= 2


def _fixed_cases(lbx, ubx, N, nu, seed=5):
    """bound sets with fixed decision variables (lbx == ubx): the gimbal rates held at 0
    on every stage, the speed held at 20 on the first three stages, 8 random variables
    held at random interior values"""
    rng = np.random.default_rng(seed)
    cases = []
    if nu == 6:
        l1, u1 = lbx.copy(), ubx.copy()
        for k in range(N):
            for c in (3, 4, 5):
                l1[nu * k + c] = u1[nu * k + c] = 0.0
        cases.append(("gimbal rates fixed", l1, u1))
    l2, u2 = lbx.copy(), ubx.copy()
    for k in range(3):
        l2[nu * k] = u2[nu * k] = 20.0
    cases.append(("speed fixed", l2, u2))
    l3, u3 = lbx.copy(), ubx.copy()
    idx = rng.choice(len(lbx), 8, replace=False)
    l3[idx] = u3[idx] = lbx[idx] + rng.uniform(0.2, 0.8, 8) * (ubx[idx] - lbx[idx])
    cases.append(("random fixed", l3, u3))
    return cases


@pytest.mark.parametrize("model", ["uav8g", "uav5"])
def test_fixed_variables_make_parameter_match_oracle(model):
    """lbx == ubx (IPOPT's default fixed_variable_treatment = make_parameter: the variable
    leaves the NLP -- held at the bound, no step, no bound multipliers, out of the scaling
    and the error norms -- and its lam_x is 0, IPOPT 3.12 as bundled by CasADi 3.5.5),
    against the oracle's dense restatement of the same treatment."""
    from nmpc_amd import make_spec, draw_scenarios

    N = 10
    spec = make_spec("race_track_2", N=N, T=0.2, model=model)
    prob = orc.make_problem("race_track_2", N=N, T=0.2, model=model)
    B = 6
    P = draw_scenarios(spec, B, seed=77)
    lbx, ubx, lbg, ubg = spec.bounds()
    ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    s = _solver(spec)
    for name, lo, hi in _fixed_cases(lbx, ubx, N, spec.nu):
        sol = s(x0=np.zeros(spec.nw), lbx=lo, ubx=hi, lbg=lbg, ubg=ubg, p=P.T)
        st, its = s.stats()["status_code"], s.stats()["iter_count"]
        fx = lo == hi
        for b in range(B):
            r = ref.solve(np.zeros(spec.nw), lo, hi, lbg, ubg, P[b])
            assert int(st[b]) == r["status"], (name, b, st[b], r["status"])
            assert abs(int(its[b]) - r["iter"]) <= 1, (name, b, its[b], r["iter"])
            assert np.all(sol["x"][fx, b] == lo[fx]) and np.all(sol["lam_x"][fx, b] == 0.0)
            if r["status"] in (0, 1):
                assert _rel(sol["x"][:, b], r["x"]) <= TOL, name
                assert abs(sol["f"][0, b] - r["f"]) <= TOL * (1 + abs(r["f"]))
                assert _rel(sol["lam_x"][:, b], r["lam_x"]) <= 1e-5, name
        print(f"{model} {name}: statuses {dict(zip(*np.unique(st, return_counts=True)))}, "
              f"iterations {its.tolist()}")
