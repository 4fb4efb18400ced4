"""GPU parity against the oracle's closed-loop fixtures (tests/golden/gen_closed_loop.py):
BASELINE config 1 (no-gimbal model, N=10, 32 scenarios x 10 steps), config 2 (N=20,
no obstacles, 32 x 10), config 3 (the bench's workload: N=20, 10 obstacles, 64
scenarios x 20 warm-started MPC steps) and config 5 (N=50, dynamic obstacles moving
per MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230; 16 cold solves and
16 scenarios x 10 warm-started steps).

Two comparisons per case:
  * per step: the HIP solver on exactly the (w, p) the oracle saw at every step,
    so no earlier difference propagates -- status, iteration count, and x / f at
    the north-star tolerance |a - b| <= 1e-6 (1 + |b|);
  * chained: nmpc_closed_loop_dev from the fixture's start, compared step by step
    (status, u0, f) until the two loops first disagree.
Every mismatch is printed.  The thresholds are the measured agreement of the current
kernel minus at most one scenario or step of slack, so a
regression that breaks even one scenario in a few hundred fails loudly.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-6


def _load(name):
    path = os.path.join(GOLD, f"closed_loop_{name}.npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path} (python tests/golden/gen_closed_loop.py {name})")
    return np.load(path)


def _solver(cfg):
    from nmpc_amd import nlpsol, config_spec, REFERENCE_OPTS

    spec = config_spec(cfg)
    return spec, nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)


def _relerr(a, b):
    return np.max(np.abs(a - b) / (1.0 + np.abs(b)), axis=-1)


def _per_step(name):
    z = _load(name)
    spec, s = _solver(int(z["cfg"]))
    lbx, ubx, lbg, ubg = spec.bounds()
    W = z["w"].reshape(-1, spec.nw)
    Pp = z["p"].reshape(-1, spec.np)
    sol = s(x0=W.T, lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=Pp.T)
    st, it = s.stats()["status_code"], s.stats()["iter_count"]
    ost, oit = z["status"].ravel(), z["iter"].ravel()
    ox, of = z["x"].reshape(-1, spec.nw), z["f"].ravel()
    same = st == ost
    conv = same & np.isin(ost, (0, 1))
    ex = _relerr(sol["x"].T, ox)
    ef = np.abs(sol["f"][0] - of) / (1 + np.abs(of))
    ok_x = conv & (ex <= TOL) & (ef <= TOL)
    print(f"\n{name} per step: {len(ost)} solves; status agree {same.mean():.4f}; iterations agree "
          f"{(it == oit).mean():.4f}; converged+agreeing {conv.sum()}, within 1e-6 {ok_x.sum()}; "
          f"oracle statuses {dict(zip(*np.unique(ost, return_counts=True)))}")
    for i in np.flatnonzero(~same | (conv & ~ok_x) | (it != oit)):
        print(f"  step {i}: gpu status {st[i]} it {it[i]} | oracle status {ost[i]} it {oit[i]} | "
              f"x rel err {ex[i]:.2e} f rel err {ef[i]:.2e}")
    return same, conv, ok_x, it == oit


# measured (round 2/3 kernels): statuses 318/320, 320/320, 1280/1280, 160/160; iterations
# 1277/1280 (config 3), 160/160 (config 5); every converged agreeing step within 1e-6
PER_STEP_MIN = {"config1": (318, 314), "config2": (320, 318), "config3": (1280, 1276), "config5": (160, 159)}
CHAIN_MIN = {"config1": 31, "config2": 32, "config3": 63, "config5": 14}  # identical chains (of 32/32/64/16)


@pytest.mark.parametrize("name", ["config1", "config2", "config3", "config5"])
def test_per_step_parity_with_oracle_fixture(name):
    same, conv, ok_x, same_it = _per_step(name)
    smin, imin = PER_STEP_MIN[name]
    assert same.sum() >= smin
    assert ok_x.sum() == conv.sum()
    assert same_it.sum() >= imin


def test_config5_cold_solves_match_oracle():
    """N=50 cold starts (u = 0, Python/NMPC_TT.py:329): the oracle's status mix,
    including its max-iterations share, is reproduced solve by solve."""
    z = _load("config5")
    spec, s = _solver(5)
    lbx, ubx, lbg, ubg = spec.bounds()
    n = len(z["cold_status"])
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=z["P"][:n].T)
    st, it = s.stats()["status_code"], s.stats()["iter_count"]
    print(f"\nconfig5 cold: gpu {dict(zip(*np.unique(st, return_counts=True)))} "
          f"oracle {dict(zip(*np.unique(z['cold_status'], return_counts=True)))}; "
          f"iterations agree {(it == z['cold_iter']).mean():.3f}")
    assert (st == z["cold_status"]).sum() >= 15
    conv = (st == z["cold_status"]) & np.isin(st, (0, 1))
    if conv.any():
        assert np.all(_relerr(sol["x"].T[conv], z["cold_x"][conv]) <= TOL)


@pytest.mark.parametrize("name", ["config1", "config2", "config3", "config5"])
def test_chained_closed_loop_matches_oracle_fixture(name):
    import torch

    z = _load(name)
    spec, s = _solver(int(z["cfg"]))
    B, K = z["status"].shape
    f64 = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    p = torch.tensor(z["P"], **f64)
    w = torch.zeros(B, spec.nw, **f64)
    vt, wt = torch.full((B,), float(z["vt"]), **f64), torch.full((B,), float(z["wt"]), **f64)
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda"),
            "iters": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, p, w, vt, wt, hist, p_step=torch.tensor(z["p_step"], **f64))
    torch.cuda.synchronize()
    H = {k: v.cpu().numpy() for k, v in hist.items()}
    nu = spec.nu
    matched, total, full = 0, B * K, 0
    for b in range(B):
        ok_chain = True
        for k in range(K):
            o_u = z["x"][b, k, :nu]
            g_u = H["u"][k, b, :nu]
            conv = z["status"][b, k] in (0, 1)
            ok = (H["status"][k, b] == z["status"][b, k] and
                  (not conv or (np.max(np.abs(g_u - o_u) / (1 + np.abs(o_u))) <= TOL and
                                abs(H["f"][k, b] - z["f"][b, k]) <= TOL * (1 + abs(z["f"][b, k])))))
            if not ok:
                eu = np.max(np.abs(g_u - o_u) / (1 + np.abs(o_u)))
                ef = abs(H["f"][k, b] - z["f"][b, k]) / (1 + abs(z["f"][b, k]))
                print(f"  scenario {b} diverges at step {k}: gpu status {H['status'][k, b]} it {H['iters'][k, b]}"
                      f" | oracle {z['status'][b, k]} it {z['iter'][b, k]} | u0 rel err {eu:.2e}, f rel err {ef:.2e}")
                ok_chain = False
                break
            matched += 1
        full += ok_chain
    print(f"\n{name} chained: {full}/{B} chains identical over {K} steps; {matched}/{total} steps before "
          f"the first divergence")
    # the device loop's shift (fused multiply-adds) and numpy's differ by rounding; near a
    # termination threshold that can change an iteration count and the chain from there
    # on (the per-step test above compares every step from identical inputs)
    assert full >= CHAIN_MIN[name]
    assert matched >= total - (B - CHAIN_MIN[name]) * K


def test_config3_closed_loop_at_bench_scale_matches_cpu_restatement():
    """The bench's own workload (BASELINE config 3: 4096 scenarios, seed 1003, 20
    warm-started closed-loop MPC steps from u = 0, target controls (12, 0.01)) through
    nmpc_closed_loop_dev and through the compiled CPU restatement
    (oracle/cpu_ipopt.cpp, pinned to the numpy oracle by tests/test_cpu_restatement.py),
    compared step by step until each chain first disagrees: status, and u0 / f within
    the north-star 1e-6 (1 + |ref|) for converged steps."""
    import sys
    import torch
    from nmpc_amd import config_spec, draw_scenarios

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import cpu_ipopt, nmpc_oracle as orc

    spec, s = _solver(3)
    B, K = 4096, 20
    P = draw_scenarios(spec, B, seed=1003)
    prob = orc.make_problem("race_track_2", N=spec.N, T=spec.T)
    ref = cpu_ipopt.closed_loop(prob, P, K, *orc.bounds(prob), orc.REFERENCE_OPTS, vt=12.0, wt=0.01, threads=16)
    assert np.all(ref["steps"] == K)
    f64 = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64),
                         torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64), hist)
    torch.cuda.synchronize()
    H = {k: v.cpu().numpy() for k, v in hist.items()}
    gs, rs = H["status"].T, ref["status"]
    agree = (gs == rs).mean()
    matched, full, worst = 0, 0, 0.0
    for b in range(B):
        chain = True
        for k in range(K):
            ok = gs[b, k] == rs[b, k]
            if ok and rs[b, k] in (0, 1):
                eu = np.max(np.abs(H["u"][k, b] - ref["u0"][b, k]) / (1 + np.abs(ref["u0"][b, k])))
                ef = abs(H["f"][k, b] - ref["f"][b, k]) / (1 + abs(ref["f"][b, k]))
                ok = eu <= TOL and ef <= TOL
                if ok:
                    worst = max(worst, eu, ef)
            if not ok:
                print(f"  scenario {b} parts at step {k}: gpu status {gs[b, k]} | cpu status {rs[b, k]}")
                chain = False
                break
            matched += 1
        full += chain
    print(f"\nconfig 3 at bench scale: status agreement {agree:.4f} over {B * K} steps; {full}/{B} chains "
          f"identical; {matched} steps before the first divergence; max rel err {worst:.2e}")
    # measured: agreement 0.995, 3,865-3,877 identical chains, 79,987-80,112 steps
    assert agree >= 0.994
    assert full >= 3860
    assert matched >= 79900


def test_config3_fov_error_sums_match_oracle():
    """The reference's only printed result: the run's sum of |FOV centre - target|
    (Python/NMPC_TT.py:397-400,433-440), here per scenario over the fixture's 20
    closed-loop steps -- the device loop's FOV history (nmpc_closed_loop_dev) against
    the same sum recomputed from the oracle's own trajectory (tests/golden
    closed_loop_config3), for every chain that converges at all 20 steps on both sides."""
    import sys
    import torch

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import nmpc_oracle as orc

    z = _load("config3")
    spec, s = _solver(3)
    B, K = z["status"].shape
    f64 = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    hist = {"fov": torch.empty(K, B, **f64), "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, torch.tensor(z["P"], **f64), torch.zeros(B, spec.nw, **f64),
                         torch.full((B,), float(z["vt"]), **f64), torch.full((B,), float(z["wt"]), **f64), hist)
    torch.cuda.synchronize()
    fov, st = hist["fov"].cpu().numpy(), hist["status"].cpu().numpy()
    prob = orc.make_problem("race_track_2", N=spec.N, T=spec.T)
    nx, compared, worst, tot_g, tot_o = 8, 0, 0.0, 0.0, 0.0
    for b in range(B):
        if not (np.all(st[:, b] == z["status"][b]) and np.all(np.isin(z["status"][b], (0, 1)))):
            continue  # a max-iter / infeasible step returns an unconverged u0: not comparable
        ref = 0.0
        for k in range(K):
            p = z["p"][b, k]
            x1, _, _ = orc.shift_timestep(prob, p[:nx], z["x"][b, k].reshape(spec.N, 6).T, p[nx:nx + 3],
                                          con_t=(float(z["vt"]), float(z["wt"])))
            xe, ye = orc.fov_centre(x1)
            ref += float(np.hypot(xe - p[nx], ye - p[nx + 1]))
        got = float(fov[:, b].sum())
        worst = max(worst, abs(got - ref) / (1 + abs(ref)))
        tot_g, tot_o = tot_g + got, tot_o + ref
        compared += 1
    print(f"\nFOV-error sums over {K} steps: {compared}/{B} scenarios compared; total {tot_g:.6f} (GPU) vs "
          f"{tot_o:.6f} (oracle); max per-scenario rel. difference {worst:.2e}")
    assert compared >= 54  # measured 55 / 64 (the others have a max_iter / infeasible step)
    assert worst <= 1e-6


def test_config5_closed_loop_sample_matches_cpu_restatement():
    """BASELINE config 5 at a larger sample than its fixture: 1,024 scenarios (seed
    1005) of the N=50 dynamic-obstacle problem, 5 closed-loop steps from u = 0 with the
    obstacle schedule of MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230
    from MPC iteration 195, through nmpc_closed_loop_dev and through the compiled CPU
    restatement, compared step by step until each chain first disagrees."""
    import sys
    import torch
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.targets import obstacle_steps

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import cpu_ipopt, nmpc_oracle as orc

    spec, s = _solver(5)
    B, K = 1024, 5
    P = draw_scenarios(spec, B, seed=1005)
    dp = obstacle_steps(195, K, spec.np)
    prob = orc.make_problem("dynamic", N=spec.N, T=spec.T, dynamic=True)
    ref = cpu_ipopt.closed_loop(prob, P, K, *orc.bounds(prob), orc.REFERENCE_OPTS, vt=12.0, wt=0.01, p_step=dp,
                                threads=16)
    assert np.all(ref["steps"] == K)
    f64 = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64),
                         torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64), hist,
                         p_step=torch.tensor(dp, **f64))
    torch.cuda.synchronize()
    H = {k: v.cpu().numpy() for k, v in hist.items()}
    gs, rs = H["status"].T, ref["status"]
    agree = (gs == rs).mean()
    matched, full = 0, 0
    for b in range(B):
        chain = True
        for k in range(K):
            ok = gs[b, k] == rs[b, k]
            if ok and rs[b, k] in (0, 1):
                ok = (np.max(np.abs(H["u"][k, b] - ref["u0"][b, k]) / (1 + np.abs(ref["u0"][b, k]))) <= TOL and
                      abs(H["f"][k, b] - ref["f"][b, k]) <= TOL * (1 + abs(ref["f"][b, k])))
            if not ok:
                print(f"  scenario {b} parts at step {k}: gpu status {gs[b, k]} | cpu status {rs[b, k]}")
                chain = False
                break
            matched += 1
        full += chain
    print(f"\nconfig 5 sample: status agreement {agree:.4f} over {B * K} steps (CPU statuses "
          f"{dict(zip(*np.unique(rs, return_counts=True)))}); {full}/{B} chains identical; {matched} steps "
          f"before the first divergence")
    # a max_iter step (a fifth of them here) returns an unconverged iterate, which the
    # next step starts from: chains can part at rounding level there (last run: status
    # agreement 0.9955, 885/1024 chains identical, 4682/5120 steps before divergence)
    assert agree >= 0.995
    assert full >= 880
    assert matched >= 4670
