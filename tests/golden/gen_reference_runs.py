"""Reference-run fixtures: the reference scripts' OWN closed loops, restated literally
and driven through the oracle (test infrastructure only).

Every parity case elsewhere draws synthetic scenarios; these are the three runs the
reference itself performs, with the inputs its scripts hard-code:

  nmpc_tt       Python/NMPC_TT.py: x0 = [90,150,80,0,0,0,0,0] (:321), target
                (100,150,0) (:316-318), T = 1, N = 15 (:57-58), 3 obstacles r = 30
                (:224-231), target controls con_t = (12, 0.01) (:25), 700 steps (:339)
  10_obstacles  Python/10_obstacles.py: x0 = [99,150,80,0,...] (:376), T = 0.2 (:95),
                N = 15, 10 obstacle rows (3 active, r = 100, :247-269), the
                mpc_iter-keyed turn schedule (:28-60), 1,595 steps (:388)
  race_track_2  Python/Race Track 2.py: x0 = [99,150,80,0,...] (:356), T = 0.2,
                N = 15, all 10 obstacles active (r = 50, :223-244), schedule
                (:28-36), 2,000 steps (:363)

Each step is the reference loop body (NMPC_TT.py:348-402): p = [x0; xs] (:350-353),
warm start vec(u0) (:355-356), solve (:358-365) with the script's own bound vectors
(:269-306, the literal N = 15 strides), u = reshape(x, 6, N) (:367), then
shift_timestep (:13-30) with the script's con_t for the current mpc_iter.  The FOV
error of step i is |FOV centre of x0 after step i - target before step i|
(:399-402, :433-435), and the run's printed result is its sum (:438-440).

Recorded per step: p (the solver's parameter input; the warm start is the shift of
the previous step's x, reconstructed exactly by the test), status, iterations,
x, f, and the FOV error; plus the run's FOV-error sum.

Round 4 adds the two MATLAB runs that define BASELINE configs 1 and 5:

  matlab_nmpc_tt     MATLAB/Dynamic Obstacles/NMPC_TT.m (no gimbal): x0 = [90,150,80,0,0],
                     xs = [100,150,0] (:139-140), T = 0.2, N = 15 (:10-11),
                     sim_time/T = 100 steps (:144,156), literal lbg(1:2:32) / lbx(1:3:3N-1)
                     (:129-134), target con_t = [15; 0.12] (shift1.m:9).  The script
                     prints nothing; its plotted result is the UAV-target ground track
                     (:193), so the per-step "fov" here is |(x, y) of x0 after step i -
                     target before step i| (a camera without gimbal angles looks straight
                     down, the kernel's convention for this model).
  dynamic_obstacles  MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m (gimbal model):
                     x0 = [-501,150,80,0,...], xs = [-500,150,0] (:183-184), T = 0.2,
                     N = 15 (:10-11), loop_run = 1,500 steps (:199), literal
                     lbg(1,r:15:240) / lbx(c:6:6N) (:156-178), p = [x0; xs; y_o_1..6]
                     (:211) with the y_o windows applied AFTER args.p is formed (:213-230,
                     nmpc_amd.targets.DYNAMIC_OBSTACLE_WINDOWS), printed result
                     sum(error) (:264-267,325) with error(i) = |FOV(x0 after step i) -
                     target before step i| (:257-260, ss(:,i)).
                     The call at :251 is shift1(T, t0, x0, u, f_u, xs, sc): seven
                     arguments against shift1.m:1's (T, t0, x0, u, f_u, f_t, xs), so inside
                     shift1 the target would be the counter sc and xs(3) would fail -- the
                     script does not run against the committed shift1.m.  Reading taken:
                     the committed shift1.m body on the target state, i.e. the unicycle
                     step with con_t = [15; 0.12] (shift1.m:8-12) every step; sc (the step
                     counter) selects nothing.

Round 5 adds one DERIVED run (not a run the reference performs):

  dynamic_obstacles_derived  Dynamic Obstacle avoidance.m with everything the script fixes
                     kept -- its obstacle table (:98-119), the y_o windows (:213-230), its
                     literal bounds (:156-178), T, N and con_t = [15; 0.12] (shift1.m:9) --
                     except the start: the UAV at (-61, 150, 80) and the target at
                     (-60, 150), heading +x, inside the obstacle corridor, 600 steps.  The
                     target then circles (radius 15 / 0.12 = 125 m) around (-60, 275), a path
                     that passes within ~60 m of obstacle 2 at x = 0 while that obstacle's y
                     moves from 300 to 1 (steps 101..399), so its moving row is active: the
                     script's own start at x = -501 never comes within 370 m of a moving
                     obstacle, which leaves the moving rows unexercised.  Labelled derived.

Solvers (`--solver`):
  numpy  oracle/nmpc_oracle.py IpoptDense (dense single-shooting IPOPT
         restatement) -- the committed fixtures (ref_run_<name>.npz);
  cpp    oracle/cpu_ipopt.cpp (compiled restatement with the Riccati step),
         written to ref_run_<name>_cpp.npz for cross-checks, not committed;
  numpy1 / numpy2 / numpy3  the numpy oracle with la_variant 1..3 (the same Newton
         steps factored in a permuted variable order: differs from `numpy` by rounding
         alone), written to ref_run_<name>_numpy<v>.npz, not committed.
The committed whole-run summary of the non-fixture solvers is made by
gen_rounding_spread.py (ref_run_<name>_spread.npz).

    python tests/golden/gen_reference_runs.py [<run>|all] [--solver numpy|cpp|numpy1|numpy2|numpy3]
"""
import argparse
import math
import multiprocessing as mp
import os
import sys
import time
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))

X0_NMPC_TT = [90.0, 150.0, 80.0, 0.0, 0.0, 0.0, 0.0, 0.0]   # Python/NMPC_TT.py:321
X0_10_OBS = [99.0, 150.0, 80.0, 0.0, 0.0, 0.0, 0.0, 0.0]    # Python/10_obstacles.py:376, Race Track 2.py:356
XS0 = [100.0, 150.0, 0.0]                                    # NMPC_TT.py:316-318 (same in both others)
X0_MATLAB_NG = [90.0, 150.0, 80.0, 0.0, 0.0]                 # MATLAB/Dynamic Obstacles/NMPC_TT.m:139
X0_DYNAMIC = [-501.0, 150.0, 80.0, 0.0, 0.0, 0.0, 0.0, 0.0]  # Dynamic Obstacle avoidance.m:183
XS0_DYNAMIC = [-500.0, 150.0, 0.0]                           # Dynamic Obstacle avoidance.m:184
Y_OBS0_DYNAMIC = [0.0, 300.0, 0.0, 300.0, 0.0, 300.0]        # Dynamic Obstacle avoidance.m:98-109 (y_o_1..6)
X0_DYNAMIC_DERIVED = [-61.0, 150.0, 80.0, 0.0, 0.0, 0.0, 0.0, 0.0]  # derived start, inside the corridor
XS0_DYNAMIC_DERIVED = [-60.0, 150.0, 0.0]

RUNS = {
    "nmpc_tt": dict(layout="nmpc_tt", N=15, T=1.0, x0=X0_NMPC_TT, K=700),
    "10_obstacles": dict(layout="10_obstacles", N=15, T=0.2, x0=X0_10_OBS, K=1595),
    "race_track_2": dict(layout="race_track_2", N=15, T=0.2, x0=X0_10_OBS, K=2000),
    "matlab_nmpc_tt": dict(layout=None, N=15, T=0.2, x0=X0_MATLAB_NG, K=100, model="uav5"),
    "dynamic_obstacles": dict(layout="dynamic", N=15, T=0.2, x0=X0_DYNAMIC, xs=XS0_DYNAMIC, K=1500,
                              dynamic=True),
    # derived (see the module docstring): the script's problem from a start inside the corridor
    "dynamic_obstacles_derived": dict(layout="dynamic", N=15, T=0.2, x0=X0_DYNAMIC_DERIVED,
                                      xs=XS0_DYNAMIC_DERIVED, K=600, dynamic=True, derived=True,
                                      bounds_of="dynamic_obstacles", schedule_of="dynamic_obstacles"),
}


def run_spec(name):
    """nmpc_amd ProblemSpec of a run (tests)."""
    from nmpc_amd import make_spec

    c = RUNS[name]
    return make_spec(c["layout"], N=c["N"], T=c["T"], dynamic=c.get("dynamic", False),
                     model=c.get("model", "uav8g"))


def run_problem(name):
    """oracle Problem of a run."""
    from oracle import nmpc_oracle as orc

    c = RUNS[name]
    return orc.make_problem(c["layout"], N=c["N"], T=c["T"], dynamic=c.get("dynamic", False),
                            model=c.get("model", "uav8g"))


def literal_bounds(name, N=15):
    """The scripts' own bound vectors, built with their literal slices
    (Python/NMPC_TT.py:269-306: lbg[0:128:8] ...; 10_obstacles.py / Race Track 2.py
    :314-351: lbg[0:240:15] ...; MATLAB/Dynamic Obstacles/NMPC_TT.m:129-134:
    lbg(1:2:32), lbx(1:3:3N-1) ...; Dynamic Obstacle avoidance.m:156-178: lbg(r:15:240))."""
    pi = math.pi
    if name == "matlab_nmpc_tt":
        nu = 3
        lbx, ubx = np.zeros(nu * N), np.zeros(nu * N)
        # MATLAB 1:3:3N-1 is 0-based 0:3N-1:3 (the same 15 entries as 0::3)
        for c, (lo, hi) in enumerate([(14, 30), (-pi / 30, pi / 30), (-pi / 21, pi / 21)]):
            lbx[c:nu * N:nu], ubx[c:nu * N:nu] = lo, hi
        lbg, ubg = np.zeros(32), np.zeros(32)
        lbg[0:32:2], ubg[0:32:2] = 75, 150
        lbg[1:32:2], ubg[1:32:2] = -0.2618, 0.2618
        return lbx, ubx, lbg, ubg
    nu = 6
    lbx, ubx = np.zeros(nu * N), np.zeros(nu * N)
    for c, (lo, hi) in enumerate([(14, 30), (-pi / 30, pi / 30), (-pi / 21, pi / 21),
                                  (-pi / 30, pi / 30), (-pi / 30, pi / 30), (-pi / 30, pi / 30)]):
        lbx[c:nu * N:nu], ubx[c:nu * N:nu] = lo, hi
    m, stop = (8, 128) if name == "nmpc_tt" else (15, 240)
    lbg, ubg = np.zeros(m * (N + 1)), np.zeros(m * (N + 1))
    for r, (lo, hi) in enumerate([(75, 150), (-0.2618, 0.2618), (-pi / 6, pi / 6), (-pi / 6, pi / 6),
                                  (-pi / 2, pi / 2)]):
        lbg[r:stop:m], ubg[r:stop:m] = lo, hi
    for r in range(5, m):  # obstacle rows: (-inf, 0]
        lbg[r:stop:m], ubg[r:stop:m] = -np.inf, 0.0
    return lbx, ubx, lbg, ubg


def warm_start(x_prev, N=15, nu=6):
    """u0 <- [u[:,1:], u[:,-1]] (Python/NMPC_TT.py:20-23) of the previous solution, as vec."""
    U = x_prev.reshape(N, nu)
    return np.concatenate([U[1:], U[-1:]]).ravel()


def agree_prefix(ref, x0, status, u0, f, tol=1e-6):
    """Number of leading steps over which a closed loop agrees with the oracle's run
    `ref` (a ref_run npz): the same state in (x0 within tol), the same status, and u0 and
    f within tol -- unconverged (max_iter) steps included.  Used by the GPU test and by
    gen_rounding_spread.py with the same definition."""
    nx = x0.shape[1]
    nu = u0.shape[1]
    n = 0
    for k in range(len(ref["status"])):
        xin, ou = ref["p"][k, :nx], ref["x"][k, :nu]
        ex = np.max(np.abs(x0[k] - xin) / (1 + np.abs(xin)))
        eu = np.max(np.abs(u0[k] - ou) / (1 + np.abs(ou)))
        ef = abs(f[k] - ref["f"][k]) / (1 + abs(ref["f"][k]))
        if not (ex <= tol and status[k] == ref["status"][k] and eu <= tol and ef <= tol):
            break
        n += 1
    return n


def fov_error(name, x1, xs):
    """|FOV centre of the state after a step - target before it| (NMPC_TT.py:397-400,433-435;
    Dynamic Obstacle avoidance.m:257-267); the no-gimbal run's camera looks straight down."""
    from oracle import nmpc_oracle as orc

    if RUNS[name].get("model") == "uav5":
        xe, ye = x1[0], x1[1]
    else:
        xe, ye = orc.fov_centre(x1)
    return math.sqrt((xe - xs[0]) ** 2 + (ye - xs[1]) ** 2)


def run(name, solver="numpy", K=None, log_every=100):
    warnings.simplefilter("error", RuntimeWarning)  # no silent NaN/inf arithmetic in the checker
    from threadpoolctl import threadpool_limits
    from oracle import nmpc_oracle as orc
    from nmpc_amd.targets import con_t, obstacle_steps

    threadpool_limits(1)
    c = RUNS[name]
    K = K or c["K"]
    prob = run_problem(name)
    lbx, ubx, lbg, ubg = literal_bounds(c.get("bounds_of", name), c["N"])
    if solver.startswith("numpy"):
        ipo = orc.IpoptDense(prob, orc.REFERENCE_OPTS, la_variant=int(solver[5:] or 0))

        def solve(w, p):
            r = ipo.solve(w, lbx, ubx, lbg, ubg, p)
            return r["status"], r["iter"], r["x"], r["f"]
    else:
        from oracle import cpu_ipopt

        def solve(w, p):
            r = cpu_ipopt.solve_batch(prob, w[None], p[None], lbx, ubx, lbg, ubg, orc.REFERENCE_OPTS, threads=1)
            return int(r["status"][0]), int(r["iter"][0]), r["x"][0], float(r["f"][0])
    nx, N, nu = prob.nx, c["N"], prob.nu
    x0, xs = np.array(c["x0"]), np.array(c.get("xs", XS0))
    yobs = np.array(Y_OBS0_DYNAMIC) if c.get("dynamic") else np.zeros(0)
    dobs = obstacle_steps(0, K, prob.np_) if c.get("dynamic") else None
    w = np.zeros(nu * N)   # u0 = zeros (Python/NMPC_TT.py:329; NMPC_TT.m:143)
    rec = {k: [] for k in ("p", "status", "iter", "x", "f", "fov")}
    t0 = time.time()
    for it in range(K):
        p = np.concatenate([x0, xs, yobs])   # args.p = [x0; xs (; y_o_1..6)]
        st, ni, x, f = solve(w, p)
        U = x.reshape(N, nu).T   # ca.reshape(sol['x'], nu, N)
        x1, _, xs1 = orc.shift_timestep(prob, x0, U, xs, con_t=con_t(c.get("schedule_of", name), it))
        rec["p"].append(p); rec["status"].append(st); rec["iter"].append(ni)
        rec["x"].append(x.copy()); rec["f"].append(f)
        rec["fov"].append(fov_error(name, x1, xs))
        if dobs is not None:   # obstacle windows move y_o after args.p is formed (:213-230)
            yobs = yobs + dobs[it, nx + 3:]
        x0, xs, w = x1, xs1, warm_start(x, N, nu)
        if log_every and (it + 1) % log_every == 0:
            print(f"  {name} ({solver}): {it + 1}/{K} steps, {time.time() - t0:.0f}s", flush=True)
    out = {k: np.array(v) for k, v in rec.items()}
    out.update(name=name, solver=solver, K=K, N=N, T=c["T"], fov_sum=float(np.sum(out["fov"])),
               lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg)
    return out


def generate(args):
    name, solver, K = args
    t0 = time.time()
    out = run(name, solver, K)
    suffix = "" if solver == "numpy" else f"_{solver}"
    path = os.path.join(HERE, f"ref_run_{name}{suffix}.npz")
    np.savez_compressed(path, **out)
    st = out["status"]
    print(f"{name} ({solver}): {len(st)} steps in {time.time() - t0:.0f}s; statuses "
          f"{dict(zip(*np.unique(st, return_counts=True)))}; mean iter {out['iter'].mean():.2f}; "
          f"FOV-error sum {out['fov_sum']:.6f}", flush=True)
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("run", nargs="?", default="all")
    ap.add_argument("--solver", choices=["numpy", "cpp", "numpy1", "numpy2", "numpy3"], default="numpy")
    ap.add_argument("--steps", type=int, default=0, help="override the run length (0: the script's)")
    a = ap.parse_args()
    names = list(RUNS) if a.run == "all" else [a.run]
    jobs = [(n, a.solver, a.steps or None) for n in names]
    if len(jobs) == 1:
        generate(jobs[0])
    else:
        with mp.get_context("fork").Pool(len(jobs)) as pool:
            pool.map(generate, jobs)
