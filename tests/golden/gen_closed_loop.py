"""Closed-loop golden fixtures: the oracle's own solve + shift loop
(Python/NMPC_TT.py:348-402 restated: solve at :358-365, shift_timestep at :13-30)
on the bench's synthetic scenarios, recorded step by step.

Each case stores, for every (scenario, step): the solver inputs the oracle saw
(warm start w and parameter vector p), and its outputs (status, iterations,
x, f).  The GPU tests (tests/test_gpu.py) use them two ways:
  * per step: the HIP solver on exactly the oracle's (w, p) inputs -- no
    propagation of an earlier difference;
  * chained: nmpc_closed_loop_dev from the same start, compared step by step
    until the two loops first take a different branch.

Cases (SURVEY 8(d) distributions via nmpc_amd.draw_scenarios):
  config1 : BASELINE config 1 (no-gimbal model of MATLAB/Dynamic Obstacles/NMPC_TT.m,
            N=10, no obstacles), seed 1001, 32 scenarios x 10 warm-started steps;
  config2 : BASELINE config 2 (N=20, no obstacles, T=0.2), seed 1002, 32 scenarios
            x 10 warm-started steps;
  config3 : BASELINE config 3 (N=20, Race Track 2 obstacles, T=0.2), seed 1003,
            the first 64 scenarios, 20 warm-started steps from u = 0, target
            controls (12, 0.01) (Python/NMPC_TT.py:25) -- the bench's workload;
  config5 : BASELINE config 5 (N=50, MATLAB dynamic-obstacle layout, obstacles
            1-6 moving), seed 1005: 16 cold solves (u = 0), then 16 scenarios x
            10 warm-started steps with the obstacle schedule of
            MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230 from
            MPC iteration 195 (obstacles 2 and 3 move).

    python tests/golden/gen_closed_loop.py [config1|config2|config3|config5|all] [--procs 8]
"""
import argparse
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

CASES = {
    "config1": dict(cfg=1, seed=1001, B=32, K=10, cold=0, it0=0),
    "config2": dict(cfg=2, seed=1002, B=32, K=10, cold=0, it0=0),
    "config3": dict(cfg=3, seed=1003, B=64, K=20, cold=0, it0=0),
    "config5": dict(cfg=5, seed=1005, B=16, K=10, cold=16, it0=195),
}


def _problem(spec):
    from oracle import nmpc_oracle as orc
    layout = None if spec.n_obs == 0 else ("dynamic" if spec.np > spec.np_min else
                                           ("race_track_2" if spec.n_obs == 10 else "nmpc_tt"))
    return orc.make_problem(layout, N=spec.N, T=spec.T, dynamic=spec.np > spec.np_min, model=spec.model)


def _chain(args):
    """One scenario's closed loop on the oracle."""
    name, b, p0, K, vt, wt, dp = args
    warnings.simplefilter("error", RuntimeWarning)  # no silent NaN/inf arithmetic in the checker
    from threadpoolctl import threadpool_limits
    from oracle import nmpc_oracle as orc
    from nmpc_amd import config_spec

    threadpool_limits(1)
    spec = config_spec(CASES[name]["cfg"])
    prob = _problem(spec)
    solver = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    nx, nu, N = prob.nx, prob.nu, prob.N
    p, w = p0.copy(), np.zeros(prob.nw)
    rows = []
    for k in range(K):
        r = solver.solve(w, lbx, ubx, lbg, ubg, p)
        rows.append(dict(w=w.copy(), p=p.copy(), status=r["status"], iter=r["iter"], x=r["x"].copy(), f=r["f"],
                         wd=sum(solver.wd_events.values())))
        x1, u1, xs1 = orc.shift_timestep(prob, p[:nx], r["x"].reshape(N, nu).T, p[nx:nx + 3], con_t=(vt, wt))
        p = np.concatenate([x1, xs1, p[nx + 3:] + dp[k, nx + 3:]])
        w = u1.T.ravel()
    return b, rows


def _cold(args):
    name, b, p0 = args
    warnings.simplefilter("error", RuntimeWarning)
    from threadpoolctl import threadpool_limits
    from oracle import nmpc_oracle as orc
    from nmpc_amd import config_spec

    threadpool_limits(1)
    prob = _problem(config_spec(CASES[name]["cfg"]))
    solver = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    r = solver.solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p0)
    return b, dict(status=r["status"], iter=r["iter"], x=r["x"], f=r["f"], wd=sum(solver.wd_events.values()))


def generate(name, procs):
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.targets import obstacle_steps

    c = CASES[name]
    spec = config_spec(c["cfg"])
    P = draw_scenarios(spec, c["B"], seed=c["seed"])
    K = c["K"]
    vt, wt = 12.0, 0.01
    dp = obstacle_steps(c["it0"], K, spec.np) if spec.np > spec.np_min else np.zeros((K, spec.np))
    t0 = time.time()
    out = dict(cfg=c["cfg"], seed=c["seed"], K=K, vt=vt, wt=wt, p_step=dp, P=P, it0=c["it0"])
    with mp.get_context("fork").Pool(procs) as pool:
        if c["cold"]:
            res = dict(pool.map(_cold, [(name, b, P[b]) for b in range(c["cold"])]))
            for key in ("status", "iter", "x", "f", "wd"):
                out["cold_" + key] = np.array([res[b][key] for b in range(c["cold"])])
        res = dict(pool.map(_chain, [(name, b, P[b], K, vt, wt, dp) for b in range(c["B"])]))
    for key in ("w", "p", "status", "iter", "x", "f", "wd"):
        out[key] = np.array([[res[b][k][key] for k in range(K)] for b in range(c["B"])])
    path = os.path.join(HERE, f"closed_loop_{name}.npz")
    np.savez_compressed(path, **out)
    st = out["status"]
    print(f"{name}: {st.size} steps in {time.time() - t0:.0f}s; statuses "
          f"{dict(zip(*np.unique(st, return_counts=True)))}; watchdog events in {int((out['wd'] > 0).sum())} solves;"
          f" mean iter {out['iter'].mean():.2f}")
    if c["cold"]:
        print(f"  cold: statuses {dict(zip(*np.unique(out['cold_status'], return_counts=True)))}, "
              f"mean iter {out['cold_iter'].mean():.1f}")
    return path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("case", nargs="?", default="all")
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    for n in (CASES if a.case == "all" else [a.case]):
        generate(n, a.procs)
