"""GPU parity on the reference scripts' OWN runs (tests/golden/gen_reference_runs.py):
Python/NMPC_TT.py (700 steps, T = 1), Python/10_obstacles.py (1,595 steps, its turn
schedule) and Python/Race Track 2.py (2,000 steps, 10 active obstacles), each with the
script's x0, target, con_t schedule and literal N = 15 bound vectors, driven through
the numpy oracle (oracle/nmpc_oracle.py IpoptDense).

Three comparisons per run:
  (a) per step: the HIP solver on exactly the oracle's (w, p) at every step of the
      run -- status, iteration count, and x / f at the north-star tolerance
      |a - b| <= 1e-6 (1 + |b|) for converged steps;
  (b) chained: nmpc_closed_loop_dev with B = 1 and K = the run's full length (the
      script's own loop on the device, its schedule as a (K, 1) target-control table),
      compared step by step with the oracle's run until the two loops first part;
  (c) the reference's printed result -- the sum of |FOV centre - target|
      (Python/NMPC_TT.py:433-440, 10_obstacles.py:534-542, Race Track 2.py:509-517)
      -- over that agreeing prefix, at 1e-6.
A closed loop of a nonconvex NLP is chaotic: two correct solvers that differ by
rounding part after some steps (the compiled CPU restatement and the numpy oracle part
at steps 8 / 102 / 111 of the three runs, tests/test_cpu_restatement.py), so (b)/(c)
are judged on the agreeing prefix and the whole-run numbers are printed beside them.
"""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
TOL = 1e-6
sys.path.insert(0, GOLD)

# measured agreement, minus at most one step of slack
PER_STEP_MIN = {  # (status agreement, iteration agreement, converged x outside 1e-6) in steps
    # measured: 699 / 685 / 11 (nmpc_tt), 1595 / 1559 / 2 (10_obstacles), 1995 / 1965 / 1 (race_track_2)
    "nmpc_tt": (698, 684, 12), "10_obstacles": (1594, 1558, 3), "race_track_2": (1994, 1964, 2)}
# measured agreeing prefixes 22 / 98 / 99 steps, each ended by a max_iter step whose unconverged
# iterate parts at rounding level (the compiled restatement parts from the oracle at 8 / 102 / 111)
CHAIN_MIN = {"nmpc_tt": 21, "10_obstacles": 97, "race_track_2": 98}


def _load(name):
    path = os.path.join(GOLD, f"ref_run_{name}.npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path} (python tests/golden/gen_reference_runs.py {name})")
    return np.load(path)


def _spec(z):
    from nmpc_amd import make_spec
    from gen_reference_runs import RUNS

    c = RUNS[str(z["name"])]
    return make_spec(c["layout"], N=c["N"], T=c["T"])


def _warm_starts(z):
    from gen_reference_runs import warm_start

    K = len(z["status"])
    W = np.zeros((K, z["x"].shape[1]))
    for k in range(1, K):
        W[k] = warm_start(z["x"][k - 1])
    return W


@pytest.mark.parametrize("name", ["nmpc_tt", "10_obstacles", "race_track_2"])
def test_reference_run_per_step(name):
    from nmpc_amd import nlpsol, REFERENCE_OPTS

    z = _load(name)
    spec = _spec(z)
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    W = _warm_starts(z)
    sol = s(x0=W.T, lbx=z["lbx"], ubx=z["ubx"], lbg=z["lbg"], ubg=z["ubg"], p=z["p"].T)
    st, it = s.stats()["status_code"], s.stats()["iter_count"]
    ost, oit = z["status"], z["iter"]
    same = st == ost
    conv = same & np.isin(ost, (0, 1))
    ex = np.max(np.abs(sol["x"].T - z["x"]) / (1 + np.abs(z["x"])), axis=1)
    ef = np.abs(sol["f"][0] - z["f"]) / (1 + np.abs(z["f"]))
    bad_x, bad_f = conv & (ex > TOL), conv & (ef > TOL)
    K = len(ost)
    print(f"\n{name} per step: {K} solves; status agree {same.sum()}/{K}; iterations agree {(it == oit).sum()}/{K}; "
          f"converged+agreeing {conv.sum()}: x outside 1e-6 {bad_x.sum()}, f outside 1e-6 {bad_f.sum()}; "
          f"oracle statuses {dict(zip(*np.unique(ost, return_counts=True)))}")
    for i in np.flatnonzero(~same | bad_x | bad_f | (it != oit)):
        print(f"  step {i}: gpu status {st[i]} it {it[i]} | oracle status {ost[i]} it {oit[i]} | "
              f"x rel err {ex[i]:.2e} f rel err {ef[i]:.2e}")
    smin, imin, xbad = PER_STEP_MIN[name]
    assert same.sum() >= smin
    assert (it == oit).sum() >= imin
    # a converged step whose termination fell one iteration apart stops elsewhere in the
    # tol = 1e-8 neighbourhood: x may differ beyond 1e-6 along the cost's flat directions
    # while f agrees (the compiled CPU restatement shows the same)
    assert bad_f.sum() <= 1
    assert bad_x.sum() <= xbad


@pytest.mark.parametrize("name", ["nmpc_tt", "10_obstacles", "race_track_2"])
def test_reference_run_chained_and_fov_sum(name):
    import torch
    from nmpc_amd import nlpsol, REFERENCE_OPTS
    from nmpc_amd.targets import schedule

    z = _load(name)
    spec = _spec(z)
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    K = len(z["status"])
    f64 = dict(dtype=torch.float64, device="cuda")
    bnd = [torch.tensor(z[k], **f64) for k in ("lbx", "ubx", "lbg", "ubg")]
    vt, wt = schedule(name, 0, K)
    hist = {"u": torch.empty(K, 1, 6, **f64), "x": torch.empty(K, 1, 8, **f64), "f": torch.empty(K, 1, **f64),
            "fov": torch.empty(K, 1, **f64), "status": torch.empty(K, 1, dtype=torch.int32, device="cuda"),
            "iters": torch.empty(K, 1, dtype=torch.int32, device="cuda")}
    p = torch.tensor(z["p"][:1], **f64)       # [x0; xs] of the script (NMPC_TT.py:350-353)
    w = torch.zeros(1, spec.nw, **f64)        # u0 = zeros (:329)
    s.closed_loop_device(K, *bnd, p, w, torch.tensor(vt[:, None], **f64).contiguous(),
                         torch.tensor(wt[:, None], **f64).contiguous(), hist)
    torch.cuda.synchronize()
    H = {k: v.cpu().numpy()[:, 0] for k, v in hist.items()}
    # agreeing prefix: every step so far had the same state in (x0 within 1e-6), the same
    # status, and u0 and f within 1e-6 -- unconverged (max_iter) steps included: their
    # returned iterate must agree too, or the FOV errors of the prefix could not
    n = 0
    eu = ex = ef = 0.0
    for k in range(K):
        xin, ou = z["p"][k, :8], z["x"][k, :6]
        ex = np.max(np.abs(H["x"][k] - xin) / (1 + np.abs(xin)))
        eu = np.max(np.abs(H["u"][k] - ou) / (1 + np.abs(ou)))
        ef = abs(H["f"][k] - z["f"][k]) / (1 + abs(z["f"][k]))
        if not (ex <= TOL and H["status"][k] == z["status"][k] and eu <= TOL and ef <= TOL):
            break
        n += 1
    fg, fo = float(H["fov"][:n].sum()), float(z["fov"][:n].sum())
    sts = dict(zip(*np.unique(H["status"], return_counts=True)))
    print(f"\n{name} chained: {n}/{K} steps agree before the loops part; FOV-error sum over them {fg:.9f} (GPU) vs "
          f"{fo:.9f} (oracle); whole run: FOV-error sum {H['fov'].sum():.3f} (GPU) vs {float(z['fov_sum']):.3f} "
          f"(oracle), statuses {sts} vs {dict(zip(*np.unique(z['status'], return_counts=True)))}, mean iterations "
          f"{H['iters'].mean():.2f} vs {z['iter'].mean():.2f}")
    if n < K:
        print(f"  step {n}: gpu status {H['status'][n]} it {H['iters'][n]} | oracle status {z['status'][n]} "
              f"it {z['iter'][n]} | x0 rel err {ex:.2e}, u0 {eu:.2e}, f {ef:.2e}")
    assert n >= CHAIN_MIN[name]
    assert abs(fg - fo) <= TOL * (1 + abs(fo))
    assert np.all(np.isfinite(H["fov"])) and np.all(H["status"] != -1000)
