"""Generate the committed golden fixtures (run from the repo root:
``python tests/golden/gen_golden.py``).

1. derivs_*.npz -- SymPy restatement of the reference NLP, symbolically
   differentiated: F, grad F, g, J = dg/dw and W = d2/dw2 (of*F + lam^T g)
   of the single-shooting NLP at seeded points.  Formulas follow
   Python/NMPC_TT.py:139-148 (dynamics), :160-167 (Euler rollout),
   :209-220 (FOV/distance cost), :234-244 (constraint rows); the dynamic
   obstacle parameterisation follows MATLAB/Dynamic Obstacles/
   Dynamic Obstacle avoidance.m:128-133.  Independent of the hand-derived
   derivatives in oracle/nmpc_oracle.py.
2. solutions_*.npz -- converged solutions of the oracle's IPOPT restatement
   (x, f, lam_x, lam_g, status, iter) on seeded scenarios, together with
   SciPy SLSQP's objective from the same start (independent solver, not
   IPOPT).  These pin the oracle against regressions.

There is no CasADi/IPOPT in this environment and the reference ships no
golden vectors, so IPOPT parity itself stays unpinned.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import sympy as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def sympy_problem(N, T, obs, ypidx, npar):
    """Symbolic single-shooting NLP (functions of w and p)."""
    w = sp.symbols(f"w0:{6 * N}")
    p = sp.symbols(f"p0:{npar}")
    U = [[w[6 * k + j] for j in range(6)] for k in range(N)]
    X = [list(p[0:8])]
    for k in range(N):
        x = X[-1]
        u = U[k]
        f = [u[0] * sp.cos(x[4]) * sp.cos(x[3]), u[0] * sp.sin(x[4]) * sp.cos(x[3]), u[0] * sp.sin(x[3]),
             u[1], u[2], u[3], u[4], u[5]]
        X.append([x[i] + T * f[i] for i in range(8)])
    VF = HF = 1
    w1, w2 = 1, 2
    obj = 0
    for k in range(N):
        s = X[k]
        a = (s[2] * sp.tan(s[6] + sp.Rational(VF, 2)) - s[2] * sp.tan(s[6] - sp.Rational(VF, 2))) / 2
        b = (s[2] * sp.tan(s[5] + sp.Rational(HF, 2)) - s[2] * sp.tan(s[5] - sp.Rational(HF, 2))) / 2
        A = sp.cos(s[7]) ** 2 / a ** 2 + sp.sin(s[7]) ** 2 / b ** 2
        B = 2 * sp.cos(s[7]) * sp.sin(s[7]) * (1 / a ** 2 - 1 / b ** 2)
        C = sp.sin(s[7]) ** 2 / a ** 2 + sp.cos(s[7]) ** 2 / b ** 2
        XE = s[0] + a + s[2] * sp.tan(s[6] - sp.Rational(VF, 2))
        YE = s[1] + b + s[2] * sp.tan(s[5] - sp.Rational(HF, 2))
        obj += w1 * sp.sqrt((s[0] - p[8]) ** 2 + (s[1] - p[9]) ** 2) + \
            w2 * ((A * (p[8] - XE) ** 2 + B * (p[9] - YE) * (p[8] - XE) + C * (p[9] - YE) ** 2) - 1)
    g = []
    for k in range(N + 1):
        s = X[k]
        g += [s[2], s[3], s[5], s[6], s[7]]
        for j, (ox, oy, r) in enumerate(obs):
            oyv = p[ypidx[j]] if ypidx[j] >= 0 else oy
            g.append(-sp.sqrt((s[0] - ox) ** 2 + (s[1] - oyv) ** 2) + r)
    return w, p, obj, g


def gen_derivs(name, N, T, obs, ypidx, npar, npts, seed):
    from oracle import nmpc_oracle as orc

    w, p, obj, g = sympy_problem(N, T, obs, ypidx, npar)
    ng = len(g)
    lam = sp.symbols(f"l0:{ng}")
    of = sp.Symbol("of")
    grad = [sp.diff(obj, wi) for wi in w]
    jac = [[sp.diff(gi, wj) for wj in w] for gi in g]
    L = of * obj + sum(lam[i] * g[i] for i in range(ng))
    gradL = [sp.diff(L, wi) for wi in w]
    hess = [[sp.diff(gl, wj) for wj in w] for gl in gradL]
    args = list(w) + list(p) + list(lam) + [of]
    fF = sp.lambdify(args, obj, "math")
    fgrad = sp.lambdify(args, grad, "math")
    fg = sp.lambdify(args, g, "math")
    fJ = sp.lambdify(args, jac, "math")
    fW = sp.lambdify(args, hess, "math")
    prob = orc.Problem(N=N, T=T, obs_x=[o[0] for o in obs], obs_y=[o[1] for o in obs],
                       obs_rsum=[o[2] for o in obs], obs_y_pidx=ypidx, np_=npar)
    lbx, ubx, _, _ = orc.bounds(prob)
    rng = np.random.default_rng(seed)
    rec = {k: [] for k in ("w", "p", "lam", "of", "F", "grad", "g", "J", "W")}
    for _ in range(npts):
        wv = rng.uniform(lbx, ubx)
        pv = np.zeros(npar)
        pv[:8] = [rng.uniform(0, 300), rng.uniform(0, 300), rng.uniform(80, 140), rng.uniform(-.2, .2),
                  rng.uniform(-np.pi, np.pi), rng.uniform(-.4, .4), rng.uniform(-.4, .4), rng.uniform(-1.4, 1.4)]
        pv[8:11] = [pv[0] + rng.uniform(-60, 60), pv[1] + rng.uniform(-60, 60), rng.uniform(-np.pi, np.pi)]
        for j in range(len(obs)):
            if ypidx[j] >= 0:
                pv[ypidx[j]] = obs[j][1] + rng.uniform(-50, 50)
        lv = rng.normal(size=ng)
        ofv = float(rng.uniform(0.3, 1.0))
        a = list(wv) + list(pv) + list(lv) + [ofv]
        rec["w"].append(wv); rec["p"].append(pv); rec["lam"].append(lv); rec["of"].append(ofv)
        rec["F"].append(fF(*a)); rec["grad"].append(np.array(fgrad(*a), float))
        rec["g"].append(np.array(fg(*a), float)); rec["J"].append(np.array(fJ(*a), float))
        rec["W"].append(np.array(fW(*a), float))
    meta = dict(N=N, T=T, obs=np.array(obs, float).reshape(-1, 3), ypidx=np.array(ypidx, int), npar=npar)
    np.savez_compressed(os.path.join(HERE, f"derivs_{name}.npz"),
                        **{k: np.array(v) for k, v in rec.items()}, **meta)
    print("wrote", name)


def gen_solutions(name, layout, N, T, B, seed):
    from scipy.optimize import minimize
    from oracle import nmpc_oracle as orc

    prob = orc.make_problem(layout, N=N, T=T)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    rng = np.random.default_rng(seed)
    Ps, X, F, LX, LG, ST, IT, SF = [], [], [], [], [], [], [], []
    solver = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    while len(Ps) < B:
        xt, yt, pt = rng.uniform(-200, 1800), rng.uniform(-100, 1000), rng.uniform(-np.pi, np.pi)
        x0 = np.array([xt + rng.uniform(-30, 30), yt + rng.uniform(-30, 30), rng.uniform(80, 140),
                       rng.uniform(-.2, .2), rng.uniform(-np.pi, np.pi), rng.uniform(-.4, .4),
                       rng.uniform(-.4, .4), rng.uniform(-1.4, 1.4)])
        if prob.n_obs and np.any(np.hypot(x0[0] - prob.obs_x, x0[1] - prob.obs_y) <= prob.obs_rsum + 10):
            continue
        pv = np.concatenate([x0, [xt, yt, pt]])
        r = solver.solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, pv)
        fin = np.isfinite(lbg)
        cons = [dict(type="ineq", fun=lambda w_, pv=pv: (orc.constraints(prob, w_, pv) - lbg)[fin]),
                dict(type="ineq", fun=lambda w_, pv=pv: ubg - orc.constraints(prob, w_, pv))]
        s = minimize(lambda w_: orc.objective(prob, w_, pv), r["x"], method="SLSQP",
                     bounds=list(zip(lbx, ubx)), constraints=cons, options=dict(maxiter=200, ftol=1e-13))
        Ps.append(pv); X.append(r["x"]); F.append(r["f"]); LX.append(r["lam_x"]); LG.append(r["lam_g"])
        ST.append(r["status"]); IT.append(r["iter"]); SF.append(s.fun)
    np.savez_compressed(os.path.join(HERE, f"solutions_{name}.npz"), p=np.array(Ps), x=np.array(X),
                        f=np.array(F), lam_x=np.array(LX), lam_g=np.array(LG), status=np.array(ST),
                        iter=np.array(IT), slsqp_f=np.array(SF), N=N, T=T, layout=str(layout))
    print("wrote", name, "status", ST, "iters", IT)


if __name__ == "__main__":
    # N=3: 2 static obstacles ; N=2: 3 obstacles, the first two with p-indexed y (dynamic)
    gen_derivs("n3_static", 3, 0.2, [(120.0, 90.0, 35.0), (-40.0, 200.0, 105.0)], [-1, -1], 11, 4, 11)
    gen_derivs("n2_dynamic", 2, 1.0, [(150.0, 0.0, 55.0), (0.0, 300.0, 55.0), (60.0, 60.0, 55.0)],
               [11, 12, -1], 13, 3, 12)
    gen_solutions("race_track_2_n10", "race_track_2", 10, 0.2, 6, 21)
    gen_solutions("nmpc_tt_n15", "nmpc_tt", 15, 1.0, 3, 22)
