"""Dev tool: numpy model of the HIP kernel's structured Newton step (Riccati on
stage blocks), compared against the oracle's dense condensed solve."""
import os, sys, math
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import nmpc_oracle as orc

BOX = [2, 3, 5, 6, 7]

def model_step(prob, ev, x, s, y, zl, zu, vl, vu, dl, du, xl, xu, dc, df, mu, delta, kd=1e-5):
    N, m, T = prob.N, prob.m, prob.T
    X = ev.X
    # stage data
    lam = np.zeros((N + 2, 8))
    w = np.zeros((N + 1, 8))
    G = ev.Gk  # (N+1, m, 8) unscaled
    for k in range(N + 1):
        w[k] = df * ev.gl[k] + G[k].T @ (dc[k*m:(k+1)*m] * y[k*m:(k+1)*m])
    for k in range(N, 0, -1):
        lam[k] = w[k] + (ev.A[k].T @ lam[k+1] if k < N else 0)
    # rows
    lo, hi = np.isfinite(dl), np.isfinite(du)
    Sl = np.where(lo, s - dl, 1.0); Su = np.where(hi, du - s, 1.0)
    D = np.where(lo, vl / Sl, 0) + np.where(hi, vu / Su, 0) + delta
    rs = -y - np.where(lo, mu / Sl, 0) + np.where(hi, mu / Su, 0) + kd * mu * ((lo & ~hi) * 1.0 - (hi & ~lo) * 1.0)
    rd = ev.g * dc - s  # d - s
    wr = y + D * rd + rs
    # U barrier
    xlo, xhi = np.isfinite(xl), np.isfinite(xu)
    SXl = np.where(xlo, x - xl, 1.0); SXu = np.where(xhi, xu - x, 1.0)
    sigx = np.where(xlo, zl / SXl, 0) + np.where(xhi, zu / SXu, 0)
    ru = -np.where(xlo, mu / SXl, 0) + np.where(xhi, mu / SXu, 0) + kd * mu * ((xlo & ~xhi) * 1.0 - (xhi & ~xlo) * 1.0)
    Qs, qs = [], []
    for k in range(N + 1):
        Gt = dc[k*m:(k+1)*m, None] * G[k]
        Q = df * ev.Hl[k] + Gt.T @ (D[k*m:(k+1)*m, None] * Gt)
        if prob.n_obs:
            cy = y[k*m+5:(k+1)*m] * dc[k*m+5:(k+1)*m]
            Q[0:2, 0:2] += np.einsum('j,jab->ab', cy, ev.Hg[k])
        q = df * ev.gl[k] + Gt.T @ wr[k*m:(k+1)*m]
        Ss = np.zeros((6, 8))
        if k < N:
            Hxx, Hxu = orc.dyn_hess(prob, X[:, k], ev.U[:, k], lam[k+1])
            Q = Q + Hxx; Ss = Hxu.T
        Qs.append((Q, Ss)); qs.append(q)
    P = Qs[N][0].copy(); p = qs[N].copy()
    Ks, ks = [None]*N, [None]*N
    ok = True
    for k in range(N - 1, -1, -1):
        A, B = ev.A[k], ev.B[k]
        Q, Ss = Qs[k]
        R = np.diag(sigx[6*k:6*k+6] + delta)
        Rt = R + B.T @ P @ B
        St = Ss + B.T @ P @ A
        rt = ru[6*k:6*k+6] + B.T @ p
        try:
            np.linalg.cholesky(Rt)
        except np.linalg.LinAlgError:
            ok = False; break
        K = -np.linalg.solve(Rt, St); kk = -np.linalg.solve(Rt, rt)
        Ks[k], ks[k] = K, kk
        P = Q + A.T @ P @ A + St.T @ K
        p = qs[k] + A.T @ p + K.T @ rt
    if not ok:
        return None
    dX = np.zeros((N + 1, 8)); dU = np.zeros((N, 6))
    for k in range(N):
        dU[k] = Ks[k] @ dX[k] + ks[k]
        dX[k+1] = ev.A[k] @ dX[k] + ev.B[k] @ dU[k]
    return dU.ravel()

def dense_step(prob, ev, x, s, y, zl, zu, vl, vu, dl, du, xl, xu, dc, df, mu, delta, kd=1e-5):
    J = dc[:, None] * ev.J
    W = ev.hessian(df, dc * y)
    lo, hi = np.isfinite(dl), np.isfinite(du)
    Sl = np.where(lo, s - dl, 1.0); Su = np.where(hi, du - s, 1.0)
    SigS = np.where(lo, vl / Sl, 0) + np.where(hi, vu / Su, 0)
    xlo, xhi = np.isfinite(xl), np.isfinite(xu)
    SXl = np.where(xlo, x - xl, 1.0); SXu = np.where(xhi, xu - x, 1.0)
    SigX = np.where(xlo, zl / SXl, 0) + np.where(xhi, zu / SXu, 0)
    gphi = df * ev.gradF - np.where(xlo, mu / SXl, 0) + np.where(xhi, mu / SXu, 0) + kd * mu * ((xlo & ~xhi) * 1.0 - (xhi & ~xlo) * 1.0)
    rs = -y - np.where(lo, mu / Sl, 0) + np.where(hi, mu / Su, 0) + kd * mu * ((lo & ~hi) * 1.0 - (hi & ~lo) * 1.0)
    rd = dc * ev.g - s
    D = SigS + delta
    M = W + np.diag(SigX + delta) + J.T @ (D[:, None] * J)
    return -np.linalg.solve(M, gphi + J.T @ (y + D * rd + rs))

if __name__ == "__main__":
    prob = orc.make_problem("race_track_2", N=20, T=0.2)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    rng = np.random.default_rng(5)
    p = np.array([500., 400, 100, 0.05, 0.3, 0.1, -0.1, 0.3, 520, 410, 0.2])
    x = np.clip(rng.uniform(lbx, ubx), lbx + 0.01, ubx - 0.01)
    ev = orc.SSEval(prob, x, p)
    m = prob.m; ng = prob.ng
    dc = rng.uniform(0.5, 1.0, ng); df = 0.7
    dl = np.where(np.isfinite(lbg), dc * lbg, -np.inf); du = np.where(np.isfinite(ubg), dc * ubg, np.inf)
    d = dc * ev.g
    s = np.clip(d + rng.normal(0, 0.1, ng), np.where(np.isfinite(dl), dl + 0.05, -1e300), np.where(np.isfinite(du), du - 0.05, 1e300))
    y = rng.normal(0, 1, ng); vl = rng.uniform(0.1, 2, ng) * np.isfinite(dl); vu = rng.uniform(0.1, 2, ng) * np.isfinite(du)
    zl = rng.uniform(0.1, 2, prob.nw); zu = rng.uniform(0.1, 2, prob.nw)
    for delta in (0.0, 1e-2, 10.0):
        a = model_step(prob, ev, x, s, y, zl, zu, vl, vu, dl, du, lbx, ubx, dc, df, 0.1, delta)
        b = dense_step(prob, ev, x, s, y, zl, zu, vl, vu, dl, du, lbx, ubx, dc, df, 0.1, delta)
        if a is None:
            print('delta', delta, 'riccati: not PD;', 'dense PD?', np.all(np.linalg.eigvalsh((lambda M: M)(np.eye(1)))))
            continue
        print('delta', delta, 'max |model - dense| =', np.max(np.abs(a - b)), 'scale', np.max(np.abs(b)))
