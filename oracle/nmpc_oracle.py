"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY. NOT PART OF THE PRODUCT.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the *checker*.  The product path
(``mpc-implementation_amd/``) never imports it and has no CPU fallback.

What this is
------------
A plain numpy fp64 restatement of the per-timestep NLP of
``Python/NMPC_TT.py`` (UAV + 3-DoF gimbal target tracking, FOV cost,
obstacle-distance constraints) and of the algorithm that solves it there,
``ca.nlpsol('solver', 'ipopt', ...)`` (``Python/NMPC_TT.py:250-267``).

* Problem functions follow the reference line by line:
  dynamics ``Python/NMPC_TT.py:139-148``, Euler single-shooting rollout
  ``:153-167``, FOV/distance objective ``:192-221``, constraint vector
  ``:234-244`` (10-row layouts: ``Python/10_obstacles.py:272-289``,
  ``Python/Race Track 2.py:247-264``), bounds ``:269-306`` (generalised to any
  N / obstacle count), plant/target shift ``:13-30``.
* Derivatives are hand-derived (chain rule through the ellipse form
  Q = (r1/a)^2 + (r2/b)^2 of ``:209-220``) and pinned against SymPy goldens
  (``tests/golden/gen_golden.py``).
* The solver is a restatement of IPOPT's published primal-dual interior-point
  filter line-search method (Waechter & Biegler, Math. Prog. 106(1), 2006;
  IPOPT 3.12/3.14 default options, the version CasADi 3.5.5 -- named in
  ``MATLAB/Dynamic Obstacles/NMPC_TT.m:2`` -- bundles) applied to the
  reference's *single-shooting* NLP (decision vector = vec(U) only, F1).
  Linear algebra is DENSE here: the condensed 6N x 6N primal-dual matrix is
  assembled explicitly and Cholesky-factorised (inertia test = Cholesky
  success).  The HIP product computes the same Newton step with a stage-wise
  Riccati recursion; agreement of the two is the parity test.

Parity status: CasADi/IPOPT is not installed here nor on the GPU box and the
reference holds no golden vectors, so parity with IPOPT itself is UNPINNED.
The function layer is pinned by SymPy; converged solutions are cross-checked
against SciPy's independent SLSQP solver (KKT-point agreement).

Restated IPOPT subset: gradient-based NLP scaling, bound
relaxation, bound push, least-squares constraint-multiplier initialisation,
monotone (Fiacco-McCormick) barrier update with fast decrease, inertia
correction on the Hessian block, fraction-to-boundary, filter line search with
Armijo/F-type switching, second-order corrections, tiny-step detection,
kappa_sigma multiplier safeguard, soft restoration phase, the feasibility
restoration phase (min rho*sum(p+n) + eta/2*|D_R(x-x_R)|^2 s.t. d(x)-p+n in
[d_L,d_U], its own filter line search, return test against the original
filter, bound-multiplier reconstruction), return to the last acceptable point
when restoration is called at an almost feasible point, optimal/acceptable/
max-iter/infeasible termination, honor_original_bounds, and the watchdog
procedure (watchdog_shortened_iter_trigger / watchdog_trial_iter_max) in the
main and the restoration line search.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

PI = math.pi
EPS = np.finfo(np.float64).eps
INF = 1e19  # IPOPT nlp_lower/upper_bound_inf: |b| >= 1e19 means "no bound"

# --- reference constants: Python/NMPC_TT.py:57-89, :204-205, :224-231 -------
V_MIN, V_MAX = 14.0, 30.0
W2U, W3U, WG = PI / 30, PI / 21, PI / 30
THETA_U, Z_MIN, Z_MAX = 0.2618, 75.0, 150.0
PHI_G, THETA_G, SHI_G = PI / 6, PI / 6, PI / 2
UAV_R = 5.0

# Obstacle layouts (x, y) and obstacle radius.
OBSTACLE_LAYOUTS = {
    # Python/NMPC_TT.py:224-231
    "nmpc_tt": ([(175, 820), (-134, 155), (441, 343)], 30.0),
    # Python/10_obstacles.py:247-269 (obstacles 4-10 parked at 10000,10000)
    "10_obstacles": ([(500, 20), (1700, 197), (130, 830)] + [(10000, 10000)] * 7, 100.0),
    # Python/Race Track 2.py:223-244 (all 10 active)
    "race_track_2": ([(0, 80), (500, 245), (1000, 70), (1500, 295), (1765, 550),
                      (1500, 750), (1000, 1005), (500, 800), (-100, 950), (-200, 550)], 50.0),
    # MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:98-119 (y of 1-6 are
    # parameters P(12:17) = p[11:17], :128-133); values here are the initial ys
    "dynamic": ([(2500, 0), (0, 300), (500, 0), (1000, 300), (1500, 0), (2000, 300),
                 (1300, 1300), (1300, 1300), (1300, 1300), (1300, 1300)], 50.0),
}


@dataclass
class Problem:
    """The reference NLP for one horizon length / obstacle table.

    obs_x_pidx / obs_y_pidx: -1 = constant coordinate, else index into p
    (dynamic obstacles, MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:128-133).
    """
    N: int = 15
    T: float = 1.0
    obs_x: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_y: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_rsum: np.ndarray = field(default_factory=lambda: np.zeros(0))
    obs_x_pidx: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=int))
    obs_y_pidx: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=int))
    w1: float = 1.0
    w2: float = 2.0
    vfov: float = 1.0
    hfov: float = 1.0
    np_: int = 11
    # cost weights taken from p (batched weight sweep): index or -1
    w1_pidx: int = -1
    w2_pidx: int = -1
    # "uav8g": 8 states / 6 controls (Python/NMPC_TT.py:94-151);
    # "uav5": no gimbal, 5 states / 3 controls, distance cost, rows [z, theta]
    # (MATLAB/Dynamic Obstacles/NMPC_TT.m:26-35,102-111,129-134)
    model: str = "uav8g"

    @property
    def nx(self):
        return 5 if self.model == "uav5" else 8

    @property
    def nu(self):
        return 3 if self.model == "uav5" else 6

    @property
    def box_states(self):
        """state index of each box row of a stage (z, theta, x5, x6, x7 / z, theta)."""
        return [2, 3] if self.model == "uav5" else [2, 3, 5, 6, 7]

    @property
    def nb(self):
        return len(self.box_states)

    @property
    def target_index(self):
        """index of the target's x in p (P(6) in the no-gimbal script, P(9) else)."""
        return self.nx

    def __post_init__(self):
        self.obs_x = np.asarray(self.obs_x, dtype=float)
        self.obs_y = np.asarray(self.obs_y, dtype=float)
        self.obs_rsum = np.asarray(self.obs_rsum, dtype=float)
        n = len(self.obs_x)
        if len(self.obs_x_pidx) != n:
            self.obs_x_pidx = -np.ones(n, dtype=int)
        if len(self.obs_y_pidx) != n:
            self.obs_y_pidx = -np.ones(n, dtype=int)
        self.obs_x_pidx = np.asarray(self.obs_x_pidx, dtype=int)
        self.obs_y_pidx = np.asarray(self.obs_y_pidx, dtype=int)

    @property
    def n_obs(self):
        return len(self.obs_x)

    @property
    def m(self):
        return self.nb + self.n_obs

    @property
    def nw(self):
        return self.nu * self.N

    @property
    def ng(self):
        return self.m * (self.N + 1)

    def weighted(self, p):
        """This problem with w1/w2 read from p where w1_pidx/w2_pidx are set."""
        if self.w1_pidx < 0 and self.w2_pidx < 0:
            return self
        import dataclasses
        return dataclasses.replace(
            self, w1=float(p[self.w1_pidx]) if self.w1_pidx >= 0 else self.w1,
            w2=float(p[self.w2_pidx]) if self.w2_pidx >= 0 else self.w2)

    def obstacles(self, p):
        ox = self.obs_x.copy()
        oy = self.obs_y.copy()
        for j in range(self.n_obs):
            if self.obs_x_pidx[j] >= 0:
                ox[j] = p[self.obs_x_pidx[j]]
            if self.obs_y_pidx[j] >= 0:
                oy[j] = p[self.obs_y_pidx[j]]
        return ox, oy


def make_problem(layout: str | None, N: int, T: float, dynamic: bool = False, model: str = "uav8g") -> Problem:
    """Problem for a named reference obstacle layout (None = 0 obstacles)."""
    np0 = 8 if model == "uav5" else 11
    if layout is None:
        return Problem(N=N, T=T, model=model, np_=np0)
    xy, r = OBSTACLE_LAYOUTS[layout]
    ox = np.array([a for a, _ in xy], float)
    oy = np.array([b for _, b in xy], float)
    rs = np.full(len(xy), UAV_R + r)
    ypidx = -np.ones(len(xy), dtype=int)
    np_ = np0
    if dynamic:
        ypidx[:6] = np.arange(np0, np0 + 6)  # P(12:17) in MATLAB 1-based
        np_ = np0 + 6
    return Problem(N=N, T=T, obs_x=ox, obs_y=oy, obs_rsum=rs, obs_y_pidx=ypidx, np_=np_, model=model)


def bounds(prob: Problem):
    N = prob.N
    if prob.model == "uav5":  # MATLAB/Dynamic Obstacles/NMPC_TT.m:140-149
        lbx = np.tile([V_MIN, -W2U, -W3U], N)
        ubx = np.tile([V_MAX, W2U, W3U], N)
        lrow = np.concatenate([[Z_MIN, -THETA_U], np.full(prob.n_obs, -np.inf)])
        urow = np.concatenate([[Z_MAX, THETA_U], np.zeros(prob.n_obs)])
        return lbx, ubx, np.tile(lrow, N + 1), np.tile(urow, N + 1)
    lbx = np.tile([V_MIN, -W2U, -W3U, -WG, -WG, -WG], N)
    ubx = np.tile([V_MAX, W2U, W3U, WG, WG, WG], N)
    lrow = np.concatenate([[Z_MIN, -THETA_U, -PHI_G, -THETA_G, -SHI_G], np.full(prob.n_obs, -np.inf)])
    urow = np.concatenate([[Z_MAX, THETA_U, PHI_G, THETA_G, SHI_G], np.zeros(prob.n_obs)])
    return lbx, ubx, np.tile(lrow, N + 1), np.tile(urow, N + 1)


def _pad8(x):
    """no-gimbal state / control padded into the gimbal model's (the no-gimbal
    dynamics are its first five components, MATLAB/Dynamic Obstacles/NMPC_TT.m:37-38)."""
    out = np.zeros(8 if len(x) == 5 else 6)
    out[:len(x)] = x
    return out


# --- model: Python/NMPC_TT.py:139-148 ----------------------------------------
def dynamics(x, u):
    th, ps, v = x[3], x[4], u[0]
    return np.array([v * math.cos(ps) * math.cos(th), v * math.sin(ps) * math.cos(th),
                     v * math.sin(th), u[1], u[2], u[3], u[4], u[5]])


def unpack_w(prob, w):
    """w = vec(U), U is nu x N column-major (Python/NMPC_TT.py:247-248)."""
    return np.asarray(w, float).reshape(prob.N, prob.nu).T


def dynamics5(x, u):
    """No-gimbal kinematics, MATLAB/Dynamic Obstacles/NMPC_TT.m:37-38."""
    th, ps, v = x[3], x[4], u[0]
    return np.array([v * math.cos(ps) * math.cos(th), v * math.sin(ps) * math.cos(th),
                     v * math.sin(th), u[1], u[2]])


def rollout(prob, U, x0):
    """X[:,0] = P[0:nx]; X[:,k+1] = X[:,k] + T f(X[:,k], U[:,k])  (:160-167; NMPC_TT.m:49-54)."""
    f = dynamics5 if prob.model == "uav5" else dynamics
    X = np.zeros((prob.nx, prob.N + 1))
    X[:, 0] = x0
    for k in range(prob.N):
        X[:, k + 1] = X[:, k] + prob.T * f(X[:, k], U[:, k])
    return X


def stage_cost(prob, xk, xt, yt):
    """Literal restatement of Python/NMPC_TT.py:209-220 for one stage (no-gimbal
    model: the distance term only, MATLAB/Dynamic Obstacles/NMPC_TT.m:102-105)."""
    if prob.model == "uav5":
        return prob.w1 * math.sqrt((xk[0] - xt) ** 2 + (xk[1] - yt) ** 2)
    hv, hh = prob.vfov / 2, prob.hfov / 2
    z = xk[2]
    a = (z * math.tan(xk[6] + hv) - z * math.tan(xk[6] - hv)) / 2
    b = (z * math.tan(xk[5] + hh) - z * math.tan(xk[5] - hh)) / 2
    c7, s7 = math.cos(xk[7]), math.sin(xk[7])
    A = c7 ** 2 / a ** 2 + s7 ** 2 / b ** 2
    B = 2 * c7 * s7 * ((1 / a ** 2) - (1 / b ** 2))
    C = s7 ** 2 / a ** 2 + c7 ** 2 / b ** 2
    XE = xk[0] + a + z * math.tan(xk[6] - hv)
    YE = xk[1] + b + z * math.tan(xk[5] - hh)
    return (prob.w1 * math.sqrt((xk[0] - xt) ** 2 + (xk[1] - yt) ** 2)
            + prob.w2 * ((A * (xt - XE) ** 2 + B * (yt - YE) * (xt - XE) + C * (yt - YE) ** 2) - 1))


def stage_rows(prob, xk, ox, oy):
    """g rows for one stage (Python/NMPC_TT.py:234-244)."""
    d = np.sqrt((xk[0] - ox) ** 2 + (xk[1] - oy) ** 2)
    return np.concatenate([xk[prob.box_states], -d + prob.obs_rsum])


def objective(prob, w, p):
    prob = prob.weighted(p)
    X = rollout(prob, unpack_w(prob, w), p[:prob.nx])
    ti = prob.target_index
    return sum(stage_cost(prob, X[:, k], p[ti], p[ti + 1]) for k in range(prob.N))


def constraints(prob, w, p):
    X = rollout(prob, unpack_w(prob, w), p[:prob.nx])
    ox, oy = prob.obstacles(p)
    return np.concatenate([stage_rows(prob, X[:, k], ox, oy) for k in range(prob.N + 1)])


def lam_p(prob, w, p, lam_g, h=1e-6):
    """CasADi nlpsol's lam_p = -grad_p (f + lam_g' g) at (w, p), by central differences
    of objective() / constraints() (checker for the kernel's analytic lam_p; relative
    step h, accuracy ~h^2 plus rounding)."""
    p = np.asarray(p, dtype=float)
    out = np.zeros_like(p)
    for i in range(len(p)):
        d = h * max(1.0, abs(p[i]))
        pp, pm = p.copy(), p.copy()
        pp[i] += d
        pm[i] -= d
        Lp = objective(prob, w, pp) + lam_g @ constraints(prob, w, pp)
        Lm = objective(prob, w, pm) + lam_g @ constraints(prob, w, pm)
        out[i] = -(Lp - Lm) / (2 * d)
    return out


# --- hand-derived derivatives ------------------------------------------------
_V = [0, 1, 2, 5, 6, 7]  # state indices the stage cost depends on


def _as8(prob):
    """the gimbal-model problem whose first 5 states / 3 controls are the no-gimbal model's."""
    import dataclasses
    return dataclasses.replace(prob, model="uav8g", w2=0.0)


def stage_cost_derivs(prob, xk, xt, yt):
    if prob.model == "uav5":
        v, g, H = stage_cost_derivs(_as8(prob), _pad8(xk), xt, yt)
        return v, g[:5], H[:5, :5]
    return _stage_cost_derivs8(prob, xk, xt, yt)


def _stage_cost_derivs8(prob, xk, xt, yt):
    """(value, grad (8,), hess (8,8)) of the stage cost of :209-220.

    Uses the algebraically equal form  Q = A ex^2 + B ex ey + C ey^2
    = (r1/a)^2 + (r2/b)^2,  r1 = c ex + s ey, r2 = s ex - c ey,
    ex = xt - XE, ey = yt - YE, XE = x + z*be6, YE = y + z*be5,
    a = z*al6, b = z*al5, al = (tan(+)-tan(-))/2, be = (tan(+)+tan(-))/2.
    Local variable order v = (x, y, z, x5, x6, x7).
    """
    hv, hh = prob.vfov / 2, prob.hfov / 2
    x, y, z, x5, x6, x7 = (xk[i] for i in _V)
    t6p, t6m = math.tan(x6 + hv), math.tan(x6 - hv)
    t5p, t5m = math.tan(x5 + hh), math.tan(x5 - hh)
    al6, be6 = (t6p - t6m) / 2, (t6p + t6m) / 2
    al5, be5 = (t5p - t5m) / 2, (t5p + t5m) / 2
    al6d, be6d = (t6p ** 2 - t6m ** 2) / 2, (2 + t6p ** 2 + t6m ** 2) / 2
    al5d, be5d = (t5p ** 2 - t5m ** 2) / 2, (2 + t5p ** 2 + t5m ** 2) / 2
    s6p, s6m = t6p * (1 + t6p ** 2), t6m * (1 + t6m ** 2)
    s5p, s5m = t5p * (1 + t5p ** 2), t5m * (1 + t5m ** 2)
    al6dd, be6dd = s6p - s6m, s6p + s6m
    al5dd, be5dd = s5p - s5m, s5p + s5m

    ex = xt - x - z * be6
    ey = yt - y - z * be5
    gex = np.array([-1.0, 0, -be6, 0, -z * be6d, 0])
    gey = np.array([0, -1.0, -be5, -z * be5d, 0, 0])
    Hex = np.zeros((6, 6)); Hex[2, 4] = Hex[4, 2] = -be6d; Hex[4, 4] = -z * be6dd
    Hey = np.zeros((6, 6)); Hey[2, 3] = Hey[3, 2] = -be5d; Hey[3, 3] = -z * be5dd
    a = z * al6
    ga = np.array([0, 0, al6, 0, z * al6d, 0])
    Ha = np.zeros((6, 6)); Ha[2, 4] = Ha[4, 2] = al6d; Ha[4, 4] = z * al6dd
    b = z * al5
    gb = np.array([0, 0, al5, z * al5d, 0, 0])
    Hb = np.zeros((6, 6)); Hb[2, 3] = Hb[3, 2] = al5d; Hb[3, 3] = z * al5dd

    c, s = math.cos(x7), math.sin(x7)
    e7 = np.zeros(6); e7[5] = 1.0
    r1 = c * ex + s * ey
    r2 = s * ex - c * ey
    u1 = -s * gex + c * gey
    u2 = c * gex + s * gey
    gr1 = c * gex + s * gey - r2 * e7
    gr2 = s * gex - c * gey + r1 * e7
    Hr1 = c * Hex + s * Hey + np.outer(e7, u1) + np.outer(u1, e7) - r1 * np.outer(e7, e7)
    Hr2 = s * Hex - c * Hey + np.outer(e7, u2) + np.outer(u2, e7) - r2 * np.outer(e7, e7)

    e1 = r1 / a
    ge1 = (gr1 - e1 * ga) / a
    He1 = (Hr1 - np.outer(ge1, ga) - np.outer(ga, ge1) - e1 * Ha) / a
    e2 = r2 / b
    ge2 = (gr2 - e2 * gb) / b
    He2 = (Hr2 - np.outer(ge2, gb) - np.outer(gb, ge2) - e2 * Hb) / b
    Q = e1 * e1 + e2 * e2
    gQ = 2 * (e1 * ge1 + e2 * ge2)
    HQ = 2 * (np.outer(ge1, ge1) + np.outer(ge2, ge2) + e1 * He1 + e2 * He2)

    dx, dy = x - xt, y - yt
    d = math.sqrt(dx * dx + dy * dy)
    gd = np.zeros(6); gd[0], gd[1] = dx / d, dy / d
    Hd = np.zeros((6, 6))
    d3 = d ** 3
    Hd[0, 0], Hd[0, 1], Hd[1, 1] = dy * dy / d3, -dx * dy / d3, dx * dx / d3
    Hd[1, 0] = Hd[0, 1]

    val = prob.w1 * d + prob.w2 * (Q - 1)
    g6 = prob.w1 * gd + prob.w2 * gQ
    H6 = prob.w1 * Hd + prob.w2 * HQ
    g = np.zeros(8); g[_V] = g6
    H = np.zeros((8, 8)); H[np.ix_(_V, _V)] = H6
    return val, g, H


def obstacle_derivs(xk, ox, oy):
    """Row -sqrt((x-ox)^2+(y-oy)^2)+R: gradients (n,2) and Hessians (n,2,2) in (x,y)."""
    dx, dy = xk[0] - ox, xk[1] - oy
    d = np.sqrt(dx * dx + dy * dy)
    G = -np.stack([dx / d, dy / d], axis=1)
    d3 = d ** 3
    H = np.zeros((len(ox), 2, 2))
    H[:, 0, 0] = -dy * dy / d3
    H[:, 0, 1] = H[:, 1, 0] = dx * dy / d3
    H[:, 1, 1] = -dx * dx / d3
    return G, H


def dyn_jac(prob, xk, uk):
    """A = I + T f_x, B = T f_u for the Euler step (:162-167)."""
    if prob.model == "uav5":
        A, B = dyn_jac(_as8(prob), _pad8(xk), _pad8(uk))
        return A[:5, :5], B[:5, :3]
    T = prob.T
    th, ps, v = xk[3], xk[4], uk[0]
    ct, st, cp, sp = math.cos(th), math.sin(th), math.cos(ps), math.sin(ps)
    A = np.eye(8)
    A[0, 3], A[0, 4] = -T * v * cp * st, -T * v * sp * ct
    A[1, 3], A[1, 4] = -T * v * sp * st, T * v * cp * ct
    A[2, 3] = T * v * ct
    B = np.zeros((8, 6))
    B[0, 0], B[1, 0], B[2, 0] = T * cp * ct, T * sp * ct, T * st
    for j in range(5):
        B[3 + j, 1 + j] = T
    return A, B


def dyn_hess(prob, xk, uk, lam):
    """Second derivatives of lam^T (T f(x,u)): (Hxx (8,8), Hxu (8,6))."""
    if prob.model == "uav5":
        Hxx, Hxu = dyn_hess(_as8(prob), _pad8(xk), _pad8(uk), _pad8(lam))
        return Hxx[:5, :5], Hxu[:5, :3]
    T = prob.T
    th, ps, v = xk[3], xk[4], uk[0]
    ct, st, cp, sp = math.cos(th), math.sin(th), math.cos(ps), math.sin(ps)
    l0, l1, l2 = lam[0], lam[1], lam[2]
    Hxx = np.zeros((8, 8))
    Hxx[3, 3] = T * (-l0 * v * cp * ct - l1 * v * sp * ct - l2 * v * st)
    Hxx[4, 4] = T * (-l0 * v * cp * ct - l1 * v * sp * ct)
    Hxx[3, 4] = Hxx[4, 3] = T * (l0 * v * sp * st - l1 * v * cp * st)
    Hxu = np.zeros((8, 6))
    Hxu[3, 0] = T * (-l0 * cp * st - l1 * sp * st + l2 * ct)
    Hxu[4, 0] = T * (-l0 * sp * ct + l1 * cp * ct)
    return Hxx, Hxu


class SSEval:
    """Single-shooting evaluation of the reference NLP at one point w.

    Provides F, grad F, g, J = dg/dw (dense), and the Lagrangian Hessian
    W = d2/dw2 (obj_factor*F + lam^T g) via the reduced-Hessian identity
    W = [Z;E]^T H_L [Z;E] with the adjoint multipliers of the Euler dynamics.
    """

    def __init__(self, prob: Problem, w, p):
        prob = prob.weighted(np.asarray(p, float))
        self.prob = prob
        N, nw = prob.N, prob.nw
        self.p = np.asarray(p, float)
        nx, nu = prob.nx, prob.nu
        self.U = unpack_w(prob, w)
        self.X = rollout(prob, self.U, self.p[:nx])
        self.ox, self.oy = prob.obstacles(self.p)
        xt, yt = self.p[prob.target_index], self.p[prob.target_index + 1]
        self.F = 0.0
        self.gl = np.zeros((N + 1, nx))
        self.Hl = np.zeros((N + 1, nx, nx))
        for k in range(N):
            v, g, H = stage_cost_derivs(prob, self.X[:, k], xt, yt)
            self.F += v
            self.gl[k], self.Hl[k] = g, H
        self.g = np.concatenate([stage_rows(prob, self.X[:, k], self.ox, self.oy) for k in range(N + 1)])
        # dynamics jacobians and forward sensitivities Z_k = dX_k/dw
        self.A = np.zeros((N, nx, nx))
        self.B = np.zeros((N, nx, nu))
        self.Z = np.zeros((N + 1, nx, nw))
        for k in range(N):
            self.A[k], self.B[k] = dyn_jac(prob, self.X[:, k], self.U[:, k])
            self.Z[k + 1] = self.A[k] @ self.Z[k]
            self.Z[k + 1][:, nu * k:nu * k + nu] += self.B[k]
        # constraint-row jacobians wrt X_k
        m = prob.m
        self.Gk = np.zeros((N + 1, m, nx))
        self.Hg = np.zeros((N + 1, prob.n_obs, 2, 2))
        for k in range(N + 1):
            for i, idx in enumerate(prob.box_states):
                self.Gk[k, i, idx] = 1.0
            if prob.n_obs:
                G2, H2 = obstacle_derivs(self.X[:, k], self.ox, self.oy)
                self.Gk[k, prob.nb:, 0:2] = G2
                self.Hg[k] = H2
        # stage 0 is constant in w (X_0 = p[0:8], F7): Z_0 = 0, so its terms are
        # structurally absent -- as in CasADi's symbolic AD -- and are skipped
        # rather than multiplied by zero (a 0*NaN would poison the result).
        self.gradF = sum((self.Z[k].T @ self.gl[k] for k in range(1, N)), np.zeros(nw))
        self.J = np.concatenate([np.zeros((m, nw))] + [self.Gk[k] @ self.Z[k] for k in range(1, N + 1)], axis=0)

    def hessian(self, obj_factor, lam_g):
        prob = self.prob
        N, m, nw = prob.N, prob.m, prob.nw
        lam = np.asarray(lam_g, float).reshape(N + 1, m)
        # adjoint: lam_k = obj*gl_k + G_k^T y_k + A_k^T lam_{k+1}
        nx, nu, nb = prob.nx, prob.nu, prob.nb
        adj = np.zeros((N + 2, nx))
        for k in range(N, 0, -1):
            adj[k] = obj_factor * self.gl[k] + self.Gk[k].T @ lam[k]
            if k < N:
                adj[k] += self.A[k].T @ adj[k + 1]
        W = np.zeros((nw, nw))
        for k in range(1, N + 1):
            Hxx = obj_factor * self.Hl[k]
            if prob.n_obs:
                Hxx[0:2, 0:2] += np.einsum("j,jab->ab", lam[k, nb:], self.Hg[k])
            Hxu = np.zeros((nx, nu))
            if k < N:
                dHxx, Hxu = dyn_hess(prob, self.X[:, k], self.U[:, k], adj[k + 1])
                Hxx = Hxx + dHxx
            Zk = self.Z[k]
            W += Zk.T @ Hxx @ Zk
            if k < N:
                C = Zk.T @ Hxu  # (nw, nu)
                W[:, nu * k:nu * k + nu] += C
                W[nu * k:nu * k + nu, :] += C.T
        return W


# --- IPOPT restatement --------------------------------------------------------
IPOPT_DEFAULTS = dict(
    max_iter=3000, tol=1e-8, acceptable_tol=1e-6, acceptable_iter=15,
    acceptable_obj_change_tol=1e20, acceptable_dual_inf_tol=1e10,
    acceptable_constr_viol_tol=1e-2, acceptable_compl_inf_tol=1e-2,
    dual_inf_tol=1.0, constr_viol_tol=1e-4, compl_inf_tol=1e-4,
    mu_init=0.1, kappa_mu=0.2, theta_mu=1.5, barrier_tol_factor=10.0, tau_min=0.99,
    bound_push=1e-2, bound_frac=1e-2, slack_bound_push=1e-2, slack_bound_frac=1e-2,
    bound_relax_factor=1e-8, bound_mult_init_val=1.0, constr_mult_init_max=1e3,
    nlp_scaling_max_gradient=100.0, nlp_scaling_min_value=1e-8,
    kappa_d=1e-5, kappa_sigma=1e10, s_max=100.0,
    theta_max_fact=1e4, theta_min_fact=1e-4, gamma_theta=1e-5, gamma_phi=1e-8,
    delta=1.0, s_theta=1.1, s_phi=2.3, eta_phi=1e-8, alpha_red_factor=0.5,
    alpha_min_frac=0.05, max_soc=4, kappa_soc=0.99, obj_max_inc=5.0,
    first_hessian_perturbation=1e-4, min_hessian_perturbation=1e-20,
    max_hessian_perturbation=1e20, perturb_inc_fact_first=100.0,
    perturb_inc_fact=8.0, perturb_dec_fact=1.0 / 3.0,
    tiny_step_tol=10 * EPS, soft_resto_pderror_reduction_factor=0.9999,
    max_soft_resto_iters=10,
    # watchdog procedure (BacktrackingLineSearch::StartWatchDog / StopWatchDog)
    watchdog_shortened_iter_trigger=10, watchdog_trial_iter_max=3,
    # feasibility restoration phase (RestoMinC_1Nrm / RestoIpoptNLP defaults)
    resto_penalty_parameter=1000.0, resto_proximity_weight=1.0,
    required_infeasibility_reduction=0.9, bound_mult_reset_threshold=1000.0,
    constr_mult_reset_threshold=0.0,
)

# The reference's option dict (Python/NMPC_TT.py:257-265)
REFERENCE_OPTS = dict(max_iter=100, acceptable_tol=1e-8, acceptable_obj_change_tol=1e-6)

# IPOPT ApplicationReturnStatus codes
SOLVE_SUCCEEDED, SOLVED_TO_ACCEPTABLE_LEVEL, SEARCH_DIRECTION_TOO_SMALL = 0, 1, 3
INFEASIBLE_PROBLEM_DETECTED = 2
MAXIMUM_ITERATIONS_EXCEEDED, RESTORATION_FAILED, ERROR_IN_STEP_COMPUTATION = -1, -2, -3
INVALID_NUMBER_DETECTED = -13


def _compare_le(lhs, rhs, basval):
    """IPOPT's Compare_le: lhs <= rhs up to 10*eps*|basval|."""
    return lhs - rhs <= 10.0 * EPS * abs(basval)


class _Chol:
    """Cholesky factor of the condensed Newton matrix and its solve.  variant 0 is the
    plain factorisation (the committed fixtures); variant v > 0 factors P M P^T for a fixed
    symmetric permutation P of the variables (IpoptDense.la_variant): 1 reverses the
    order, 2 takes the even then the odd positions, 3 rotates by a third.  Each is the
    same Newton step in exact arithmetic and differs from variant 0 by rounding alone."""

    def __init__(self, M, variant=0):
        n = M.shape[0]
        self.perm = None
        if variant == 1:
            self.perm = np.arange(n)[::-1]
        elif variant == 2:
            self.perm = np.concatenate([np.arange(0, n, 2), np.arange(1, n, 2)])
        elif variant == 3:
            self.perm = np.roll(np.arange(n), n // 3)
        self.L = np.linalg.cholesky(M if self.perm is None else M[np.ix_(self.perm, self.perm)])

    def solve(self, b):
        if self.perm is not None:
            b = b[self.perm]
        t = np.linalg.solve(self.L, b)
        x = np.linalg.solve(self.L.T, t)
        if self.perm is None:
            return x
        out = np.empty_like(x)
        out[self.perm] = x
        return out


class IpoptDense:
    """Dense restatement of IPOPT on the reference single-shooting NLP."""

    def __init__(self, prob: Problem, opts=None, la_variant=0):
        """la_variant (parity diagnostics only): 0 = the fixtures' linear algebra; 1..3 = the
        same Cholesky factorisation and solves with the variables symmetrically permuted
        (P M P^T, _Chol) -- mathematically the identical Newton step, different by
        rounding alone.  Running a step under both measures how far that
        step's result moves under rounding-level changes of the linear algebra
        (tests/golden/gen_rounding_spread.py)."""
        self.prob = prob
        self.la_variant = int(la_variant)
        o = dict(IPOPT_DEFAULTS)
        if opts:
            for k, v in opts.items():
                if k not in o:
                    raise KeyError(f"unknown IPOPT option {k}")
                o[k] = v
        self.o = o

    # ----- helpers -----------------------------------------------------------
    def _relax(self, b, sign):
        o = self.o
        fin = np.abs(b) < INF
        r = np.minimum(o["constr_viol_tol"], o["bound_relax_factor"] * np.maximum(1.0, np.abs(b)))
        out = b.copy()
        out[fin] = b[fin] + sign * r[fin]
        return out

    @staticmethod
    def _push(x, lo, hi, lm, um, kp, kf):
        """IPOPT DefaultIterateInitializer::push_variables."""
        x = x.copy()
        both = lm & um
        lo = np.where(lm, lo, 0.0)  # absent bounds never enter the arithmetic (no inf - inf)
        hi = np.where(um, hi, 0.0)
        pl = kp * np.maximum(1.0, np.abs(lo))
        pu = kp * np.maximum(1.0, np.abs(hi))
        span = np.where(both, hi - lo, np.inf)
        pl = np.minimum(pl, kf * span)
        pu = np.minimum(pu, kf * span)
        x = np.where(lm, np.maximum(x, lo + pl), x)
        x = np.where(um, np.minimum(x, hi - pu), x)
        return x

    def _evaluate(self, w):
        ev = SSEval(self.prob, w, self.p)
        return ev

    # ----- main entry --------------------------------------------------------
    def solve(self, x0, lbx, ubx, lbg, ubg, p, trace=False):
        prob, o = self.prob, self.o
        n, m = prob.nw, prob.ng
        self.p = np.asarray(p, float).ravel()
        lbx, ubx = np.asarray(lbx, float).ravel(), np.asarray(ubx, float).ravel()
        lbg, ubg = np.asarray(lbg, float).ravel(), np.asarray(ubg, float).ravel()
        w0 = np.asarray(x0, float).ravel()
        # equality rows (lbg == ubg): IPOPT's TNLPAdapter makes them c(x) = g(x) - g_l = 0,
        # with a multiplier and no slack, no bound multipliers and no bound relaxation.  Here
        # they keep a row slot whose "slack" is pinned at the (scaled) target, so d - s = c
        # enters theta, the residuals and the filter unchanged; the Newton step treats them
        # through the Schur complement of the augmented system (solve_dir).
        eq = (np.abs(lbg) < INF) & (lbg == ubg)
        neq = int(eq.sum())
        # fixed variables (lbx == ubx): IPOPT's default fixed_variable_treatment =
        # make_parameter (TNLPAdapter) removes them from the NLP -- held at the bound,
        # no bound multipliers, no step, excluded from the scaling maxima and the
        # error norms; their lam_x is 0 (IPOPT 3.12, the version CasADi 3.5.5 bundles)
        fixed = (np.abs(lbx) < INF) & (lbx == ubx)
        fr = ~fixed
        nf = int(fr.sum())
        # free-variable selection; a plain slice when nothing is fixed, so that case
        # runs the exact same array operations as without the feature
        F = slice(None) if nf == n else np.flatnonzero(fr)

        def sq(M_):
            return M_ if nf == n else M_[np.ix_(F, F)]
        w0 = np.where(fixed, lbx, w0)
        xlm, xum = (lbx > -INF) & fr, (ubx < INF) & fr
        slm, sum_ = (lbg > -INF) & ~eq, (ubg < INF) & ~eq
        xl, xu = self._relax(lbx, -1.0), self._relax(ubx, +1.0)
        gl_, gu_ = self._relax(lbg, -1.0), self._relax(ubg, +1.0)
        damp_xl = (xlm & ~xum).astype(float)
        damp_xu = (xum & ~xlm).astype(float)
        damp_sl = (slm & ~sum_).astype(float)
        damp_su = (sum_ & ~slm).astype(float)

        # gradient-based scaling at the user's starting point
        ev0 = self._evaluate(w0)
        if not (np.all(np.isfinite(ev0.gradF[F])) and np.all(np.isfinite(ev0.J[:, F]))):
            return self._result(w0, w0, 0, INVALID_NUMBER_DETECTED, 1.0, np.ones(m),
                                np.zeros(n), np.zeros(n), np.zeros(m), lbx, ubx, [])
        gmax = np.max(np.abs(ev0.gradF[F])) if nf else 0.0
        df = 1.0
        if gmax > o["nlp_scaling_max_gradient"]:
            df = o["nlp_scaling_max_gradient"] / gmax
        df = max(df, o["nlp_scaling_min_value"])
        rowmax = np.max(np.abs(ev0.J[:, F]), axis=1) if (m and nf) else np.zeros(m)
        dc = np.ones(m)
        if m and np.max(rowmax) > o["nlp_scaling_max_gradient"]:
            with np.errstate(divide="ignore"):
                dc = np.minimum(1.0, o["nlp_scaling_max_gradient"] / rowmax)
            dc = np.maximum(dc, o["nlp_scaling_min_value"])
        dl, du = dc * gl_, dc * gu_
        dl = np.where(slm, dl, -np.inf)
        du = np.where(sum_, du, np.inf)

        # initial point
        x = self._push(w0, xl, xu, xlm, xum, o["bound_push"], o["bound_frac"])
        ev = self._evaluate(x)
        s = self._push(dc * ev.g, dl, du, slm, sum_, o["slack_bound_push"], o["slack_bound_frac"])
        s = np.where(eq, dc * lbg, s)  # equality rows: pinned at the scaled target
        zl = np.where(xlm, o["bound_mult_init_val"], 0.0)
        zu = np.where(xum, o["bound_mult_init_val"], 0.0)
        vl = np.where(slm, o["bound_mult_init_val"], 0.0)
        vu = np.where(sum_, o["bound_mult_init_val"], 0.0)
        y = np.zeros(m)
        if o["constr_mult_init_max"] > 0 and m > 0:
            J = dc[:, None] * ev.J[:, F]
            bx = (df * ev.gradF - zl + zu)[F]
            bs = vu - vl
            y = ls_mults(J, bx, bs, eq)
            if np.max(np.abs(y)) > o["constr_mult_init_max"]:
                y = np.zeros(m)
        mu = o["mu_init"]
        tau = max(o["tau_min"], 1.0 - mu)

        nzx = int(xlm.sum() + xum.sum())
        nzs = int(slm.sum() + sum_.sum())

        def slacks(x_, s_):
            return (np.where(xlm, x_ - xl, 1.0), np.where(xum, xu - x_, 1.0),
                    np.where(slm, s_ - dl, 1.0), np.where(sum_, du - s_, 1.0))

        def barrier_obj(f_, x_, s_, mu_):
            Sxl, Sxu, Ssl, Ssu = slacks(x_, s_)
            val = f_
            # a trial slack that rounds to exactly 0 gives log 0 = -inf: phi is then not
            # finite and the trial counts as an evaluation error (as on the device)
            with np.errstate(divide="ignore"):
                val -= mu_ * (np.sum(np.log(Sxl[xlm])) + np.sum(np.log(Sxu[xum]))
                              + np.sum(np.log(Ssl[slm])) + np.sum(np.log(Ssu[sum_])))
            val += o["kappa_d"] * mu_ * (np.dot(damp_xl, Sxl * xlm) + np.dot(damp_xu, Sxu * xum)
                                         + np.dot(damp_sl, Ssl * slm) + np.dot(damp_su, Ssu * sum_))
            return val

        def grad_lag(gf, J, y_, zl_, zu_, vl_, vu_):
            # the slack components exist for the inequality rows only
            return np.where(fr, gf + J.T @ y_ - zl_ + zu_, 0.0), np.where(eq, 0.0, -y_ - vl_ + vu_)

        def compl(x_, s_, zl_, zu_, vl_, vu_, mu_):
            Sxl, Sxu, Ssl, Ssu = slacks(x_, s_)
            parts = [(Sxl * zl_ - mu_)[xlm], (Sxu * zu_ - mu_)[xum],
                     (Ssl * vl_ - mu_)[slm], (Ssu * vu_ - mu_)[sum_]]
            return np.concatenate(parts) if parts else np.zeros(0)

        def err_scaling(y_, zl_, zu_, vl_, vu_):
            smax = o["s_max"]
            nd = m + nzx + nzs
            sd = (np.sum(np.abs(y_)) + np.sum(np.abs(zl_)) + np.sum(np.abs(zu_))
                  + np.sum(np.abs(vl_)) + np.sum(np.abs(vu_))) / nd if nd else 0.0
            sd = max(smax, sd) / smax
            nc = nzx + nzs
            sc = (np.sum(np.abs(zl_)) + np.sum(np.abs(zu_)) + np.sum(np.abs(vl_)) + np.sum(np.abs(vu_))) / nc if nc else 0.0
            sc = max(smax, sc) / smax
            return sd, sc

        def amax(v):
            return float(np.max(np.abs(v))) if v.size else 0.0

        def frac_to_bound(tau_, x_, s_, dx_, ds_):
            Sxl, Sxu, Ssl, Ssu = slacks(x_, s_)
            a = 1.0
            for S, dS, msk in ((Sxl, dx_, xlm), (Sxu, -dx_, xum), (Ssl, ds_, slm), (Ssu, -ds_, sum_)):
                sel = msk & (dS < 0)
                if np.any(sel):
                    a = min(a, float(np.min(-tau_ * S[sel] / dS[sel])))
            return a

        def dual_frac_to_bound(tau_, zl_, zu_, vl_, vu_, dzl, dzu, dvl, dvu):
            a = 1.0
            for z_, dz_, msk in ((zl_, dzl, xlm), (zu_, dzu, xum), (vl_, dvl, slm), (vu_, dvu, sum_)):
                sel = msk & (dz_ < 0)
                if np.any(sel):
                    a = min(a, float(np.min(-tau_ * z_[sel] / dz_[sel])))
            return a

        # state of the algorithm
        f = df * ev.F
        d = dc * ev.g
        gf = df * ev.gradF
        J = dc[:, None] * ev.J
        filt = []  # list of (phi, theta)
        theta_max = theta_min = None
        delta_last, delta_curr = 0.0, 0.0
        in_soft_resto, soft_resto_counter = False, 0
        tiny_step_flag = False
        mu_initialized = False
        acc_counter = 0
        last_obj, curr_obj, last_obj_iter = -1e50, -1e50, -1
        it = 0
        tr = []
        self.chk = []
        status = None
        acc_point = None
        # watchdog procedure (BacktrackingLineSearch): successive shortened steps,
        # active flag, trial iterations, the stored point / step / reference values
        wd_cnt, in_wd, wd_trial, wd_point, wd_alpha = 0, False, 0, None, 1.0
        self.wd_events = {"start": 0, "stop": 0, "success": 0, "resto_start": 0, "resto_stop": 0}
        self.wd_stop_its = []  # main-phase iterations whose line search ran after StopWatchDog
        wd_trigger, wd_max = o["watchdog_shortened_iter_trigger"], o["watchdog_trial_iter_max"]

        def nlp_error(x_, s_, d_, gf_, J_, y_, zl_, zu_, vl_, vu_):
            sd, sc = err_scaling(y_, zl_, zu_, vl_, vu_)
            glx, gls = grad_lag(gf_, J_, y_, zl_, zu_, vl_, vu_)
            dinf = max(amax(glx), amax(gls))
            cviol = amax(np.concatenate([np.maximum(0.0, dl - d_)[slm], np.maximum(0.0, d_ - du)[sum_],
                                         np.abs(d_ - s_)[eq]]))
            cmp = amax(compl(x_, s_, zl_, zu_, vl_, vu_, 0.0))
            return max(dinf / sd, cviol, cmp / sc), dinf, cviol, cmp

        def barrier_error(x_, s_, d_, gf_, J_, y_, zl_, zu_, vl_, vu_, mu_):
            sd, sc = err_scaling(y_, zl_, zu_, vl_, vu_)
            glx, gls = grad_lag(gf_, J_, y_, zl_, zu_, vl_, vu_)
            dinf = max(amax(glx), amax(gls))
            return max(dinf / sd, amax(d_ - s_), amax(compl(x_, s_, zl_, zu_, vl_, vu_, mu_)) / sc)

        def pd_error(x_, s_, d_, gf_, J_, y_, zl_, zu_, vl_, vu_, mu_):
            glx, gls = grad_lag(gf_, J_, y_, zl_, zu_, vl_, vu_)
            dual = (np.sum(np.abs(glx)) + np.sum(np.abs(gls))) / (nf + m - neq)
            prim = np.sum(np.abs(d_ - s_)) / m if m else 0.0
            nc = nzx + nzs
            cm = np.sum(np.abs(compl(x_, s_, zl_, zu_, vl_, vu_, mu_))) / nc if nc else 0.0
            return dual + prim + cm

        def restoration(x0_, s0_, d0_, ev0_, y0_, zl0_, zu0_, vl0_, vu0_, mu0_, tau0_, theta0_, phi0_,
                        ofilt, it_, trace_, tr_):
            """IPOPT's feasibility restoration phase (Waechter & Biegler 2006, sec. 3.3;
            RestoMinC_1Nrm, RestoIpoptNLP, RestoIterateInitializer, RestoConvergenceCheck)
            on the scaled problem:  min  rho*sum(p+n) + eta/2*|D_R (x - x_R)|^2,
            eta = resto_proximity_weight*sqrt(mu_R), D_R = diag(1/max(1,|x_R|)),
            s.t. d(x) - p + n = s, s in [d_L, d_U], x in [x_L, x_U], p, n >= 0.
            p and n are eliminated row by row from the Newton system, which keeps the
            stage structure: each row gets the weight D~ = D/(1 + D(1/Sp + 1/Sn))."""
            rho = o["resto_penalty_parameter"]
            xR = x0_.copy()
            DR2 = (1.0 / np.maximum(1.0, np.abs(xR))) ** 2
            c0 = d0_ - s0_
            muR = max(mu0_, amax(c0))
            tauR = max(o["tau_min"], 1.0 - muR)
            # initial n, p: minimiser of rho(p+n) - mu ln p - mu ln n s.t. p - n = c, i.e. the
            # positive root of n^2 - 2a n - b = 0 (RestoIterateInitializer's solve_quadratic)
            qa = muR / (2.0 * rho) - 0.5 * c0
            qb = c0 * muR / (2.0 * rho)
            nn = qa + np.sqrt(qa * qa + qb)
            pp = c0 + nn
            xR_, sR = x0_.copy(), s0_.copy()
            zlR = np.where(xlm, np.minimum(rho, zl0_), 0.0)
            zuR = np.where(xum, np.minimum(rho, zu0_), 0.0)
            vlR = np.where(slm, np.minimum(rho, vl0_), 0.0)
            vuR = np.where(sum_, np.minimum(rho, vu0_), 0.0)
            zp, zn = muR / pp, muR / nn
            evR = ev0_
            dR = d0_
            JR = dc[:, None] * evR.J

            def eta(mu_):
                return o["resto_proximity_weight"] * math.sqrt(mu_)

            # least-squares multipliers of the restoration NLP (constr_mult_init_max)
            yR = np.zeros(m)
            if o["constr_mult_init_max"] > 0 and m > 0:
                Jfull = np.hstack([JR[:, F], -np.eye(m), np.eye(m)])
                bx = np.concatenate([(eta(muR) * DR2 * (xR_ - xR) - zlR + zuR)[F], rho - zp, rho - zn])
                bs = vuR - vlR
                yR = ls_mults(Jfull, bx, bs, eq)
                if np.max(np.abs(yR)) > o["constr_mult_init_max"]:
                    yR = np.zeros(m)
            nzp = 2 * m  # p, n: lower bounds only

            def fR(x_, p_, n_, mu_):
                dd = x_ - xR
                return rho * float(np.sum(p_ + n_)) + 0.5 * eta(mu_) * float(np.sum(DR2 * dd * dd))

            def phiR(x_, s_, p_, n_, mu_):
                Sxl, Sxu, Ssl, Ssu = slacks(x_, s_)
                val = fR(x_, p_, n_, mu_)
                with np.errstate(divide="ignore"):  # log 0 = -inf -> evaluation error (barrier_obj)
                    val -= mu_ * (np.sum(np.log(Sxl[xlm])) + np.sum(np.log(Sxu[xum]))
                                  + np.sum(np.log(Ssl[slm])) + np.sum(np.log(Ssu[sum_]))
                                  + np.sum(np.log(p_)) + np.sum(np.log(n_)))
                val += o["kappa_d"] * mu_ * (np.dot(damp_xl, Sxl * xlm) + np.dot(damp_xu, Sxu * xum)
                                             + np.dot(damp_sl, Ssl * slm) + np.dot(damp_su, Ssu * sum_)
                                             + np.sum(p_) + np.sum(n_))
                return val

            def thetaR(d_, s_, p_, n_):
                return float(np.sum(np.abs(d_ - s_ - p_ + n_)))

            def errR(x_, s_, d_, J_, p_, n_, y_, zl_, zu_, vl_, vu_, zp_, zn_, mu_, mu_c):
                """(overall error, dual inf, constraint violation, complementarity) of the resto NLP."""
                glx = np.where(fr, eta(mu_) * DR2 * (x_ - xR) + J_.T @ y_ - zl_ + zu_, 0.0)
                gls = np.where(eq, 0.0, -y_ - vl_ + vu_)
                glp, gln = rho - y_ - zp_, rho + y_ - zn_
                dinf_ = max(amax(glx), amax(gls), amax(glp), amax(gln))
                dr = d_ - p_ + n_
                cv = amax(np.concatenate([np.maximum(0.0, dl - dr)[slm], np.maximum(0.0, dr - du)[sum_],
                                          np.abs(dr - s_)[eq]]))
                cm = amax(np.concatenate([compl(x_, s_, zl_, zu_, vl_, vu_, mu_c), p_ * zp_ - mu_c, n_ * zn_ - mu_c]))
                smax = o["s_max"]
                nd = m + nzx + nzs + nzp
                sd = (np.sum(np.abs(y_)) + np.sum(np.abs(zl_)) + np.sum(np.abs(zu_)) + np.sum(np.abs(vl_))
                      + np.sum(np.abs(vu_)) + np.sum(np.abs(zp_)) + np.sum(np.abs(zn_))) / nd
                sd = max(smax, sd) / smax
                nc = nzx + nzs + nzp
                sc = (np.sum(np.abs(zl_)) + np.sum(np.abs(zu_)) + np.sum(np.abs(vl_)) + np.sum(np.abs(vu_))
                      + np.sum(np.abs(zp_)) + np.sum(np.abs(zn_))) / nc
                sc = max(smax, sc) / smax
                return max(dinf_ / sd, cv, cm / sc), dinf_, cv, cm, sd, sc, amax(d_ - s_ - p_ + n_)

            def ftb_R(tau_, x_, s_, p_, n_, dx_, ds_, dp_, dn_):
                a = frac_to_bound(tau_, x_, s_, dx_, ds_)
                for S, dS in ((p_, dp_), (n_, dn_)):
                    sel = dS < 0
                    if np.any(sel):
                        a = min(a, float(np.min(-tau_ * S[sel] / dS[sel])))
                return a

            def dftb_R(tau_, zl_, zu_, vl_, vu_, zp_, zn_, st):
                a = dual_frac_to_bound(tau_, zl_, zu_, vl_, vu_, st[4], st[5], st[6], st[7])
                for z_, dz_ in ((zp_, st[8]), (zn_, st[9])):
                    sel = dz_ < 0
                    if np.any(sel):
                        a = min(a, float(np.min(-tau_ * z_[sel] / dz_[sel])))
                return a

            rfilt = []
            th_max = th_min = None
            dlast, dcurr = 0.0, 0.0
            first = True
            racc, rlast_obj, rcurr_obj, rlast_it = 0, -1e50, -1e50, -1
            rwd_cnt, rin_wd, rwd_trial, rwd_point, rwd_alpha = 0, False, 0, None, 1.0
            xx, ss = xR_, sR
            while True:
                # ---- progress w.r.t. the original problem (RestoConvergenceCheck)
                if not first:
                    th_o = float(np.sum(np.abs(dR - ss)))
                    f_o = df * evR.F
                    phi_o = barrier_obj(f_o, xx, ss, mu0_)
                    if th_o <= o["required_infeasibility_reduction"] * theta0_ and np.isfinite(phi_o):
                        ok = (_compare_le(th_o, (1.0 - o["gamma_theta"]) * theta0_, theta0_)
                              or _compare_le(phi_o - phi0_, -o["gamma_phi"] * theta0_, phi0_))
                        if ok and all(phi_o <= fp or th_o <= ft for fp, ft in ofilt):
                            break
                # ---- the restoration NLP's own termination
                err_r, dinf_r, cv_r, cm_r, sd_r, sc_r, _ = errR(xx, ss, dR, JR, pp, nn, yR, zlR, zuR, vlR, vuR, zp,
                                                                zn, muR, 0.0)
                if trace_:  # the restoration NLP's own check (the kernel's trace: negative error)
                    self.chk.append(dict(it=it_, err=err_r, dinf=dinf_r / sd_r, cviol=cv_r, cmp=cm_r / sc_r,
                                         resto=True))
                if not np.isfinite(err_r):
                    return dict(status=INVALID_NUMBER_DETECTED, it=it_, x=xx)
                conv = (err_r <= o["tol"] and dinf_r <= o["dual_inf_tol"] and cv_r <= o["constr_viol_tol"]
                        and cm_r <= o["compl_inf_tol"])
                if it_ != rlast_it:
                    rlast_obj, rcurr_obj, rlast_it = rcurr_obj, fR(xx, pp, nn, muR), it_
                racc_ok = (err_r <= o["acceptable_tol"] and dinf_r <= o["acceptable_dual_inf_tol"]
                           and cv_r <= o["acceptable_constr_viol_tol"] and cm_r <= o["acceptable_compl_inf_tol"]
                           and abs(rcurr_obj - rlast_obj) / max(1.0, abs(rcurr_obj)) <= o["acceptable_obj_change_tol"])
                if o["acceptable_iter"] > 0 and racc_ok:
                    racc += 1
                else:
                    racc = 0
                if conv or (o["acceptable_iter"] > 0 and racc >= o["acceptable_iter"]):
                    # converged restoration problem: original infeasibility not reducible
                    if cviol_unscaled(dR, dc, gl_, gu_, slm, sum_, eq, lbg) > o["constr_viol_tol"]:
                        return dict(status=INFEASIBLE_PROBLEM_DETECTED, it=it_, x=xx)
                    break
                if it_ >= o["max_iter"]:
                    return dict(status=MAXIMUM_ITERATIONS_EXCEEDED, it=it_, x=xx)
                first = False
                # ---- monotone barrier update of the restoration problem
                def sub_err(mu_):
                    e_, _, _, _, sd_, sc_, pinf_ = errR(xx, ss, dR, JR, pp, nn, yR, zlR, zuR, vlR, vuR, zp, zn,
                                                        mu_, mu_)
                    glx = np.where(fr, eta(mu_) * DR2 * (xx - xR) + JR.T @ yR - zlR + zuR, 0.0)
                    gls = np.where(eq, 0.0, -yR - vlR + vuR)
                    dinf_ = max(amax(glx), amax(gls), amax(rho - yR - zp), amax(rho + yR - zn))
                    cm_ = amax(np.concatenate([compl(xx, ss, zlR, zuR, vlR, vuR, mu_), pp * zp - mu_,
                                               nn * zn - mu_]))
                    return max(dinf_ / sd_, pinf_, cm_ / sc_)
                se = sub_err(muR)
                done = False
                while se <= o["barrier_tol_factor"] * muR and not done:
                    new_mu = min(o["kappa_mu"] * muR, muR ** o["theta_mu"])
                    new_mu = max(new_mu, min(o["tol"], o["compl_inf_tol"]) / (o["barrier_tol_factor"] + 1.0))
                    changed = new_mu != muR
                    muR = new_mu
                    tauR = max(o["tau_min"], 1.0 - muR)
                    if not changed:
                        done = True
                    else:
                        se = sub_err(muR)
                        done = se > o["barrier_tol_factor"] * muR
                    if done and changed:
                        rfilt = []
                # ---- Newton step (p, n eliminated per row)
                Sxl, Sxu, Ssl, Ssu = slacks(xx, ss)
                SigX = np.where(xlm, zlR / Sxl, 0.0) + np.where(xum, zuR / Sxu, 0.0)
                SigS = np.where(slm, vlR / Ssl, 0.0) + np.where(sum_, vuR / Ssu, 0.0)
                Sp, Sn = zp / pp, zn / nn
                et = eta(muR)
                gphi = (et * DR2 * (xx - xR) - np.where(xlm, muR / Sxl, 0.0) + np.where(xum, muR / Sxu, 0.0)
                        + o["kappa_d"] * muR * (damp_xl - damp_xu))
                rs_ = (-yR - np.where(slm, muR / Ssl, 0.0) + np.where(sum_, muR / Ssu, 0.0)
                       + o["kappa_d"] * muR * (damp_sl - damp_su))
                rp = rho - yR - muR / pp + o["kappa_d"] * muR
                rn = rho + yR - muR / nn + o["kappa_d"] * muR
                cR = dR - ss - pp + nn
                Wr = evR.hessian(0.0, dc * yR) + np.diag(et * DR2)
                if dcurr > 0:
                    dlast = dcurr
                delta_ = 0.0
                fact = None
                while True:
                    D_ = SigS + delta_
                    Spd, Snd = Sp + delta_, Sn + delta_
                    Dt = D_ / (1.0 + D_ * (1.0 / Spd + 1.0 / Snd))
                    Dt = np.where(eq, 1.0 / (1.0 / Spd + 1.0 / Snd), Dt)  # equality rows: D = inf
                    # row weight D~ = (1/D + 1/Sp + 1/Sn)^-1 (p, n eliminated); written
                    # without 1/D so rows with no bound (D = 0) stay finite
                    M = Wr + np.diag(SigX + delta_) + JR.T @ (Dt[:, None] * JR)
                    try:
                        fact = _Chol(sq(M), self.la_variant)
                        break
                    except np.linalg.LinAlgError:
                        if delta_ == 0.0:
                            delta_ = (o["first_hessian_perturbation"] if dlast == 0.0
                                      else max(o["min_hessian_perturbation"], dlast * o["perturb_dec_fact"]))
                        else:
                            if dlast == 0.0 or 1e5 * dlast < delta_:
                                delta_ *= o["perturb_inc_fact_first"]
                            else:
                                delta_ *= o["perturb_inc_fact"]
                        if delta_ > o["max_hessian_perturbation"]:
                            fact = None
                            break
                dcurr = delta_
                if fact is None:
                    return dict(status=ERROR_IN_STEP_COMPUTATION, it=it_, x=xx)
                D_ = SigS + delta_
                Spd, Snd = Sp + delta_, Sn + delta_
                den = 1.0 / (1.0 + D_ * (1.0 / Spd + 1.0 / Snd))
                Dt = D_ * den
                den = np.where(eq, 0.0, den)  # equality rows (no slack): the D -> inf limit
                Dt = np.where(eq, 1.0 / (1.0 / Spd + 1.0 / Snd), Dt)

                def rdir(c_):
                    # dy = D~ (J dx + c + rs/D + rp/Sp - rn/Sn), with D~ rs/D = rs * den
                    Dr = Dt * (c_ + rp / Spd - rn / Snd) + rs_ * den
                    rhs = -(gphi + JR.T @ (yR + Dr))
                    dx_ = np.zeros(n)
                    dx_[F] = fact.solve(rhs[F])
                    jd = JR @ dx_
                    dy_ = Dt * jd + Dr
                    dp_ = (dy_ - rp) / Spd
                    dn_ = (-dy_ - rn) / Snd
                    ds_ = np.where(eq, 0.0, jd + c_ - dp_ + dn_)  # linearised d(x) - s - p + n = 0
                    dzl_ = np.where(xlm, muR / Sxl - zlR - zlR / Sxl * dx_, 0.0)
                    dzu_ = np.where(xum, muR / Sxu - zuR + zuR / Sxu * dx_, 0.0)
                    dvl_ = np.where(slm, muR / Ssl - vlR - vlR / Ssl * ds_, 0.0)
                    dvu_ = np.where(sum_, muR / Ssu - vuR + vuR / Ssu * ds_, 0.0)
                    dzp_ = muR / pp - zp - Sp * dp_
                    dzn_ = muR / nn - zn - Sn * dn_
                    return dx_, ds_, dy_, dp_, dzl_, dzu_, dvl_, dvu_, dzp_, dzn_, dn_

                stp = rdir(cR)
                # ---- filter line search on the restoration problem
                th_ref = thetaR(dR, ss, pp, nn)
                ph_ref = phiR(xx, ss, pp, nn, muR)
                gphi_s = (-np.where(slm, muR / Ssl, 0.0) + np.where(sum_, muR / Ssu, 0.0)
                          + o["kappa_d"] * muR * (damp_sl - damp_su))
                gpn_p = rho - muR / pp + o["kappa_d"] * muR
                gpn_n = rho - muR / nn + o["kappa_d"] * muR
                gbd = float(np.dot(gphi, stp[0]) + np.dot(gphi_s, stp[1]) + np.dot(gpn_p, stp[3])
                            + np.dot(gpn_n, stp[10]))
                if th_max is None:
                    th_max = o["theta_max_fact"] * max(1.0, th_ref)
                    th_min = o["theta_min_fact"] * max(1.0, th_ref)

                def r_ftype(a):
                    return gbd < 0.0 and a * (-gbd) ** o["s_phi"] > o["delta"] * th_ref ** o["s_theta"]

                def r_armijo(a, ph):
                    return _compare_le(ph - ph_ref, o["eta_phi"] * a * gbd, ph_ref)

                def r_acc_iter(ph, th):
                    if ph > ph_ref:
                        basval = 1.0
                        if abs(ph_ref) > 10.0:
                            basval = math.log10(abs(ph_ref))
                        if math.log10(ph - ph_ref) > o["obj_max_inc"] + basval:
                            return False
                    return (_compare_le(th, (1.0 - o["gamma_theta"]) * th_ref, th_ref)
                            or _compare_le(ph - ph_ref, -o["gamma_phi"] * th_ref, ph_ref))

                def r_check(a_test, ph, th):
                    if th > th_max:
                        return False
                    if a_test > 0.0 and r_ftype(a_test) and th_ref <= th_min:
                        ok = r_armijo(a_test, ph)
                    else:
                        ok = r_acc_iter(ph, th)
                    return ok and all(ph <= fp or th <= ft for fp, ft in rfilt)

                def r_trial(a, st):
                    xt, s_t = xx + a * st[0], ss + a * st[1]
                    pt, nt = pp + a * st[3], nn + a * st[10]
                    evt = self._evaluate(xt)
                    dtt = dc * evt.g
                    if not np.all(np.isfinite(dtt)):
                        return None
                    ph = phiR(xt, s_t, pt, nt, muR)
                    if not np.isfinite(ph):
                        return None
                    return xt, s_t, pt, nt, evt, dtt, ph, thetaR(dtt, s_t, pt, nt)

                def r_line_search(skip_first):
                    """DoBacktrackingLineSearch of the restoration NLP on `stp` (see the main
                    loop's line_search): (accepted, n_steps, a_test, eval_error, first trial)."""
                    amax_p = ftb_R(tauR, xx, ss, pp, nn, stp[0], stp[1], stp[3], stp[10])
                    if rin_wd:
                        tri = r_trial(amax_p, stp)
                        if tri is not None and r_check(rwd_alpha, tri[6], tri[7]):
                            return (amax_p, stp, tri), 0, rwd_alpha, False, tri
                        return None, 0, rwd_alpha, tri is None, tri
                    amin = o["gamma_theta"]
                    if gbd < 0:
                        amin = min(o["gamma_theta"], o["gamma_phi"] * th_ref / (-gbd))
                        if th_ref <= th_min:
                            amin = min(amin, o["delta"] * th_ref ** o["s_theta"] / (-gbd) ** o["s_phi"])
                    amin *= o["alpha_min_frac"]
                    a = amax_p * (o["alpha_red_factor"] if skip_first else 1.0)
                    n_ = 0
                    while a > amin or n_ == 0:
                        tri = r_trial(a, stp)
                        if tri is not None and r_check(a, tri[6], tri[7]):
                            return (a, stp, tri), n_, a, False, None
                        if tri is not None and a == amax_p and th_ref <= tri[7] and o["max_soc"] > 0:
                            th_tr, th_old, a_soc, cms, cnt, cur = tri[7], 0.0, a, cR.copy(), 0, tri
                            while cnt < o["max_soc"] and (cnt == 0 or th_tr <= o["kappa_soc"] * th_old):
                                th_old = th_tr
                                cms = a_soc * cms + (cur[5] - cur[1] - cur[2] + cur[3])
                                st2 = rdir(cms)
                                a_soc = ftb_R(tauR, xx, ss, pp, nn, st2[0], st2[1], st2[3], st2[10])
                                cur = r_trial(a_soc, st2)
                                if cur is None:
                                    break
                                if r_check(a, cur[6], cur[7]):
                                    return (a_soc, st2, cur), n_, a, False, None
                                cnt += 1
                                th_tr = cur[7]
                        a *= o["alpha_red_factor"]
                        n_ += 1
                    return None, n_, a, False, None

                # ---- watchdog procedure of the restoration phase's own line search
                if wd_trigger > 0 and not rin_wd and rwd_cnt >= wd_trigger:
                    rwd_point = (xx, ss, pp, nn, evR, dR, JR, yR, zlR, zuR, vlR, vuR, zp, zn, stp,
                                 th_ref, ph_ref, gbd)
                    rwd_alpha = ftb_R(tauR, xx, ss, pp, nn, stp[0], stp[1], stp[3], stp[10])
                    rwd_trial, rin_wd = 0, True
                    self.wd_events["resto_start"] += 1
                if rin_wd:
                    th_ref, ph_ref, gbd = rwd_point[15], rwd_point[16], rwd_point[17]
                skip_first, forced = False, False
                while True:
                    acc, nsteps, a, ev_err, wtri = r_line_search(skip_first)
                    if not rin_wd:
                        break
                    if acc is not None:
                        rin_wd = False
                        break
                    rwd_trial += 1
                    if ev_err or rwd_trial > wd_max:
                        (xx, ss, pp, nn, evR, dR, JR, yR, zlR, zuR, vlR, vuR, zp, zn, stp,
                         th_ref, ph_ref, gbd) = rwd_point
                        rin_wd, rwd_cnt, skip_first = False, 0, True
                        self.wd_events["resto_stop"] += 1
                        continue
                    acc = (ftb_R(tauR, xx, ss, pp, nn, stp[0], stp[1], stp[3], stp[10]), stp, wtri)
                    forced = True
                    break
                if acc is None:  # no restoration inside the restoration phase
                    return dict(status=RESTORATION_FAILED, it=it_, x=xx)
                rwd_cnt = 0 if nsteps == 0 else rwd_cnt + 1
                a_acc, st, tri = acc
                if not forced and not (r_ftype(a) and r_armijo(a, tri[6])):
                    rfilt.append((ph_ref - o["gamma_phi"] * th_ref, (1.0 - o["gamma_theta"]) * th_ref))
                ad = dftb_R(tauR, zlR, zuR, vlR, vuR, zp, zn, st)
                xx, ss, pp, nn, evR, dR = tri[0], tri[1], tri[2], tri[3], tri[4], tri[5]
                yR = yR + a_acc * st[2]
                zlR, zuR = zlR + ad * st[4], zuR + ad * st[5]
                vlR, vuR = vlR + ad * st[6], vuR + ad * st[7]
                zp, zn = zp + ad * st[8], zn + ad * st[9]
                Sxl, Sxu, Ssl, Ssu = slacks(xx, ss)
                ks = o["kappa_sigma"]
                zlR = np.where(xlm, np.maximum(np.minimum(zlR, ks * muR / Sxl), muR / (ks * Sxl)), 0.0)
                zuR = np.where(xum, np.maximum(np.minimum(zuR, ks * muR / Sxu), muR / (ks * Sxu)), 0.0)
                vlR = np.where(slm, np.maximum(np.minimum(vlR, ks * muR / Ssl), muR / (ks * Ssl)), 0.0)
                vuR = np.where(sum_, np.maximum(np.minimum(vuR, ks * muR / Ssu), muR / (ks * Ssu)), 0.0)
                zp = np.maximum(np.minimum(zp, ks * muR / pp), muR / (ks * pp))
                zn = np.maximum(np.minimum(zn, ks * muR / nn), muR / (ks * nn))
                JR = dc[:, None] * evR.J
                it_ += 1
                if trace_:
                    tr_.append(dict(iter=it_, mu=muR, f=fR(xx, pp, nn, muR), theta=thetaR(dR, ss, pp, nn),
                                    delta=dcurr, alpha_p=a_acc, alpha_d=ad, ls=nsteps + 1, soc=False, resto=True))
            # ---- back to the original problem (RestoMinC_1Nrm::PerformRestoration)
            # bound multipliers: Newton step for complementarity with the primal change
            # over the whole restoration phase, fraction-to-boundary, reset if large
            Sxl0, Sxu0, Ssl0, Ssu0 = slacks(x0_, s0_)
            Sxl1, Sxu1, Ssl1, Ssu1 = slacks(xx, ss)

            def bstep(z_, S0, S1, msk):
                return np.where(msk, (mu0_ - z_ * (S1 - S0)) / S0 - z_, 0.0)

            dzl_ = bstep(zl0_, Sxl0, Sxl1, xlm)
            dzu_ = bstep(zu0_, Sxu0, Sxu1, xum)
            dvl_ = bstep(vl0_, Ssl0, Ssl1, slm)
            dvu_ = bstep(vu0_, Ssu0, Ssu1, sum_)
            ad = dual_frac_to_bound(tau0_, zl0_, zu0_, vl0_, vu0_, dzl_, dzu_, dvl_, dvu_)
            zl1, zu1 = zl0_ + ad * dzl_, zu0_ + ad * dzu_
            vl1, vu1 = vl0_ + ad * dvl_, vu0_ + ad * dvu_
            if max(amax(zl1), amax(zu1), amax(vl1), amax(vu1)) > o["bound_mult_reset_threshold"]:
                zl1, zu1 = np.where(xlm, 1.0, 0.0), np.where(xum, 1.0, 0.0)
                vl1, vu1 = np.where(slm, 1.0, 0.0), np.where(sum_, 1.0, 0.0)
            # constraint multipliers: least-squares estimate, ignored above
            # constr_mult_reset_threshold (default 0: always zero)
            y1 = np.zeros(m)
            if o["constr_mult_reset_threshold"] > 0 and m > 0:
                J1 = dc[:, None] * evR.J[:, F]
                bx = (df * evR.gradF - zl1 + zu1)[F]
                bs = vu1 - vl1
                wx = np.linalg.solve(np.eye(nf) + J1.T @ J1, bx + J1.T @ bs)
                y1 = bs - J1 @ wx
                if np.max(np.abs(y1)) > o["constr_mult_reset_threshold"]:
                    y1 = np.zeros(m)
            return dict(status=None, it=it_, x=xx, s=ss, ev=evR, y=y1, zl=zl1, zu=zu1, vl=vl1, vu=vu1)

        while True:
            # ---------------- convergence check ----------------
            err, dinf, cviol, cmp = nlp_error(x, s, d, gf, J, y, zl, zu, vl, vu)
            if not np.isfinite(err):
                status = INVALID_NUMBER_DETECTED
                break
            u_dinf, u_cviol, u_cmp = dinf / df, cviol_unscaled(d, dc, gl_, gu_, slm, sum_, eq, lbg), cmp / df
            if trace:  # the convergence check's quantities (parity diagnostics: which test decided)
                sd_, sc_ = err_scaling(y, zl, zu, vl, vu)
                self.chk.append(dict(it=it, err=err, dinf=dinf / sd_, cviol=cviol, cmp=cmp / sc_, f=f))
            if (err <= o["tol"] and u_dinf <= o["dual_inf_tol"] and u_cviol <= o["constr_viol_tol"]
                    and u_cmp <= o["compl_inf_tol"]):
                status = SOLVE_SUCCEEDED
                break
            if it != last_obj_iter:
                last_obj, curr_obj, last_obj_iter = curr_obj, f, it
            acceptable = (err <= o["acceptable_tol"] and u_dinf <= o["acceptable_dual_inf_tol"]
                          and u_cviol <= o["acceptable_constr_viol_tol"]
                          and u_cmp <= o["acceptable_compl_inf_tol"]
                          and abs(curr_obj - last_obj) / max(1.0, abs(curr_obj)) <= o["acceptable_obj_change_tol"])
            if o["acceptable_iter"] > 0 and acceptable:
                acc_counter += 1
                if acc_counter >= o["acceptable_iter"]:
                    status = SOLVED_TO_ACCEPTABLE_LEVEL
                    break
            else:
                acc_counter = 0
            if it >= o["max_iter"]:
                status = MAXIMUM_ITERATIONS_EXCEEDED
                break
            if acceptable:  # BacktrackingLineSearch::StoreAcceptablePoint
                acc_point = (x.copy(), zl.copy(), zu.copy(), y.copy())

            # ---------------- barrier parameter update ----------------
            sub_err = barrier_error(x, s, d, gf, J, y, zl, zu, vl, vu, mu)
            done = False
            tsf = tiny_step_flag
            while (sub_err <= o["barrier_tol_factor"] * mu or tsf) and not done:
                new_mu = min(o["kappa_mu"] * mu, mu ** o["theta_mu"])
                new_mu = max(new_mu, min(o["tol"], o["compl_inf_tol"]) / (o["barrier_tol_factor"] + 1.0))
                changed = new_mu != mu
                if not changed and tsf:
                    status = SEARCH_DIRECTION_TOO_SMALL
                    break
                mu = new_mu
                tau = max(o["tau_min"], 1.0 - mu)
                if not changed:
                    done = True
                else:
                    sub_err = barrier_error(x, s, d, gf, J, y, zl, zu, vl, vu, mu)
                    done = sub_err > o["barrier_tol_factor"] * mu
                if done and changed:
                    filt = []
                    in_soft_resto = False
                tsf = False
            if status is not None:
                break
            mu_initialized = True
            tiny_step_flag = False

            # ---------------- search direction ----------------
            Sxl, Sxu, Ssl, Ssu = slacks(x, s)
            SigX = np.where(xlm, zl / Sxl, 0.0) + np.where(xum, zu / Sxu, 0.0)
            SigS = np.where(slm, vl / Ssl, 0.0) + np.where(sum_, vu / Ssu, 0.0)
            gphi = (gf - np.where(xlm, mu / Sxl, 0.0) + np.where(xum, mu / Sxu, 0.0)
                    + o["kappa_d"] * mu * (damp_xl - damp_xu))
            rs = (-y - np.where(slm, mu / Ssl, 0.0) + np.where(sum_, mu / Ssu, 0.0)
                  + o["kappa_d"] * mu * (damp_sl - damp_su))
            rd = d - s
            W = ev.hessian(df, dc * y)
            if delta_curr > 0:
                delta_last = delta_curr
            delta = 0.0
            fact = None
            while True:
                D = np.where(eq, 0.0, SigS + delta)
                M = W + np.diag(SigX + delta) + J.T @ (D[:, None] * J)
                try:
                    if neq:  # the augmented system's inertia (PDPerturbationHandler)
                        fact = eq_kkt(sq(M), J[eq][:, F], mu)
                        if fact is None:
                            raise np.linalg.LinAlgError("wrong inertia of the augmented system")
                    else:
                        fact = _Chol(sq(M), self.la_variant)
                    break
                except np.linalg.LinAlgError:
                    if delta == 0.0:
                        delta = (o["first_hessian_perturbation"] if delta_last == 0.0
                                 else max(o["min_hessian_perturbation"], delta_last * o["perturb_dec_fact"]))
                    else:
                        if delta_last == 0.0 or 1e5 * delta_last < delta:
                            delta *= o["perturb_inc_fact_first"]
                        else:
                            delta *= o["perturb_inc_fact"]
                    if delta > o["max_hessian_perturbation"]:
                        fact = None
                        break
            delta_curr = delta
            if fact is None:
                status = ERROR_IN_STEP_COMPUTATION
                break
            D = np.where(eq, 0.0, SigS + delta)

            def solve_dir(rd_):
                # equality rows contribute J_c^T y_c to the gradient, no slack elimination
                rhs = -(gphi + J.T @ np.where(eq, y, y + D * rd_ + rs))
                dx_ = np.zeros(n)
                dyc = None
                if neq:  # [M J_c^T; J_c -delta_c I] [dx; dy_c] = [rhs; -c]
                    sol = np.linalg.solve(fact, np.concatenate([rhs[F], -rd_[eq]]))
                    dx_[F], dyc = sol[:nf], sol[nf:]
                else:
                    dx_[F] = fact.solve(rhs[F])
                ds_ = np.where(eq, 0.0, J @ dx_ + rd_)
                dy_ = D * ds_ + rs
                if neq:
                    dy_[eq] = dyc
                dzl_ = np.where(xlm, mu / Sxl - zl - zl / Sxl * dx_, 0.0)
                dzu_ = np.where(xum, mu / Sxu - zu + zu / Sxu * dx_, 0.0)
                dvl_ = np.where(slm, mu / Ssl - vl - vl / Ssl * ds_, 0.0)
                dvu_ = np.where(sum_, mu / Ssu - vu + vu / Ssu * ds_, 0.0)
                return dx_, ds_, dy_, dzl_, dzu_, dvl_, dvu_

            dx, ds, dy, dzl, dzu, dvl, dvu = solve_dir(rd)

            # ---------------- line search ----------------
            theta_ref = float(np.sum(np.abs(rd)))
            phi_ref = barrier_obj(f, x, s, mu)
            gphi_s = (-np.where(slm, mu / Ssl, 0.0) + np.where(sum_, mu / Ssu, 0.0)
                      + o["kappa_d"] * mu * (damp_sl - damp_su))
            gBD = float(np.dot(gphi, dx) + np.dot(gphi_s, ds))
            if theta_max is None:
                theta_max = o["theta_max_fact"] * max(1.0, theta_ref)
                theta_min = o["theta_min_fact"] * max(1.0, theta_ref)

            def is_ftype(a):
                return gBD < 0.0 and a * (-gBD) ** o["s_phi"] > o["delta"] * theta_ref ** o["s_theta"]

            def armijo(a, phi_t):
                return _compare_le(phi_t - phi_ref, o["eta_phi"] * a * gBD, phi_ref)

            def acceptable_to_iterate(phi_t, th_t):
                if phi_t > phi_ref:
                    basval = 1.0
                    if abs(phi_ref) > 10.0:
                        basval = math.log10(abs(phi_ref))
                    if math.log10(phi_t - phi_ref) > o["obj_max_inc"] + basval:
                        return False
                return (_compare_le(th_t, (1.0 - o["gamma_theta"]) * theta_ref, theta_ref)
                        or _compare_le(phi_t - phi_ref, -o["gamma_phi"] * theta_ref, phi_ref))

            def filter_ok(phi_t, th_t):
                return all(phi_t <= fp or th_t <= ft for fp, ft in filt)

            def check_accept(a_test, phi_t, th_t):
                if th_t > theta_max:
                    return False
                if a_test > 0.0 and is_ftype(a_test) and theta_ref <= theta_min:
                    ok = armijo(a_test, phi_t)
                else:
                    ok = acceptable_to_iterate(phi_t, th_t)
                if not ok:
                    return False
                return filter_ok(phi_t, th_t)

            def trial(a, dx_, ds_):
                xt = x + a * dx_
                st = s + a * ds_
                evt = self._evaluate(xt)
                ft = df * evt.F
                dt = dc * evt.g
                if not (np.isfinite(ft) and np.all(np.isfinite(dt))):
                    return None
                phit = barrier_obj(ft, xt, st, mu)
                tht = float(np.sum(np.abs(dt - st)))
                if not np.isfinite(phit):
                    return None
                return xt, st, evt, ft, dt, phit, tht

            def try_soft_resto(step):
                dx_, ds_, dy_, dzl_, dzu_, dvl_, dvu_ = step
                ap = frac_to_bound(tau, x, s, dx_, ds_)
                ad = dual_frac_to_bound(tau, zl, zu, vl, vu, dzl_, dzu_, dvl_, dvu_)
                a = min(ap, ad)
                tri = trial(a, dx_, ds_)
                if tri is None:
                    return None
                xt, st, evt, ft, dt, phit, tht = tri
                yt, zlt, zut, vlt, vut = y + a * dy_, zl + a * dzl_, zu + a * dzu_, vl + a * dvl_, vu + a * dvu_
                gft, Jt = df * evt.gradF, dc[:, None] * evt.J
                e_t = pd_error(xt, st, dt, gft, Jt, yt, zlt, zut, vlt, vut, mu)
                e_c = pd_error(x, s, d, gf, J, y, zl, zu, vl, vu, mu)
                if e_t <= o["soft_resto_pderror_reduction_factor"] * e_c:
                    orig = check_accept(0.0, phit, tht)
                    return (a, a, xt, st, evt, ft, dt, yt, zlt, zut, vlt, vut, orig)
                return None

            def line_search(skip_first):
                """BacktrackingLineSearch::DoBacktrackingLineSearch on `step` from the
                current point.  Returns (accepted, n_steps, trials, soc, a_test, eval_error,
                first trial).  In the watchdog procedure only the full step is tried, with
                the watchdog's reference values and alpha test, and no SOC."""
                dx_, ds_ = step[0], step[1]
                amax_p = frac_to_bound(tau, x, s, dx_, ds_)
                if in_wd:
                    tri = trial(amax_p, dx_, ds_)
                    if tri is not None and check_accept(wd_alpha, tri[5], tri[6]):
                        return ("reg", amax_p, step, tri), 0, 1, False, wd_alpha, False, tri
                    return None, 0, 1, False, wd_alpha, tri is None, tri
                amin = o["gamma_theta"]
                if gBD < 0:
                    amin = min(o["gamma_theta"], o["gamma_phi"] * theta_ref / (-gBD))
                    if theta_ref <= theta_min:
                        amin = min(amin, o["delta"] * theta_ref ** o["s_theta"] / (-gBD) ** o["s_phi"])
                amin *= o["alpha_min_frac"]
                a = amax_p * (o["alpha_red_factor"] if skip_first else 1.0)
                n_ = 0
                trials = 0
                while a > amin or n_ == 0:
                    trials += 1
                    tri = trial(a, dx_, ds_)
                    if tri is not None and check_accept(a, tri[5], tri[6]):
                        return ("reg", a, step, tri), n_, trials, False, a, False, None
                    if tri is not None and a == amax_p and theta_ref <= tri[6] and o["max_soc"] > 0:
                        # second-order correction (FilterLSAcceptor::TrySecondOrderCorrection)
                        th_tr = tri[6]
                        th_old = 0.0
                        a_soc = a
                        dms = rd.copy()
                        cnt = 0
                        cur = tri
                        while cnt < o["max_soc"] and (cnt == 0 or th_tr <= o["kappa_soc"] * th_old):
                            th_old = th_tr
                            dms = a_soc * dms + (cur[4] - cur[1])
                            stp = solve_dir(dms)
                            a_soc = frac_to_bound(tau, x, s, stp[0], stp[1])
                            cur = trial(a_soc, stp[0], stp[1])
                            trials += 1
                            if cur is None:
                                break
                            if check_accept(a, cur[5], cur[6]):
                                return ("reg", a_soc, stp, cur), n_, trials, True, a, False, None
                            cnt += 1
                            th_tr = cur[6]
                    a *= o["alpha_red_factor"]
                    n_ += 1
                return None, n_, trials, False, a, False, None

            accepted = None
            ls_trials = 0
            soc_taken = False
            alpha_p = 0.0
            alpha_d = 0.0
            n_steps = 0
            # tiny step detection
            tiny = (amax(dx / (1.0 + np.abs(x))) <= o["tiny_step_tol"]
                    and amax(ds / (1.0 + np.abs(s))) <= o["tiny_step_tol"]
                    and amax(rd) <= 1e-4)
            step = (dx, ds, dy, dzl, dzu, dvl, dvu)
            # ---- watchdog procedure (BacktrackingLineSearch::FindAcceptableTrialPoint)
            if in_wd and tiny:
                # tiny step inside the watchdog: back to its stored point (StopWatchDog)
                x, s, y, zl, zu, vl, vu, ev, step, theta_ref, phi_ref, gBD = wd_point
                f, d, gf, J = df * ev.F, dc * ev.g, df * ev.gradF, dc[:, None] * ev.J
                in_wd, wd_cnt, tiny = False, 0, False
                self.wd_stop_its.append(it + 1)
            if wd_trigger > 0 and not in_wd and not tiny and not in_soft_resto and wd_cnt >= wd_trigger:
                # StartWatchDog: store the iterate, its step and the reference values
                wd_point = (x, s, y, zl, zu, vl, vu, ev, step, theta_ref, phi_ref, gBD)
                wd_alpha = frac_to_bound(tau, x, s, dx, ds)
                wd_trial, in_wd = 0, True
                self.wd_events["start"] += 1
            if in_wd:  # FilterLSAcceptor::InitThisLineSearch(in_watchdog)
                theta_ref, phi_ref, gBD = wd_point[9], wd_point[10], wd_point[11]
            wd_forced = False
            if in_soft_resto:
                soft_resto_counter += 1
                if soft_resto_counter <= o["max_soft_resto_iters"]:
                    r = try_soft_resto(step)
                    if r is not None:
                        accepted = ("soft",) + r
                        if r[-1]:
                            in_soft_resto = False
            elif tiny:
                a = frac_to_bound(tau, x, s, dx, ds)
                tri = trial(a, dx, ds)
                if tri is not None:
                    accepted = ("reg", a, step, tri)
                    tiny_step_flag = True
            else:
                skip_first = False
                while True:
                    accepted, n_steps, ntr, soc_taken, a_test, ev_err, wtri = line_search(skip_first)
                    ls_trials += ntr
                    if not in_wd:
                        break
                    if accepted is not None:  # watchdog procedure successful
                        in_wd = False
                        self.wd_events["success"] += 1
                        break
                    wd_trial += 1
                    if ev_err or wd_trial > wd_max:
                        # StopWatchDog: back to the stored point and step, then a regular
                        # backtracking search on it that skips the (already rejected) full step
                        x, s, y, zl, zu, vl, vu, ev, step, theta_ref, phi_ref, gBD = wd_point
                        f, d, gf, J = df * ev.F, dc * ev.g, df * ev.gradF, dc[:, None] * ev.J
                        in_wd, wd_cnt, skip_first = False, 0, True
                        self.wd_events["stop"] += 1
                        self.wd_stop_its.append(it + 1)
                        continue
                    # a watchdog trial iteration: the full step is taken unchecked
                    accepted = ("reg", frac_to_bound(tau, x, s, step[0], step[1]), step, wtri)
                    wd_forced = True
                    break
                if accepted is None:
                    r = try_soft_resto(step)
                    if r is not None:
                        accepted = ("soft",) + r
                        if not r[-1]:
                            in_soft_resto = True
                            soft_resto_counter = 0
                elif not wd_forced:
                    phi_acc = accepted[3][5]
                    if not (is_ftype(a_test) and armijo(a_test, phi_acc)):
                        filt.append((phi_ref - o["gamma_phi"] * theta_ref, (1.0 - o["gamma_theta"]) * theta_ref))
            if accepted is not None and accepted[0] == "reg":
                # successive shortened steps trigger the watchdog
                wd_cnt = 0 if n_steps == 0 else wd_cnt + 1

            if accepted is None:
                # feasibility restoration phase (BacktrackingLineSearch -> RestoMinC_1Nrm)
                if theta_ref <= 1e-2 * o["tol"]:
                    # called at an almost feasible point: return the last acceptable iterate
                    if acc_point is not None:
                        x, zl, zu, y = acc_point
                        status = SOLVED_TO_ACCEPTABLE_LEVEL
                    else:
                        status = RESTORATION_FAILED
                    break
                filt.append((phi_ref - o["gamma_phi"] * theta_ref, (1.0 - o["gamma_theta"]) * theta_ref))
                rres = restoration(x, s, d, ev, y, zl, zu, vl, vu, mu, tau, theta_ref, phi_ref, filt, it, trace, tr)
                it = rres["it"]
                if rres["status"] is not None:
                    status = rres["status"]
                    x = rres["x"]
                    break
                x, s, ev, y, zl, zu, vl, vu = (rres[k] for k in ("x", "s", "ev", "y", "zl", "zu", "vl", "vu"))
                f, d = df * ev.F, dc * ev.g
                in_soft_resto = False
                wd_cnt = 0
                accepted = ("resto",)

            if accepted[0] == "reg":
                _, alpha_p, stp, tri = accepted
                x, s, ev, f, d = tri[0], tri[1], tri[2], tri[3], tri[4]
                alpha_d = dual_frac_to_bound(tau, zl, zu, vl, vu, stp[3], stp[4], stp[5], stp[6])
                y = y + alpha_p * stp[2]
                zl, zu = zl + alpha_d * stp[3], zu + alpha_d * stp[4]
                vl, vu = vl + alpha_d * stp[5], vu + alpha_d * stp[6]
            elif accepted[0] == "soft":
                (_, alpha_p, alpha_d, x, s, ev, f, d, y, zl, zu, vl, vu, _) = accepted
            else:
                alpha_p = alpha_d = 1.0
            # kappa_sigma safeguard (IpoptAlgorithm::correct_bound_multiplier)
            Sxl, Sxu, Ssl, Ssu = slacks(x, s)
            ks = o["kappa_sigma"]
            zl = np.where(xlm, np.maximum(np.minimum(zl, ks * mu / Sxl), mu / (ks * Sxl)), 0.0)
            zu = np.where(xum, np.maximum(np.minimum(zu, ks * mu / Sxu), mu / (ks * Sxu)), 0.0)
            vl = np.where(slm, np.maximum(np.minimum(vl, ks * mu / Ssl), mu / (ks * Ssl)), 0.0)
            vu = np.where(sum_, np.maximum(np.minimum(vu, ks * mu / Ssu), mu / (ks * Ssu)), 0.0)
            gf = df * ev.gradF
            J = dc[:, None] * ev.J
            if accepted[0] != "resto":  # restoration iterations were counted as they ran
                it += 1
            if trace and accepted[0] != "resto":
                tr.append(dict(iter=it, mu=mu, f=f, theta=float(np.sum(np.abs(d - s))), delta=delta_curr,
                               alpha_p=alpha_p, alpha_d=alpha_d, ls=ls_trials, soc=soc_taken,
                               ymax=float(np.max(np.abs(y))) if len(y) else 0.0))

        return self._result(x, w0, it, status, df, dc, zl, zu, y, lbx, ubx, tr, mu=mu)

    def _result(self, x, w0, it, status, df, dc, zl, zu, y, lbx, ubx, tr, mu=None):
        prob = self.prob
        xf = np.minimum(np.maximum(x, lbx), ubx)  # honor_original_bounds
        ev = SSEval(prob, xf, self.p)
        X = ev.X
        return dict(x=xf, f=ev.F, g=ev.g, lam_x=(zu - zl) / df, lam_g=y * dc / df,
                    X=X, status=status, iter=it, trace=tr, df=df, dc=dc, mu=mu)


def cviol_unscaled(d, dc, gl_, gu_, slm, sum_, eq=None, gE=None):
    """Unscaled constraint violation (max norm) w.r.t. the relaxed bounds; equality rows
    (eq) by |g - g_E|."""
    g = d / dc
    parts = [np.maximum(0.0, gl_ - g)[slm], np.maximum(0.0, g - gu_)[sum_]]
    if eq is not None:
        parts.append(np.abs(g - gE)[eq])
    v = np.concatenate(parts)
    return float(np.max(v)) if v.size else 0.0


def ls_mults(J, bx, bs, eq):
    """IPOPT's least-squares constraint multipliers (LeastSquareMults): min |wx - bx|^2 +
    |ws - bs|^2 subject to J_d wx - ws = 0 (inequality rows, slack ws) and J_c wx = 0
    (equality rows); y = bs - J_d wx on the inequality rows (the sign convention of the
    plain formula (I + J^T J) wx = bx + J^T bs, y = bs - J wx, used when there are none)."""
    if not np.any(eq):
        wx = np.linalg.solve(np.eye(J.shape[1]) + J.T @ J, bx + J.T @ bs)
        return bs - J @ wx
    Jd, Jc = J[~eq], J[eq]
    nx, nc = J.shape[1], int(eq.sum())
    K = np.zeros((nx + nc, nx + nc))
    K[:nx, :nx] = np.eye(nx) + Jd.T @ Jd
    K[:nx, nx:] = -Jc.T
    K[nx:, :nx] = Jc
    y = np.zeros(J.shape[0])
    try:
        sol = np.linalg.solve(K, np.concatenate([bx + Jd.T @ bs[~eq], np.zeros(nc)]))
    except np.linalg.LinAlgError:  # rank-deficient J_c: IPOPT then starts from y = 0
        return y
    y[~eq] = bs[~eq] - Jd @ sol[:nx]
    y[eq] = sol[nx:]
    return y


def eq_kkt(M, Jc, mu, reg_value=1e-8, reg_exponent=0.25):
    """The augmented Newton matrix K = [M J_c^T; J_c -delta_c I] of a problem with
    equality rows (M: the condensed Hessian block, inequality rows eliminated) when its
    inertia is IPOPT's (n positive, m_c negative eigenvalues), else None.  By Haynsworth,
    inertia(K) = inertia(M) + inertia(-(S + delta_c I)), S = J_c M^-1 J_c^T, so with k
    negative eigenvalues of M the test is: S + delta_c I has exactly k negative ones (the
    kernel reads k from the signs of its Riccati pivots).  A singular S (rank-deficient
    J_c; eigenvalues below 1e-14 of its largest) gets IPOPT's delta_c =
    jacobian_regularization_value * mu^jacobian_regularization_exponent; a wrong inertia, a
    singular M or a still singular S returns None (the caller raises delta_w)."""
    evM = np.linalg.eigvalsh(M)
    if np.any(evM == 0.0):
        return None
    k = int(np.sum(evM < 0.0))
    S = Jc @ np.linalg.solve(M, Jc.T)
    mc = S.shape[0]
    for dcv in (0.0, reg_value * mu ** reg_exponent):
        ev = np.linalg.eigvalsh(S + dcv * np.eye(mc))
        scale = float(np.max(np.abs(ev)))
        if scale == 0.0 or np.any(np.abs(ev) <= 1e-14 * scale):
            continue
        if int(np.sum(ev < 0.0)) != k:
            return None
        return np.block([[M, Jc.T], [Jc, -dcv * np.eye(mc)]])
    return None


# --- closed loop (immediate caller, Python/NMPC_TT.py:13-30, :346-402) --------
def shift_timestep(prob, x0, u, xs, con_t=(12.0, 0.01)):
    """Plant Euler step with u[:,0], warm start shift, target unicycle step."""
    T = prob.T
    f = dynamics5 if prob.model == "uav5" else dynamics
    x0n = x0 + T * f(x0, u[:, 0])
    u0 = np.concatenate([u[:, 1:], u[:, -1:]], axis=1)
    v, w = con_t
    xsn = xs + T * np.array([v * math.cos(xs[2]), v * math.sin(xs[2]), w])
    return x0n, u0, xsn


def fov_centre(x0, vfov=1.0, hfov=1.0):
    """FOV centre of the current state (Python/NMPC_TT.py:397-400)."""
    a_p = (x0[2] * math.tan(x0[6] + vfov / 2) - x0[2] * math.tan(x0[6] - vfov / 2)) / 2
    b_p = (x0[2] * math.tan(x0[5] + hfov / 2) - x0[2] * math.tan(x0[5] - hfov / 2)) / 2
    return x0[0] + a_p + x0[2] * math.tan(x0[6] - vfov / 2), x0[1] + b_p + x0[2] * math.tan(x0[5] - hfov / 2)
