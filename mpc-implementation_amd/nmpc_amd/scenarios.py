"""Seeded synthetic scenarios.

One scenario = (x0, target xs, dynamic-obstacle ys) packed as the reference's
parameter vector p = [x0(8); xs(3)(; y_o1..y_o6)] (Python/NMPC_TT.py:350-353,
MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:128).  The stream is
drawn globally from ``default_rng(seed)`` and sliced per GPU, so results do not
depend on the number of ranks.
"""
from __future__ import annotations

import numpy as np

from .spec import ProblemSpec, THETA_U_MAX, Z_U_MIN, Z_U_MAX

# the reference's option dict (Python/NMPC_TT.py:257-265)
REFERENCE_OPTS = {"ipopt": {"max_iter": 100, "print_level": 0, "acceptable_tol": 1e-8,
                            "acceptable_obj_change_tol": 1e-6}, "print_time": 0}


def draw_scenarios(spec: ProblemSpec, B: int, seed: int) -> np.ndarray:
    """(B, np) parameter vectors.  Redraws any scenario whose stage-0 rows
    violate a bound or whose UAV is within obstacle clearance + 10 m (stage-0
    rows are constant in U)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((B, spec.np))
    ox = np.array([o.x for o in spec.obstacles])
    oy0 = np.array([o.y for o in spec.obstacles])
    rr = np.array([o.r for o in spec.obstacles])
    ydyn = np.array([o.y_pidx for o in spec.obstacles], dtype=int) if spec.n_obs else np.zeros(0, int)
    i = 0
    while i < B:
        xt, yt, pt = rng.uniform(-200, 1800), rng.uniform(-100, 1000), rng.uniform(-np.pi, np.pi)
        x0 = np.array([xt + rng.uniform(-30, 30), yt + rng.uniform(-30, 30), rng.uniform(80, 140),
                       rng.uniform(-0.2, 0.2), rng.uniform(-np.pi, np.pi), rng.uniform(-0.4, 0.4),
                       rng.uniform(-0.4, 0.4), rng.uniform(-1.4, 1.4)])
        p = np.zeros(spec.np)
        nx = spec.nx  # the no-gimbal model packs x0[:5] (same random stream)
        p[:nx], p[nx:nx + 3] = x0[:nx], (xt, yt, pt)
        oy = oy0.copy()
        if spec.np > spec.np_min:
            # dynamic obstacle ys: initial layout +- 300 m (the schedule moves them 300 m)
            for j in range(spec.n_obs):
                if ydyn[j] >= 0:
                    p[ydyn[j]] = oy0[j] + rng.uniform(-300, 300)
                    oy[j] = p[ydyn[j]]
        if not (Z_U_MIN < x0[2] < Z_U_MAX and abs(x0[3]) < THETA_U_MAX):
            continue
        if spec.n_obs and np.any(np.hypot(x0[0] - ox, x0[1] - oy) <= rr + 10.0):
            continue
        out[i] = p
        i += 1
    return out
