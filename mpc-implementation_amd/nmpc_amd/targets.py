"""Target (v, omega) schedules of the reference's closed-loop scripts.

Each reference script's ``shift_timestep`` picks the target's linear and
angular velocity ``con_t = [v, w]`` from the global MPC iteration counter
``mpc_iter`` with a chain of ``if mpc_iter >= k`` overrides, then steps the
target as a unicycle (xs <- xs + T [v cos(psi), v sin(psi), w]).  The tables
below are those chains as (first iteration, v, w) breakpoints; the unicycle
step itself runs on the device (nmpc_closed_loop_dev / nmpc_shift_dev).
"""
from __future__ import annotations

import math

import numpy as np

PI = math.pi

# name -> [(first mpc_iter, v, w), ...] in increasing order
SCHEDULES = {
    # Python/NMPC_TT.py:25
    "nmpc_tt": [(0, 12.0, 0.01)],
    # Python/10_obstacles.py:28-60
    "10_obstacles": [
        (0, 13.0, 0.0), (300, 13.0, -(PI / 2) / 24), (360, 13.0, 0.0), (410, 13.0, (PI / 2) / 24),
        (470, 13.0, 0.0), (570, 13.0, ((11 * PI) / 18) / 12), (630, 13.0, 0.0),
        (780, 13.0, ((7 * PI) / 18) / 12), (840, 13.0, 0.0), (940, 13.0, -(3 * PI / 18) / 12),
        (1000, 13.0, 0.0), (1100, 13.0, (3 * PI / 18) / 12), (1160, 13.0, 0.0),
        (1335, 13.0, (PI / 2) / 12), (1395, 13.0, 0.0), (1535, 13.0, (PI / 2) / 12),
    ],
    # Python/Race Track 2.py:28-36
    "race_track_2": [(0, 12.0, 0.0), (500, 12.0, PI / 100), (1000, 12.0, 0.0), (1500, 12.0, PI / 100)],
    # MATLAB/Dynamic Obstacles/shift1.m:9 (con_t = [15; 0.12] every step): the no-gimbal
    # NMPC_TT.m run and, by the reading in tests/golden/gen_reference_runs.py, the
    # Dynamic Obstacle avoidance.m run (whose shift1 call at :251 passes sc where
    # shift1.m expects the target)
    "matlab_nmpc_tt": [(0, 15.0, 0.12)],
    "dynamic_obstacles": [(0, 15.0, 0.12)],
    # the derived start of that script's problem (tests/golden/gen_reference_runs.py)
    "dynamic_obstacles_derived": [(0, 15.0, 0.12)],
    # Python/T_Trajectory.py:25-57
    "t_trajectory": [
        (0, 13.5, 0.0), (100, 13.5, (PI / 2) / 12), (160, 13.5, 0.0), (260, 13.5, -(PI / 2) / 12),
        (320, 13.5, 0.0), (420, 13.5, (PI / 2) / 12), (480, 13.5, 0.0), (580, 13.5, (PI / 2) / 12),
        (640, 13.5, 0.0), (740, 13.5, -(PI / 2) / 12), (800, 13.5, 0.0), (900, 13.5, (PI / 2) / 12),
        (960, 13.5, 0.0), (1060, 13.5, (PI / 2) / 12), (1120, 13.5, 0.0), (1573, 13.5, (PI / 2) / 12),
    ],
    # Python/Plus Trajectory.py:25-69 (one-step 90 degree turns every ~101 iterations)
    "plus_trajectory": [(0, 20.0, 0.0)] + [
        (k, 20.0, sgn * (PI / 2) * 5) if off == 0 else (k + 1, 20.0, 0.0)
        for k, sgn in ((101, 1), (203, -1), (305, 1), (407, 1), (509, -1), (611, 1), (713, 1),
                       (815, -1), (917, 1), (1019, 1), (1121, -1))
        for off in (0, 1)
    ],
}


def con_t(name: str, mpc_iter: int) -> tuple[float, float]:
    """(v, w) the named script uses in shift_timestep at iteration ``mpc_iter``."""
    v, w = SCHEDULES[name][0][1:]
    for k0, vk, wk in SCHEDULES[name]:
        if mpc_iter >= k0:
            v, w = vk, wk
    return v, w


def schedule(name: str, start_iter: int, K: int) -> tuple[np.ndarray, np.ndarray]:
    """(K,) arrays v[k], w[k] for MPC iterations start_iter .. start_iter+K-1
    (shared by every scenario: pass with ld_tb = 0)."""
    vw = np.array([con_t(name, start_iter + k) for k in range(K)], dtype=np.float64).reshape(K, 2)
    return np.ascontiguousarray(vw[:, 0]), np.ascontiguousarray(vw[:, 1])


# MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230: obstacle j's y
# coordinate (p[10 + j], j = 1..6) moves by +-1 m per MPC iteration inside a
# window (both ends exclusive), applied after args.p is formed (:211).
DYNAMIC_OBSTACLE_WINDOWS = [  # (obstacle j, mpciter > a, mpciter < b, step)
    (2, 100, 400, -1.0), (3, 200, 500, +1.0), (4, 300, 600, -1.0),
    (5, 500, 800, +1.0), (6, 600, 900, -1.0), (1, 1000, 1300, +1.0),
]


def obstacle_steps(start_iter: int, K: int, np_: int = 17) -> np.ndarray:
    """(K, np) increments added to p after MPC iterations start_iter ..
    start_iter+K-1 (p_step of nmpc_closed_loop_dev), dynamic-obstacle script."""
    out = np.zeros((K, np_))
    for k in range(K):
        it = start_iter + k
        for j, a, b, dy in DYNAMIC_OBSTACLE_WINDOWS:
            if a < it < b:
                out[k, 10 + j] += dy
    return out
