"""Problem specification for the batched NMPC solve step.

The reference defines its NLP symbolically in module globals
(``Python/NMPC_TT.py:56-313``); here the same problem is a frozen, structured
description that the C-ABI descriptor (``include/nmpc_amd.h::nmpc_desc``) is
built from.  Constants cite the reference lines they restate.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

PI = math.pi

# Python/NMPC_TT.py:61-89
V_U_MIN, V_U_MAX = 14.0, 30.0
OMEGA_2_U = PI / 30
OMEGA_3_U = PI / 21
OMEGA_G = PI / 30
THETA_U_MAX = 0.2618
Z_U_MIN, Z_U_MAX = 75.0, 150.0
PHI_G_MAX = PI / 6
THETA_G_MAX = PI / 6
SHI_G_MAX = PI / 2
UAV_R = 5.0  # Python/NMPC_TT.py:231

NX, NU = 8, 6  # states / controls (Python/NMPC_TT.py:105-136)

# Reference obstacle tables: (list of (x, y), obstacle radius)
LAYOUTS = {
    "nmpc_tt": ([(175, 820), (-134, 155), (441, 343)], 30.0),               # Python/NMPC_TT.py:224-230
    "10_obstacles": ([(500, 20), (1700, 197), (130, 830)] + [(10000, 10000)] * 7, 100.0),  # 10_obstacles.py:247-268
    "race_track_2": ([(0, 80), (500, 245), (1000, 70), (1500, 295), (1765, 550), (1500, 750),
                      (1000, 1005), (500, 800), (-100, 950), (-200, 550)], 50.0),          # Race Track 2.py:223-243
    "dynamic": ([(2500, 0), (0, 300), (500, 0), (1000, 300), (1500, 0), (2000, 300),
                 (1300, 1300), (1300, 1300), (1300, 1300), (1300, 1300)], 50.0),          # Dynamic Obstacle avoidance.m:98-119
}


@dataclass(frozen=True)
class Obstacle:
    x: float
    y: float
    r: float                 # UAV_r + obs_r (Python/NMPC_TT.py:241)
    x_pidx: int = -1         # -1 = constant, else index of p holding x
    y_pidx: int = -1


@dataclass(frozen=True)
class ProblemSpec:
    """Structured replacement of ``nlp_prob`` (Python/NMPC_TT.py:250-255)."""
    N: int = 15
    T: float = 1.0
    obstacles: tuple = field(default_factory=tuple)
    w1: float = 1.0
    w2: float = 2.0
    vfov: float = 1.0
    hfov: float = 1.0
    np: int = 11
    model: str = "uav8g"
    # cost weights from p (batched weight sweep): index into p or -1
    w1_pidx: int = -1
    w2_pidx: int = -1

    @property
    def n_obs(self) -> int:
        return len(self.obstacles)

    @property
    def nu(self) -> int:
        return 3 if self.model == "uav5" else NU

    @property
    def nx(self) -> int:
        return 5 if self.model == "uav5" else NX

    @property
    def nb(self) -> int:
        """box rows per stage: z, theta, x5, x6, x7 (:234-240) or z, theta (NMPC_TT.m:129-134)."""
        return 2 if self.model == "uav5" else 5

    @property
    def np_min(self) -> int:
        """length of [x0; xs]."""
        return self.nx + 3

    @property
    def m(self) -> int:
        """g rows per stage: box rows + one per obstacle (:234-244)."""
        return self.nb + self.n_obs

    @property
    def nw(self) -> int:
        return self.nu * self.N

    @property
    def ng(self) -> int:
        return self.m * (self.N + 1)

    @property
    def nX(self) -> int:
        return self.nx * (self.N + 1)

    def validate(self):
        if self.model not in ("uav8g", "uav5"):
            raise ValueError(f"unsupported model {self.model!r}")
        if not (1 <= self.N <= 63):
            raise ValueError("N must be in [1, 63]")
        if self.n_obs > 16:
            raise ValueError("at most 16 obstacles")
        if self.np < self.np_min:
            raise ValueError(f"np must be >= {self.np_min} (x0({self.nx}) + target(3))")
        for o in self.obstacles:
            for i in (o.x_pidx, o.y_pidx):
                if i != -1 and not (self.np_min <= i < self.np):
                    raise ValueError("obstacle parameter index out of range")
        for i in (self.w1_pidx, self.w2_pidx):
            if i != -1 and not (self.np_min <= i < self.np):
                raise ValueError("weight parameter index must be -1 or in [np_min, np)")
        if not self.T > 0:
            raise ValueError("T must be positive")
        return self

    def bounds(self):
        """lbx, ubx, lbg, ubg for this spec (Python/NMPC_TT.py:269-306).

        The reference hard-codes the strides for N=15 (``lbg[0:128:8]``,
        ``lbg[0:240:15]``); here stride and length follow (N, n_obs)
        (SURVEY F3), so any N gives a feasible bound set.
        """
        if self.model == "uav5":  # MATLAB/Dynamic Obstacles/NMPC_TT.m:140-149
            lbx = np.tile([V_U_MIN, -OMEGA_2_U, -OMEGA_3_U], self.N)
            ubx = np.tile([V_U_MAX, OMEGA_2_U, OMEGA_3_U], self.N)
            lrow = np.concatenate([[Z_U_MIN, -THETA_U_MAX], np.full(self.n_obs, -np.inf)])
            urow = np.concatenate([[Z_U_MAX, THETA_U_MAX], np.zeros(self.n_obs)])
            return lbx, ubx, np.tile(lrow, self.N + 1), np.tile(urow, self.N + 1)
        lbx = np.tile([V_U_MIN, -OMEGA_2_U, -OMEGA_3_U, -OMEGA_G, -OMEGA_G, -OMEGA_G], self.N)
        ubx = np.tile([V_U_MAX, OMEGA_2_U, OMEGA_3_U, OMEGA_G, OMEGA_G, OMEGA_G], self.N)
        lrow = np.concatenate([[Z_U_MIN, -THETA_U_MAX, -PHI_G_MAX, -THETA_G_MAX, -SHI_G_MAX],
                               np.full(self.n_obs, -np.inf)])
        urow = np.concatenate([[Z_U_MAX, THETA_U_MAX, PHI_G_MAX, THETA_G_MAX, SHI_G_MAX],
                               np.zeros(self.n_obs)])
        return lbx, ubx, np.tile(lrow, self.N + 1), np.tile(urow, self.N + 1)


def make_spec(layout: str | None = "nmpc_tt", N: int = 15, T: float = 1.0, dynamic: bool = False,
              obstacles: Sequence[Obstacle] | None = None, weights_in_p: bool = False,
              model: str = "uav8g") -> ProblemSpec:
    """Spec for a reference scenario family.

    layout: one of LAYOUTS (None = no obstacles).  dynamic=True makes the y
    coordinate of obstacles 1-6 parameters p[11:17] (MATLAB/Dynamic Obstacles/
    Dynamic Obstacle avoidance.m:52,128-133), np = 17.  weights_in_p=True
    appends the cost weights (w1, w2) to p, one pair per scenario: the batched
    form of the RL replay that rebuilds nlpsol per weight pair
    (MATLAB/Race Track 1/MPC.m:1,127).  model="uav5" is the
    no-gimbal variant (MATLAB/Dynamic Obstacles/NMPC_TT.m): p = [x0(5); xs(3); ...].
    """
    np0 = 8 if model == "uav5" else 11
    if obstacles is None:
        obstacles = ()
        if layout is not None:
            xy, r = LAYOUTS[layout]
            obstacles = tuple(
                Obstacle(float(x), float(y), UAV_R + r, -1, (np0 + j) if (dynamic and j < 6) else -1)
                for j, (x, y) in enumerate(xy))
    npar = np0 + 6 if dynamic else np0
    w1p = w2p = -1
    if weights_in_p:
        w1p, w2p, npar = npar, npar + 1, npar + 2
    return ProblemSpec(N=N, T=T, obstacles=tuple(obstacles), np=npar, w1_pidx=w1p, w2_pidx=w2p,
                       model=model).validate()


# SURVEY.md section 8 configurations
def config_spec(cfg: int) -> ProblemSpec:
    if cfg == 0:   # Python/NMPC_TT.py as written (N=15, T=1, 3 obstacles)
        return make_spec("nmpc_tt", N=15, T=1.0)
    if cfg == 1:   # plumbing: no-gimbal model, N=10, 0 obstacles (BASELINE configs[0])
        return make_spec(None, N=10, T=0.2, model="uav5")
    if cfg == 2:   # batch 1024, N=20, 0 obstacles, T=0.2
        return make_spec(None, N=20, T=0.2)
    if cfg in (3, 4):  # N=20, 10 active obstacles (Race Track 2.py), T=0.2
        return make_spec("race_track_2", N=20, T=0.2)
    if cfg == 5:   # N=50, dynamic obstacles
        return make_spec("dynamic", N=50, T=0.2, dynamic=True)
    raise ValueError(cfg)
