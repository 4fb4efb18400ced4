"""CPU tests: problem spec / bounds / scenarios, and the C-ABI library (loads,
exports every symbol include/nmpc_amd.h declares, struct layout, argument
validation that happens before any HIP call)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from oracle import nmpc_oracle as orc
from nmpc_amd import spec as S
from nmpc_amd import _lib, make_spec, draw_scenarios, config_spec
from nmpc_amd.nlpsol import make_options

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nmpc_amd.h")


@pytest.mark.parametrize("layout,N,T", [("nmpc_tt", 15, 1.0), ("10_obstacles", 15, 0.2),
                                        ("race_track_2", 20, 0.2), (None, 20, 0.2), ("race_track_2", 7, 0.2)])
def test_spec_matches_oracle(layout, N, T):
    sp_ = make_spec(layout, N=N, T=T)
    pr = orc.make_problem(layout, N=N, T=T)
    for a, b in zip(sp_.bounds(), orc.bounds(pr)):
        np.testing.assert_array_equal(a, b)
    assert sp_.ng == pr.ng and sp_.nw == pr.nw and sp_.m == pr.m
    np.testing.assert_array_equal([o.x for o in sp_.obstacles], pr.obs_x)
    np.testing.assert_array_equal([o.y for o in sp_.obstacles], pr.obs_y)
    np.testing.assert_array_equal([o.r for o in sp_.obstacles], pr.obs_rsum)


def test_dynamic_spec_parameter_indices():
    sp_ = make_spec("dynamic", N=10, T=0.2, dynamic=True)
    assert sp_.np == 17
    assert [o.y_pidx for o in sp_.obstacles] == [11, 12, 13, 14, 15, 16, -1, -1, -1, -1]
    pr = orc.make_problem("dynamic", N=10, T=0.2, dynamic=True)
    assert list(pr.obs_y_pidx) == [11, 12, 13, 14, 15, 16, -1, -1, -1, -1]


def test_spec_validation():
    with pytest.raises(ValueError):
        make_spec(None, N=0)
    with pytest.raises(ValueError):
        make_spec(None, N=64)
    with pytest.raises(ValueError):
        S.ProblemSpec(N=5, obstacles=tuple(S.Obstacle(0, 0, 1) for _ in range(17))).validate()


def test_scenarios_deterministic_and_shardable():
    sp_ = config_spec(3)
    a = draw_scenarios(sp_, 64, seed=1003)
    b = draw_scenarios(sp_, 128, seed=1003)
    np.testing.assert_array_equal(a, b[:64])  # global stream, sliced per rank
    ox = np.array([o.x for o in sp_.obstacles]); oy = np.array([o.y for o in sp_.obstacles])
    rr = np.array([o.r for o in sp_.obstacles])
    for p in b:
        assert np.all(np.hypot(p[0] - ox, p[1] - oy) > rr + 10)
        assert 75 < p[2] < 150 and abs(p[3]) < 0.2618


def test_library_exports_every_header_symbol():
    txt = open(HEADER).read()
    declared = set(re.findall(r"^\s*(?:int|void|const char\*)\s+(nmpc_\w+)\s*\(", txt, flags=re.M))
    assert declared == set(_lib.EXPORTS)
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name


def test_library_built_from_this_source():
    """The shared object under test was compiled from the checked-out kernel source,
    header and flags (hash embedded at build time, __graft_entry__.source_hash)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("graft_entry", os.path.join(ROOT, "__graft_entry__.py"))
    ge = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ge)
    assert _lib.lib().nmpc_build_id().decode() == ge.source_hash()


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include "nmpc_amd.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(){printf("%zu %zu %zu %zu\\n", sizeof(nmpc_desc), sizeof(nmpc_options),'
                   ' offsetof(nmpc_desc, opts), offsetof(nmpc_desc, obs_x_pidx));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    assert [int(v) for v in out] == [C.sizeof(_lib.Desc), C.sizeof(_lib.Options), _lib.Desc.opts.offset,
                                     _lib.Desc.obs_x_pidx.offset]


def test_default_options_are_ipopt_defaults():
    o = _lib.default_options()
    for k, v in orc.IPOPT_DEFAULTS.items():
        assert getattr(o, k) == pytest.approx(v, rel=1e-15), k
    r = make_options({"ipopt": {"max_iter": 100, "print_level": 0, "acceptable_tol": 1e-8,
                                "acceptable_obj_change_tol": 1e-6}, "print_time": 0})
    assert r.max_iter == 100 and r.acceptable_tol == 1e-8 and r.acceptable_obj_change_tol == 1e-6
    with pytest.raises(ValueError):
        make_options({"ipopt": {"no_such_option": 1}})
    with pytest.raises(ValueError):
        make_options({"ipopt": {"hessian_approximation": "limited-memory"}})
    make_options({"ipopt": {"fixed_variable_treatment": "make_parameter"}})  # IPOPT default: accepted
    with pytest.raises(ValueError):
        make_options({"ipopt": {"fixed_variable_treatment": "relax_bounds"}})


def _desc(**kw):
    d = _lib.Desc()
    d.model, d.N, d.np, d.n_obs, d.T, d.w1, d.w2, d.vfov, d.hfov = 0, 10, 11, 0, 0.2, 1, 2, 1, 1
    d.opts = _lib.default_options()
    for k, v in kw.items():
        setattr(d, k, v)
    return d


@pytest.mark.parametrize("bad", [dict(N=0), dict(N=64), dict(n_obs=17), dict(np=10), dict(T=0.0), dict(model=3)])
def test_create_rejects_bad_descriptor(bad):
    h = C.c_void_p()
    rc = _lib.lib().nmpc_create(C.byref(_desc(**bad)), C.byref(h))
    assert rc == -1 and not h.value
    assert _lib.lib().nmpc_last_error()


def test_null_handle_rejected():
    L = _lib.lib()
    assert L.nmpc_dims(None, None, None, None, None) == -1
    assert L.nmpc_set_trace(None, 1) == -1
    with pytest.raises(_lib.NmpcError):
        _lib.check(L.nmpc_destroy(None) or -1)


def test_product_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from nmpc_amd import nlpsol

    with pytest.raises(_lib.NmpcError):
        nlpsol("solver", "ipopt", config_spec(3), None)


def test_target_schedules_follow_reference_tables():
    """con_t chains of the reference scripts' shift_timestep."""
    import math
    from nmpc_amd.targets import con_t, schedule, SCHEDULES

    assert con_t("nmpc_tt", 0) == (12.0, 0.01)                      # NMPC_TT.py:25
    assert con_t("10_obstacles", 299) == (13.0, 0.0)                # 10_obstacles.py:28-31
    assert con_t("10_obstacles", 300) == (13.0, -(math.pi / 2) / 24)
    assert con_t("10_obstacles", 2000) == (13.0, (math.pi / 2) / 12)
    assert con_t("race_track_2", 1500) == (12.0, math.pi / 100)     # Race Track 2.py:35
    assert con_t("plus_trajectory", 101) == (20.0, (math.pi / 2) * 5)
    assert con_t("plus_trajectory", 102) == (20.0, 0.0)             # Plus Trajectory.py:26-29
    assert con_t("t_trajectory", 259) == (13.5, 0.0) and con_t("t_trajectory", 260)[1] < 0
    v, w = schedule("10_obstacles", 298, 4)
    assert list(w[:2]) == [0.0, 0.0] and w[2] == w[3] == -(math.pi / 2) / 24 and (v == 13.0).all()
    for name, tab in SCHEDULES.items():
        assert [k for k, _, _ in tab] == sorted(k for k, _, _ in tab), name


def test_dynamic_obstacle_schedule_and_weight_indices():
    """MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230 windows;
    weight parameter indices of the batched weight sweep."""
    import pytest
    from nmpc_amd import make_spec
    from nmpc_amd.targets import obstacle_steps
    from nmpc_amd.spec import ProblemSpec

    d = obstacle_steps(0, 1400)
    assert d[:, :11].sum() == 0
    assert d[100, 12] == 0 and d[101, 12] == -1 and d[399, 12] == -1 and d[400, 12] == 0  # y_o_2
    assert d[:, 13].sum() == 299 and d[:, 16].sum() == -299 and d[1001, 11] == 1
    s = make_spec("race_track_2", N=20, T=0.2, weights_in_p=True)
    assert (s.np, s.w1_pidx, s.w2_pidx) == (13, 11, 12)
    with pytest.raises(ValueError):
        ProblemSpec(N=5, np=13, w1_pidx=3).validate()


def test_longest_first_order():
    """schedule.longest_first: a permutation, largest summed cost first, ties in index order."""
    import torch
    from nmpc_amd.schedule import longest_first

    it = torch.tensor([[3, 100, 7, 7, 0], [4, 100, 1, 1, 0]], dtype=torch.int32)
    o = longest_first(it)
    assert o.dtype == torch.int32 and o.tolist() == [1, 2, 3, 0, 4]
    c = torch.tensor([5.0, 9.0, 1.0])
    assert longest_first(c).tolist() == [1, 0, 2]
    r = torch.randint(0, 100, (3, 257))
    assert sorted(longest_first(r).tolist()) == list(range(257))
