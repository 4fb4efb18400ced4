"""The fp32 leg of BASELINE config 5's fp32-vs-fp64 sweep: nlpsol option
linear_solver_precision='single' runs the Riccati factorisation and its solves in
fp32 (CapA32 / CapC32 kernels); the iterate, residuals, line search and termination
tests stay fp64.  At a loosened tolerance (1e-6, the sweep's middle point) the fp32
solutions must agree with the fp64 solver's to the accuracy that tolerance buys
(u0 and f within 1e-3 relative; measured deviations: profiles/r02_tol_sweep.jsonl),
and the fp32 kernel must really be a different path (results not bitwise fp64)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(cfg, B, prec, tol):
    from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS

    spec = config_spec(cfg)
    o = {"ipopt": dict(REFERENCE_OPTS["ipopt"], tol=tol, acceptable_tol=max(tol, 1e-8)),
         "linear_solver_precision": prec}
    s = nlpsol("solver", "ipopt", spec, o)
    lbx, ubx, lbg, ubg = spec.bounds()
    P = draw_scenarios(spec, B, seed=1000 + cfg)
    sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
    return sol, s.stats()["status_code"], s.stats()["iter_count"]


@pytest.mark.parametrize("cfg,B", [(3, 64), (5, 16)])
def test_fp32_riccati_matches_fp64_at_loosened_tolerance(cfg, B):
    s64, st64, it64 = _solve(cfg, B, "double", 1e-6)
    s32, st32, it32 = _solve(cfg, B, "single", 1e-6)
    both = np.isin(st64, (0, 1)) & np.isin(st32, (0, 1))
    print(f"\nconfig {cfg}: fp64 {dict(zip(*np.unique(st64, return_counts=True)))} mean it {it64.mean():.1f}; "
          f"fp32 {dict(zip(*np.unique(st32, return_counts=True)))} mean it {it32.mean():.1f}")
    assert both.sum() >= 0.75 * np.isin(st64, (0, 1)).sum()
    du = np.abs(s32["x"][:6, both] - s64["x"][:6, both]) / (1 + np.abs(s64["x"][:6, both]))
    df = np.abs(s32["f"][0, both] - s64["f"][0, both]) / (1 + np.abs(s64["f"][0, both]))
    print(f"  converged in both: {both.sum()}; u0 rel dev max {du.max():.2e}; f rel dev max {df.max():.2e}")
    assert df.max() <= 1e-3 and np.percentile(du.max(0), 90) <= 1e-2
    assert not np.array_equal(s32["x"], s64["x"])
