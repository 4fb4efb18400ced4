"""Dev tool: the restoration line search's cost (round 5), from the 16 captured
restoration cases replicated to B scenarios; needs the diagnostic build
-DNMPC_STAMPS -DNMPC_RESTO_TRIAL_STAMPS (NMPC_LIB=.../librstamps.so), whose slots
PH_BARR / PH_FTB / PH_DFTB hold the cycles inside trial_resto, the cycles of
second-order-correction blocks and the number of trial_resto calls."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, make_spec, REFERENCE_OPTS
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
G = np.load(os.path.join(ROOT, "tests", "golden", "resto_cases.npz"))
rep = (B + 15) // 16
W = np.tile(G["w"], (rep, 1))[:B]
Pm = np.tile(G["p"], (rep, 1))[:B]
spec = make_spec("race_track_2", N=20, T=0.2)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
for _ in range(2):
    s(x0=W.T, lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=Pm.T)
tr = s.read_trace(B)
st = tr[:, s.max_iter + 1:, :].reshape(B, -1)[:, :24]
it = s.stats()["iter_count"]
nres = np.array([(tr[b, :it[b], 7] < 0).sum() for b in range(B)])
ls_tr = np.array([-tr[b, :it[b], 7][tr[b, :it[b], 7] < 0].sum() for b in range(B)])  # backtracking trials
tot = st[:, 15]
m = lambda i: st[:, i].sum()
print(f"B={B}: iterations {it.sum()} ({nres.sum()} restoration), cycles/iteration {tot.sum() / it.sum():.4g}")
print(f"restoration line search (backtracking trials incl. the first, per trace) {ls_tr.sum()} "
      f"= {ls_tr.sum() / max(1, nres.sum()):.2f} per restoration iteration")
ntr = m(11)
print(f"trial_resto calls {ntr:.0f} ({ntr / max(1, nres.sum()):.2f} per restoration iteration): "
      f"{m(9) / ntr:.4g} cycles each, of which rollout {m(0) / ntr:.4g}, eval {m(1) / ntr:.4g} (if no other caller), "
      f"the rest (controls pass, rows pass, reductions) {(m(9) - m(0) - m(1)) / ntr:.4g}")
print(f"SOC blocks {m(10):.4g} cycles total = {m(10) / max(1, nres.sum()):.4g} per restoration iteration; "
      f"SOC re-solves {m(18):.0f} ({m(18) / max(1, nres.sum()):.3f} per restoration iteration)")
print(f"filter checks {m(23) / max(1, nres.sum()):.4g} cycles per restoration iteration; "
      f"whole restoration LS (PH_INIT) {m(14) / max(1, nres.sum()):.4g} per restoration iteration")
print(f"per restoration iteration: riccati {m(5) / it.sum():.4g} conv+mu {m(12) / it.sum():.4g} "
      f"row_step {m(8) / it.sum():.4g} accept {m(13) / it.sum():.4g} summaries {m(4) / it.sum():.4g} "
      f"forward {m(7) / it.sum():.4g} adjoint {m(3) / it.sum():.4g} derivs {m(2) / it.sum():.4g}")
