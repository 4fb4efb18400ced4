"""Dev tool: per-phase cycle breakdown of the solve kernel (needs the
-DNMPC_STAMPS build: NMPC_LIB=.../libnmpc_amd_stamps.so)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
PH = ["rollout", "eval", "derivs", "adjoint", "summaries", "riccati", "resolve", "forward", "row_step",
      "barrier", "ftb", "dual_ftb", "conv+mu", "accept", "init", "TOTAL", "ric.1", "#factor", "#soc", "ric.2", "ls-total", "sigx", "ls_setup", "filter"]
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
spec = config_spec(cfg)
P = draw_scenarios(spec, B, seed=1000 + cfg)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
t = time.time()
s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
print("wall", time.time() - t)
tr = s.read_trace(B)
st = tr[:, s.max_iter + 1:, :].reshape(B, -1)[:, :24]
it = s.stats()["iter_count"]
tot = st[:, 15].mean()
print(f"B={B} mean iters {np.mean(it):.2f}; mean total cycles/scenario {tot:.3e} ({tot/np.mean(it):.3e} per iter)")
for i, n in enumerate(PH[:15]):
    print(f"  {n:10s} {st[:, i].mean():12.4e}  {100*st[:, i].mean()/tot:6.2f}%  per-iter {st[:, i].mean()/np.mean(it):10.1f}")
print(f"  unattributed {100*(tot - st[:, :15].sum(1).mean() - st[:, 21:24].sum(1).mean())/tot:6.2f}%")
for i in range(16, 24):
    print(f"  {PH[i]:10s} {st[:, i].mean():12.4e}  {100*st[:, i].mean()/tot:6.2f}%  per-iter {st[:, i].mean()/np.mean(it):10.1f}")
tot_c = st[:, 15]
print("per-scenario total cycles: p50 %.3e p90 %.3e p99 %.3e max %.3e" % tuple(np.percentile(tot_c, [50, 90, 99, 100])))
print("iterations: p50 %d p90 %d p99 %d max %d" % tuple(np.percentile(it, [50, 90, 99, 100]).astype(int)))
print("status:", {int(k): int(v) for k, v in zip(*np.unique(s.stats()["status_code"], return_counts=True))})
