"""Dev tool: cycles per iteration of restoration-heavy solves (the closed-loop
tail), from the 16 captured restoration cases replicated to B scenarios; needs
the -DNMPC_STAMPS build (NMPC_LIB=.../libnmpc_amd_stamps.so)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, make_spec, REFERENCE_OPTS
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = np.load(os.path.join(ROOT, "tests", "golden", "resto_cases.npz"))
rep = (B + 15) // 16
W = np.tile(G["w"], (rep, 1))[:B]
Pm = np.tile(G["p"], (rep, 1))[:B]
spec = make_spec("race_track_2", N=20, T=0.2)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
for _ in range(2):
    t = time.time()
    s(x0=W.T, lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=Pm.T)
    wall = time.time() - t
tr = s.read_trace(B)
st = tr[:, s.max_iter + 1:, :].reshape(B, -1)[:, :24]
it = s.stats()["iter_count"]
tot = st[:, 15]
print(f"B={B} wall {wall*1e3:.1f} ms; iters mean {np.mean(it):.1f} max {np.max(it)}; "
      f"cycles/iter mean {np.mean(tot / it):.3e}; main-phase share {np.mean(st[:, :15].sum(1) / tot):.2f}")
PH = ["rollout", "eval", "derivs", "adjoint", "summaries", "riccati", "resolve", "forward", "row_step",
      "barrier", "ftb", "dual_ftb", "conv+mu", "accept", "init/resto-ls", "TOTAL", "ric.1", "#factor", "#soc",
      "ric.2", "ric.3", "sigx", "ls_setup", "filter"]
mi = np.mean(it)
for i, n in enumerate(PH):
    if i in (15, 17, 18):
        continue
    print(f"  {n:14s} per-iter {st[:, i].mean() / mi:10.1f}  {100 * st[:, i].mean() / tot.mean():6.2f}%")
