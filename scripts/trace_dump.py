"""Dev tool: per-iteration traces (mu, f, theta, delta, alpha_p, alpha_d, trials) of cold
config-3 solves, saved to an .npz so two builds (NMPC_LIB=...) can be compared iteration
by iteration:  python scripts/trace_dump.py out.npz [B]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
spec = config_spec(3)
P = draw_scenarios(spec, B, seed=1003)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
np.savez(sys.argv[1], trace=s.read_trace(B), x=sol["x"], it=s.stats()["iter_count"])
