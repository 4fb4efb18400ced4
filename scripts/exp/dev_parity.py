"""Dev tool: GPU solve vs the CPU oracle on a few scenarios, with iteration traces."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, make_spec, draw_scenarios, REFERENCE_OPTS
from oracle import nmpc_oracle as orc

layout = sys.argv[1] if len(sys.argv) > 1 else "race_track_2"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
T = float(sys.argv[3]) if len(sys.argv) > 3 else 0.2
B = int(sys.argv[4]) if len(sys.argv) > 4 else 6
spec = make_spec(None if layout == "none" else layout, N=N, T=T)
prob = orc.make_problem(None if layout == "none" else layout, N=N, T=T)
P = draw_scenarios(spec, B, seed=1003)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
t = time.time()
sol = s(x0=np.zeros(spec.nw), lbx=lbx, ubx=ubx, lbg=lbg, ubg=ubg, p=P.T)
print("gpu solve wall", time.time() - t, s.kernel_info())
tr = s.read_trace(B)
ref = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
for b in range(B):
    r = ref.solve(np.zeros(spec.nw), lbx, ubx, lbg, ubg, P[b], trace=True)
    st = s.stats()["status_code"][b]; it = s.stats()["iter_count"][b]
    err = np.max(np.abs(sol["x"][:, b] - r["x"]) / (1 + np.abs(r["x"])))
    print(f"b={b} gpu status={st} it={it} f={sol['f'][0,b]:.10f} | oracle status={r['status']} it={r['iter']} f={r['f']:.10f} | max rel dx={err:.3e}")
    nshow = min(int(it), len(r["trace"]), 60)
    for k in range(nshow):
        g = tr[b, k]; o = r["trace"][k]
        flag = "" if abs(g[2]-o["f"]) <= 1e-8*(1+abs(o["f"])) and abs(g[1]-o["mu"]) < 1e-15 else "  <-- differs"
        if flag or k < 3:
            print(f"   it {k+1}: gpu mu={g[1]:.3e} f={g[2]:.12f} th={g[3]:.3e} dl={g[4]:.2e} ap={g[5]:.4f} ad={g[6]:.4f} ls={int(g[7])} | cpu mu={o['mu']:.3e} f={o['f']:.12f} th={o['theta']:.3e} dl={o['delta']:.2e} ap={o['alpha_p']:.4f} ad={o['alpha_d']:.4f} ls={o['ls']}{flag}")
        if flag: break
