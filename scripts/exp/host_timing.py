"""Dev tool: host-side timing of each call in the bench step loop."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
spec = config_spec(3); B = 4096
P = draw_scenarios(spec, B, seed=1003)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
t_lbx, t_ubx, t_lbg, t_ubg = [torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)]
p = torch.tensor(P, **f64); w = torch.zeros(B, spec.nw, **f64)
out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
       "status": torch.empty(B, dtype=torch.int32, device="cuda"), "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
vt = torch.full((B,), 12.0, **f64); wt = torch.full((B,), 0.01, **f64)
st = torch.cuda.current_stream()
for k in range(6):
    t0 = time.perf_counter()
    s.solve_device(w, t_lbx, t_ubx, t_lbg, t_ubg, p, out, stream=st)
    t1 = time.perf_counter()
    s.shift_device(p, out["x"], w, vt, wt, stream=st)
    t2 = time.perf_counter()
    x = out["iters"].sum()
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"step {k}: solve_call {1e3*(t1-t0):8.3f} ms  shift_call {1e3*(t2-t1):8.3f}  sum {1e3*(t3-t2):8.3f}  sync_wait {1e3*(t4-t3):8.3f}  total {1e3*(t4-t0):8.3f}")
