"""Dev tool: kernel time vs batch size (is the launch dominated by its slowest scenario?)."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
spec = config_spec(3)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
t_lbx, t_ubx, t_lbg, t_ubg = [torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)]
Pall = draw_scenarios(spec, 16384, seed=1003)
for B in (256, 1024, 2048, 4096, 8192, 16384):
    p = torch.tensor(Pall[:B], **f64)
    out = {"x": torch.empty(B, spec.nw, **f64), "iters": torch.empty(B, dtype=torch.int32, device="cuda"),
           "status": torch.empty(B, dtype=torch.int32, device="cuda")}
    w = torch.zeros(B, spec.nw, **f64)
    s.solve_device(w, t_lbx, t_ubx, t_lbg, t_ubg, p, out); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); s.solve_device(w, t_lbx, t_ubx, t_lbg, t_ubg, p, out); e1.record(); torch.cuda.synchronize()
    it = out["iters"].cpu().numpy()
    ms = e0.elapsed_time(e1)
    print(f"B={B:6d} kernel {ms:8.2f} ms  {B/ms*1e3:10.0f} solves/s  iters mean {it.mean():.1f} max {it.max()}  sum(iters)/ms {it.sum()/ms:.0f}")
