"""Dev tool: per-step kernel time and iteration distribution of the K-step
closed loop (bench.py workload); how much of each launch is the slowest scenario."""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
spec = config_spec(3)
lbx, ubx, lbg, ubg = spec.bounds()
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
L = [torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)]
p = torch.tensor(draw_scenarios(spec, B, seed=1003), **f64).contiguous()
w = torch.zeros(B, spec.nw, **f64)
out = {"x": torch.empty(B, spec.nw, **f64), "iters": torch.empty(B, dtype=torch.int32, device="cuda"),
       "status": torch.empty(B, dtype=torch.int32, device="cuda")}
v_t = torch.full((B,), 12.0, **f64); w_t = torch.full((B,), 0.01, **f64)
its, sts, ms = [], [], []
for k in range(K):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); s.solve_device(w, *L, p, out); e1.record()
    s.shift_device(p, out["x"], w, v_t, w_t)
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1)); its.append(out["iters"].cpu().numpy()); sts.append(out["status"].cpu().numpy())
its = np.array(its); sts = np.array(sts)
for k in range(K):
    print(f"step {k:2d} kernel {ms[k]:7.2f} ms  iters mean {its[k].mean():5.1f} p99 {np.percentile(its[k],99):5.0f} max {its[k].max():3d}  n(-1) {(sts[k]==-1).sum()} n(-2) {(sts[k]==-2).sum()}")
tot = its.sum(0)
print("sum over steps of per-step max iters:", its.max(1).sum())
print("per-scenario sum of iters over K steps: mean %.1f p99 %.0f max %d" % (tot.mean(), np.percentile(tot, 99), tot.max()))
print("warm steps (1..K-1): sum of kernel ms %.1f, mean iters %.2f" % (sum(ms[1:]), its[1:].mean()))
np.savez(os.path.join(ROOT, "gpurun_out", "closed_loop_stats.npz"), its=its, sts=sts, ms=np.array(ms))
