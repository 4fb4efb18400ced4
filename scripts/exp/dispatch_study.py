"""Dev tool: the bench's timed launch (W warm-up MPC steps, then K fused steps)
with index-order and longest-first dispatch; per-scenario chain iterations and
launch times to gpurun_out/dispatch.npz for offline list-scheduling analysis."""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
from nmpc_amd.schedule import longest_first
K, B = 20, int(sys.argv[1]) if len(sys.argv) > 1 else 4096
W = int(sys.argv[2]) if len(sys.argv) > 2 else 2
spec = config_spec(3)
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
i32 = dict(dtype=torch.int32, device="cuda")
bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
p = torch.tensor(draw_scenarios(spec, B, seed=1003), **f64).contiguous()
w = torch.zeros(B, spec.nw, **f64)
vt, wt = torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64)
hw = {"iters": torch.empty(W, B, **i32)}
s.closed_loop_device(W, *bnd, p, w, vt, wt, hw)
res = {"warm": hw["iters"].cpu().numpy()}
for name, order in (("inorder", None), ("lpt", longest_first(hw["iters"]))):
    for rep in range(2):
        h = {"iters": torch.empty(K, B, **i32)}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        pp, ww = p.clone(), w.clone()
        torch.cuda.synchronize(); e0.record()
        s.closed_loop_device(K, *bnd, pp, ww, vt, wt, h, order=order)
        e1.record(); torch.cuda.synchronize()
    res[name + "_ms"] = e0.elapsed_time(e1)
    res[name + "_iters"] = h["iters"].cpu().numpy()
    print(name, res[name + "_ms"], "ms; max chain", h["iters"].sum(0).max().item())
np.savez(os.path.join(ROOT, "gpurun_out", "dispatch.npz"), **res)
