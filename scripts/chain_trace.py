"""Dev tool: the iteration mix of one scenario's closed-loop chain (default: scenario
2284 of the bench workload, the chain that bounds the config-3 launch): per step the
iterations, restoration iterations, mean / max line-search trials and the solve time."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 2284
W, K = 5, 20
spec = config_spec(3)
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
p = torch.tensor(draw_scenarios(spec, 4096, seed=1003)[b:b + 1], **f64).contiguous()
w = torch.zeros(1, spec.nw, **f64)
vt, wt = torch.full((1,), 12.0, **f64), torch.full((1,), 0.01, **f64)
out = {"x": torch.empty(1, spec.nw, **f64), "f": torch.empty(1, **f64),
       "status": torch.empty(1, dtype=torch.int32, device="cuda"), "iters": torch.empty(1, dtype=torch.int32, device="cuda")}
s.set_trace(True)
tot_it = tot_ms = 0.0
hist = {}  # (restoration?, trials) -> iterations over the timed steps
for k in range(W + K):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s.solve_device(w, *bnd, p, out)
    e1.record()
    torch.cuda.synchronize()
    tr = s.read_trace(1)[0]
    n = int(out["iters"].item())
    ls = tr[:n, 7]
    resto = int((ls < 0).sum())
    ms = e0.elapsed_time(e1)
    if k >= W:
        tot_it += n
        tot_ms += ms
        for v in ls:
            key = (bool(v < 0), int(abs(v)))
            hist[key] = hist.get(key, 0) + 1
    print(f"step {k - W:3d}: it {n:3d} status {int(out['status'].item()):3d} resto {resto:3d} "
          f"ls trials mean {np.abs(ls).mean():5.2f} max {np.abs(ls).max():4.0f}  {ms:6.2f} ms  {1e3 * ms / max(n, 1):6.1f} us/it")
    s.shift_device(p, out["x"], w, vt, wt)
print(f"timed steps: {tot_it:.0f} iterations in {tot_ms:.1f} ms alone on the GPU ({1e3 * tot_ms / tot_it:.1f} us/iteration)")
for r in (False, True):
    row = {t: c for (rr, t), c in sorted(hist.items()) if rr == r}
    tot = sum(row.values())
    if tot:
        print(("restoration" if r else "regular") + f" iterations {tot}: line-search trials -> count " +
              ", ".join(f"{t}:{c}" for t, c in row.items()) +
              f"  (mean {sum(t * c for t, c in row.items()) / tot:.2f})")
