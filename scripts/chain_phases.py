"""Dev tool (round 5): per-phase cycles of the bounding chain (default: scenario 2284 of
the bench workload, W = 5 warm-up then K = 20 timed closed-loop steps, each solved alone
with the trace on), from the -DNMPC_STAMPS build (NMPC_LIB=...); with
-DNMPC_RESTO_TRIAL_STAMPS the slots 'barrier' / 'ftb' / 'dual_ftb' hold the restoration
trials' cycles, the second-order-correction blocks' cycles and the trial count."""
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
PH = ["rollout", "eval", "derivs", "adjoint", "summaries", "riccati", "resolve", "forward", "row_step",
      "barrier", "ftb", "dual_ftb", "conv+mu", "accept", "init/resto-ls", "TOTAL", "ric.1", "#factor", "#soc",
      "ric.2", "ls-total", "sigx", "ls_setup", "filter"]
acc = np.zeros(24)
n_it = n_res = 0
for k in range(W + K):
    s.solve_device(w, *bnd, p, out)
    torch.cuda.synchronize()
    tr = s.read_trace(1)[0]
    it = int(out["iters"].item())
    if k >= W:
        acc += tr[s.max_iter + 1:].reshape(-1)[:24]
        n_it += it
        n_res += int((tr[:it, 7] < 0).sum())
    s.shift_device(p, out["x"], w, vt, wt)
print(f"scenario {b}: {n_it} iterations over the {K} timed steps ({n_res} restoration); "
      f"cycles per iteration {acc[15] / n_it:.4g}")
for i, n in enumerate(PH):
    if i == 15:
        continue
    cnt = i in (17, 18) or (n == "dual_ftb" and os.environ.get("RESTO_TRIAL"))
    print(f"  {n:14s} {'count' if cnt else 'cycles'} per iteration {acc[i] / n_it:10.1f}"
          + ("" if cnt else f"  {100 * acc[i] / acc[15]:6.2f}%"))
