"""Dev tool (round 5): the parts of the bounding chain's restoration iterations (default:
scenario 2284 of the bench workload, W = 5 warm-up then K = 20 timed closed-loop steps,
each solved alone with the trace on), from the -DNMPC_STAMPS -DNMPC_XSTAMPS build
(NMPC_LIB=...): the generic phase timers are off and the slots time the restoration
iteration's parts (XPhase in nmpc_solve.hip)."""
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
NAMES = {0: "trial: control pass", 1: "trial: rollout (1 or 2 trials)", 2: "trial: eval_fg (1 or 2)",
         3: "trial: row pass", 4: "trial: sums, phi", 5: "#trial_resto calls",
         6: "SOC: cms pass", 7: "SOC: assembly", 8: "SOC: re-solve", 9: "SOC: forward (+refine)",
         10: "SOC blocks (total)", 11: "Newton: assembly", 12: "Newton: Riccati", 13: "Newton: forward, row step",
         16: "check + mu (with adjoint)", 19: "accept", 20: "derivs", 21: "line search (total)",
         22: "restoration iteration (total)", 23: "#restoration iterations", 15: "whole solves (total)"}
acc = np.zeros(24)
n_it = 0
for k in range(W + K):
    s.solve_device(w, *bnd, p, out)
    torch.cuda.synchronize()
    tr = s.read_trace(1)[0]
    if k >= W:
        acc += tr[s.max_iter + 1:].reshape(-1)[:24]
        n_it += int(out["iters"].item())
    s.shift_device(p, out["x"], w, vt, wt)
nr = acc[23]
print(f"scenario {b}: {n_it} iterations over the {K} timed steps, {nr:.0f} restoration iterations; "
      f"restoration iteration {acc[22] / nr:.4g} cycles, whole solves {acc[15] / n_it:.4g} cycles per iteration")
for i in sorted(NAMES):
    if i in (15, 23):
        continue
    v = acc[i] / nr
    if i == 5:
        print(f"  {NAMES[i]:34s} {v:10.2f} per restoration iteration")
    else:
        print(f"  {NAMES[i]:34s} {v:10.1f} cycles per restoration iteration  {100 * acc[i] / acc[22]:6.2f}%")
