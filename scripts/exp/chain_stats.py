"""Dev tool: per-scenario iteration sums over a K-step fused closed loop (the
chain each wavefront runs) vs the launch time."""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
K = 20
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
spec = config_spec(3)
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
f64 = dict(dtype=torch.float64, device="cuda")
bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
p0 = torch.tensor(draw_scenarios(spec, B, seed=1003), **f64).contiguous()
vt, wt = torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64)
for rep in range(2):
    p, w = p0.clone(), torch.zeros(B, spec.nw, **f64)
    hist = {"iters": torch.empty(K, B, dtype=torch.int32, device="cuda"),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); s.closed_loop_device(K, *bnd, p, w, vt, wt, hist); e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
it = hist["iters"].cpu().numpy(); st = hist["status"].cpu().numpy()
chain = it.sum(0)
order = np.argsort(-chain)
print(f"launch {ms:.1f} ms; total iterations {it.sum()}; mean chain {chain.mean():.0f}; p99 {np.percentile(chain, 99):.0f}; max {chain.max()}")
print("ms per chain-iteration if the longest chain bounds the launch:", ms / chain.max())
print("top chains:", chain[order[:10]].tolist())
print("scenarios with >=5 max-iter steps:", int(((it >= 100).sum(0) >= 5).sum()))
print("status counts:", {int(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))})
out = os.environ.get("CHAIN_OUT")
if out:
    np.savez(out, iters=it, status=st, ms=ms)
