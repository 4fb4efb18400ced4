"""Dev tool: per-wave latency vs waves per SIMD.  Runs config-3 cold solves with the
stamps build (NMPC_LIB) under the capacity class / LDS padding given in the
environment (NMPC_FORCE_CLASS, NMPC_LDS_BYTES) and prints the mean shader cycles per IP
iteration per scenario (latency) and total iterations / kernel time (throughput)."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
B = int(sys.argv[1])
spec = config_spec(3)
P = draw_scenarios(spec, 4096, seed=1003)
P = np.tile(P, ((B + 4095) // 4096, 1))[:B]
s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
s.set_trace(True)
f64 = dict(dtype=torch.float64, device="cuda")
bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
p = torch.tensor(P, **f64).contiguous()
w = torch.zeros(B, spec.nw, **f64)
out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
       "status": torch.empty(B, dtype=torch.int32, device="cuda"), "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
for rep in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    s.solve_device(w, *bnd, p, out)
    e1.record()
    torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
it = out["iters"].cpu().numpy()
tr = s.read_trace(B)
tot = tr[:, s.max_iter:, :].reshape(B, -1)[:, :24][:, 15]
print(f"class={os.environ.get('NMPC_FORCE_CLASS', 'A')} lds_pad={os.environ.get('NMPC_LDS_BYTES', '-')} "
      f"B={B} kernel_info={s.kernel_info()} kernel {ms:.2f} ms; iters mean {it.mean():.2f} max {it.max()}; "
      f"cycles/iter per scenario mean {np.mean(tot / np.maximum(it, 1)):.4e}; "
      f"throughput {it.sum() / ms * 1e3:.4e} iterations/s")
