"""Dev tool: low-noise per-wave latency probe.  Times (best of R launches) a cold
solve of the 16 captured restoration cases replicated to 256 scenarios (each
wave alone on its SIMD: restoration-iteration latency, the closed-loop tail) and
a cold config-3 solve of 1024 scenarios (main iterations, one wave per SIMD)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
import torch
from nmpc_amd import nlpsol, make_spec, config_spec, draw_scenarios, REFERENCE_OPTS

R = int(os.environ.get("LAT_REPS", "5"))


def best(spec, W, P):
    dev = dict(dtype=torch.float64, device="cuda")
    B = P.shape[0]
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    bnd = [torch.tensor(v, **dev) for v in spec.bounds()]
    p = torch.tensor(P, **dev).contiguous()
    w = torch.tensor(W, **dev).contiguous()
    out = {"x": torch.empty(B, spec.nw, **dev), "f": torch.empty(B, **dev),
           "status": torch.empty(B, dtype=torch.int32, device="cuda"),
           "iters": torch.empty(B, dtype=torch.int32, device="cuda")}
    ts = []
    for _ in range(R + 1):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_device(w, *bnd, p, out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    it = out["iters"].cpu().numpy()
    return min(ts[1:]), it.mean(), it.max()


G = np.load(os.path.join(ROOT, "tests", "golden", "resto_cases.npz"))
W = np.tile(G["w"], (16, 1))[:256]
Pm = np.tile(G["p"], (16, 1))[:256]
t, im, ix = best(make_spec("race_track_2", N=20, T=0.2), W, Pm)
print(f"resto cases B=256: best {t*1e3:.3f} ms, iters mean {im:.1f} max {ix}, {t*1e6/ix:.2f} us per iteration of the longest")
spec = config_spec(3)
P = draw_scenarios(spec, 1024, seed=1003)
t, im, ix = best(spec, np.zeros((1024, spec.nw)), P)
print(f"config 3 cold B=1024: best {t*1e3:.3f} ms, iters mean {im:.1f} max {ix}, {t*1e6/ix:.2f} us per iteration of the longest")
