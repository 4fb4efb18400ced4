"""Dev tool: where the fused closed-loop launch's time goes, from per-step realtime
stamps (NMPC_STEP_TIMES).  The bench's workload (config 3, B=4096, W warm-up steps,
longest-expected-first order, K timed steps); reports the launch span, the longest
chains' busy / waiting time and per-iteration cost, and the number of steps in flight
over time (how full the GPU is in the tail)."""
import os
import sys

import numpy as np
import torch

os.environ["NMPC_STEP_TIMES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS  # noqa: E402
from nmpc_amd.schedule import longest_first  # noqa: E402

B, K, W = 4096, 20, 5
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
order = longest_first(hw["iters"])
for rep in range(2):
    pp, ww = p.clone(), w.clone()
    h = {"iters": torch.empty(K, B, **i32), "status": torch.empty(K, B, **i32)}
    s.closed_loop_device(K, *bnd, pp, ww, vt, wt, h, order=order)
    torch.cuda.synchronize()
t = s.closed_loop_times(B, K).astype(np.int64)
it = h["iters"].cpu().numpy()
if len(sys.argv) > 1:  # raw record for offline analysis (scripts/sched_sim.py)
    np.savez_compressed(sys.argv[1], times=t, iters=it, status=h["status"].cpu().numpy(),
                        order=order.cpu().numpy())
st, en = t[:, :, 0], t[:, :, 1]
t0 = st.min()
span = (en.max() - t0) / 1e5  # ms (100 MHz)
chain = it.sum(0)
busy = (en - st).sum(0) / 1e5
first, last = (st.min(0) - t0) / 1e5, (en.max(0) - t0) / 1e5
print(f"launch span {span:.1f} ms; total iterations {it.sum()}; mean busy per scenario {busy.mean():.2f} ms")
top = np.argsort(-chain)[:12]
print("longest chains: iterations, busy ms, first start ms, last end ms, waiting ms, us/iteration")
for b in top:
    print(f"  {b:5d} {chain[b]:5d} {busy[b]:7.1f} {first[b]:7.1f} {last[b]:7.1f} {last[b] - first[b] - busy[b]:7.1f} "
          f"{1e3 * busy[b] / chain[b]:6.1f}")
per_it = (en - st) / 1e2 / np.maximum(it, 1)  # us per iteration of every step
print(f"us per iteration: all steps mean {np.average(per_it, weights=it):.1f}; steps with 100 iterations "
      f"{per_it[it >= 100].mean():.1f}")
# effective shader clock per step: s_memtime cycles (t[2] >> 24) over the realtime span
cyc = (t[:, :, 2] >> 24).astype(np.float64)
mhz = cyc / np.maximum(en - st, 1) * 100.0
print(f"effective shader clock per step (MHz): mean {np.average(mhz, weights=en - st):.0f}, "
      f"p1 {np.percentile(mhz, 1):.0f}, p99 {np.percentile(mhz, 99):.0f}")
# steps in flight over time
edges = np.arange(0, span + 10, 10.0)
inflight = []
for a in edges[:-1]:
    lo, hi = t0 + a * 1e5, t0 + (a + 10) * 1e5
    ov = np.clip(np.minimum(en, hi) - np.maximum(st, lo), 0, None).sum() / (10 * 1e5)
    inflight.append(ov)
print("average steps in flight per 10 ms window:", " ".join(f"{v:.0f}" for v in inflight))
late = np.argsort(-last)[:12]
print("latest-finishing scenarios: iterations, busy ms, first start ms, last end ms, waiting ms, us/iteration")
for b in late:
    print(f"  {b:5d} {chain[b]:5d} {busy[b]:7.1f} {first[b]:7.1f} {last[b]:7.1f} {last[b] - first[b] - busy[b]:7.1f} "
          f"{1e3 * busy[b] / chain[b]:6.1f}")
b = late[0]
print("last scenario per step: iterations / start ms / duration ms / gap before ms:")
prev = 0.0
for k in range(K):
    s0, e0 = (st[k, b] - t0) / 1e5, (en[k, b] - t0) / 1e5
    print(f"  k={k:2d} it={it[k, b]:3d} start={s0:7.1f} dur={e0 - s0:6.1f} gap={s0 - prev:6.1f} "
          f"status={h['status'][k, b].item()} clock={mhz[k, b]:.0f} MHz")
    prev = e0
wait = last - first - busy
b = int(np.argmax(wait))
print(f"largest waiting scenario {b}: waited {wait[b]:.1f} ms; per step: iterations / start ms / duration ms / gap before ms / wave")
prev = None
for k in range(K):
    s0, e0 = (st[k, b] - t0) / 1e5, (en[k, b] - t0) / 1e5
    print(f"  k={k:2d} it={it[k, b]:3d} start={s0:7.1f} dur={e0 - s0:6.1f} gap={(s0 - prev) if prev is not None else 0:6.1f} "
          f"wave={(int(t[k, b, 2]) >> 8) & 0xFFFF} xcc={int(t[k, b, 2]) & 255}")
    prev = e0
