"""Dev tool (round 5): replay a fused closed-loop launch's measured per-step durations
(scripts/step_times.py <out.npz>) through scheduling policies of the step-queue
scheduler, to see how much of the launch's tail a policy leaves.  The step durations are
taken as given (independent of which wave runs them); 8 XCD sets of 128 waves, scenario
set = dispatch position mod 8, as nmpc_closed_loop_sched_kernel."""
import heapq
import sys

import numpy as np

z = np.load(sys.argv[1])
t, it, order = z["times"], z["iters"], z["order"]
d = (t[:, :, 1] - t[:, :, 0]).astype(np.float64) / 1e5  # ms
K, B = d.shape
NX, WPX = int(sys.argv[2]) if len(sys.argv) > 2 else 8, 1024 // (int(sys.argv[2]) if len(sys.argv) > 2 else 8)
pos = np.empty(B, int)
pos[order] = np.arange(B)
xset = pos % NX
chain = d.sum(0)
print(f"B={B} K={K}: measured span {(t[:, :, 1].max() - t[:, :, 0].min()) / 1e5:.1f} ms; "
      f"longest busy chain {chain.max():.1f} ms (scenario {chain.argmax()}); work/slot {d.sum() / (NX * WPX):.1f} ms")


def simulate(prio):
    """prio(b, k, done_ms, done_its, pub_time) -> sort key (smallest first) of a claimable step."""
    span = 0.0
    for x in range(NX):
        sc = [b for b in order if xset[b] == x]
        ready = []  # (key, seq, b, k)
        seq = 0
        acc_ms = np.zeros(B)
        for b in sc:
            heapq.heappush(ready, (prio(b, 0, 0.0, 0, 0.0, seq), seq, b, 0))
            seq += 1
        waves = [(0.0, w) for w in range(WPX)]
        heapq.heapify(waves)
        running = []  # (end, b, k)
        now = 0.0
        while ready or running:
            # free waves claim
            while ready and waves and waves[0][0] <= now:
                _, w = heapq.heappop(waves)
                _, _, b, k = heapq.heappop(ready)
                heapq.heappush(running, (now + d[k, b], b, k, w))
            if not running:
                break
            end, b, k, w = heapq.heappop(running)
            now = end
            span = max(span, end)
            acc_ms[b] += d[k, b]
            heapq.heappush(waves, (now, w))
            if k + 1 < K:
                heapq.heappush(ready, (prio(b, k + 1, acc_ms[b], it[:k + 1, b].sum(), now, seq), seq, b, k + 1))
                seq += 1
    return span


HOT = 50
policies = {
    "current: hot (prev >= 50 its) first, lowest step, FIFO": lambda b, k, ms, its, tp, s: (
        0 if (k > 0 and it[k - 1, b] >= HOT) else 1, k, s),
    "lowest step, FIFO (no hot family)": lambda b, k, ms, its, tp, s: (k, s),
    "most iterations so far first": lambda b, k, ms, its, tp, s: (-its, s),
    "largest predicted remaining (K-k) x mean its so far": lambda b, k, ms, its, tp, s: (
        -(K - k) * (its / k if k else 0), s),
    "hot first, then most iterations so far": lambda b, k, ms, its, tp, s: (
        0 if (k > 0 and it[k - 1, b] >= HOT) else 1, -its, s),
    "largest busy ms so far first": lambda b, k, ms, its, tp, s: (-ms, s),
    "(proxy) largest (K-k) x mean its, step 0 predicted by its own iterations": lambda b, k, ms, its, tp, s: (
        -(K - k) * (its / k if k else it[0, b]), s),
    "(proxy) largest (K-k) x mean ms, step 0 predicted by its own duration": lambda b, k, ms, its, tp, s: (
        -(K - k) * (ms / k if k else d[0, b]), s),
    "oracle: largest remaining busy first": lambda b, k, ms, its, tp, s: (-d[k:, b].sum(), s),
}
for name, f in policies.items():
    print(f"  {simulate(f):7.1f} ms  {name}")

# the same with the bounding chain made as fast as the next one (what the launch would be
# bounded by once that chain is cut): its step durations scaled to the second-longest chain
b0 = int(chain.argmax())
second = np.sort(chain)[-2]
d[:, b0] *= second / chain[b0]
print(f"with scenario {b0}'s chain scaled to {second:.1f} ms:")
for name, f in policies.items():
    print(f"  {simulate(f):7.1f} ms  {name}")
# and every step 15% faster (a per-iteration latency cut)
d *= 0.85
chain = d.sum(0)
print(f"and every step 15% faster (longest busy chain {chain.max():.1f} ms, work/slot {d.sum() / (NX * WPX):.1f} ms):")
for name, f in policies.items():
    print(f"  {simulate(f):7.1f} ms  {name}")

# what-if: max_iter steps (100 iterations, mostly restoration) f% faster, other steps unchanged
z2 = np.load(sys.argv[1])
d0 = (z2["times"][:, :, 1] - z2["times"][:, :, 0]).astype(np.float64) / 1e5
for fct in (0.95, 0.9, 0.85, 0.8):
    d = d0 * np.where(it >= 100, fct, 1.0)
    chain = d.sum(0)
    print(f"max_iter steps x{fct}: longest chain {chain.max():.1f} ms, current policy "
          f"{simulate(policies['current: hot (prev >= 50 its) first, lowest step, FIFO']):.1f} ms")
