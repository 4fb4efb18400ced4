"""Benchmark: batched NMPC steps/s on MI355X (BASELINE.json metric).

One *MPC step* = one scenario's per-timestep NLP (Python/NMPC_TT.py:358-365)
solved to termination, warm-started from the previous step's shifted solution,
followed by the closed-loop shift (Python/NMPC_TT.py:13-30).  A bench *step*
advances all B scenarios per GPU by one MPC step; --steps K of them are timed
(K=20 warm-started closed-loop steps per scenario is the headline).

Default mode "fused": the K steps run in ONE launch (nmpc_closed_loop_dev), each
scenario's closed loop on its own wavefront, so a step never waits for another
scenario's slowest solve; for N>1 GPUs the per-step results are RCCL-gathered
once at the end.  The one-launch-per-step mode (solve launch + shift launch,
gather every step) is timed from the same state and reported beside it.

Workload (config 3 of BASELINE.json / SURVEY.md section 8): 4096 scenarios
per GPU, N=20, 10 static obstacles (Python/Race Track 2.py layout), T=0.2,
fp64, the reference's IPOPT options (max_iter=100, tol 1e-8).  Weak scaling:
per-GPU batch fixed as the GPU count grows.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))

FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector = FP64 matrix peak (AMD spec)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table
KFLOP_PER_STAGE_ITER = 7.5   # ~6.2k Riccati + ~1k assembly per stage-iteration


# BASELINE.json "metric" (the headline number is quoted on its config 3: 4096
# scenarios per GPU, N=20, 10 obstacles)
METRIC = "MPC steps/sec (batched scenarios), N=20 9-state UAV, 1/2/4/8 MI355X"


def survey_bytes_per_step(spec, ibar):
    """SURVEY.md 8(d) streamed-KKT byte model (fp64)."""
    nx, nu, m, N = 8, 6, spec.m, spec.N
    s_stage = 8 * ((nx + nu) ** 2 + nx * (nx + nu) + m * nx + 3 * (nx + nu) + 2 * nx + 4 * m + 4 * nu
                   + nx * nx + nu * nx + nu * nu + nx + nu)
    b_iter = 2 * (N + 1) * s_stage
    io = 8 * ((spec.np + spec.nw) + (spec.nw + 8 * (N + 1) + 2))
    return ibar * b_iter + io, s_stage, b_iter, io


def pmc_summary(kernel, steps, batch, warmup):
    """Counters of `kernel`'s timed launch from the newest committed rocprofv3 PMC
    summary (profiles/r*_pmc.csv, written by scripts/rocpd_summary.py from the passes
    of scripts/profile_round.sh) whose profiled runs had this run's kernel, steps, batch
    and warm-up (config 3 and config 5 have their own files; the newest file that holds
    matching rows for both byte counters is taken).  HBM-side bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B):
    FETCH_SIZE counts half the bytes of 8 B/lane and 16 B/lane reads alike on gfx950
    (scripts/fetch_calib.hip, profiles/r02_fetch_calib.csv: 1 GiB read -> 512 MiB
    counted for both widths; WRITE_SIZE exact for 8 B/lane stores).  Both count
    L2-to-fabric traffic, Infinity-Cache hits included (MI355X_MICROARCH.md, HBM)."""
    import csv
    import glob
    # newest round first; within a round any file (r04_pmc.csv, r04_cfg5_pmc.csv, ...)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.csv")),
                   key=lambda f: (os.path.basename(f)[:3], f), reverse=True)
    for path in files:
        vals, run = {}, {}
        with open(path) as fh:
            for row in csv.DictReader(fh):
                if (kernel in row["kernel"] and row.get("steps", "") == str(steps)
                        and row.get("batch", "") == str(batch) and row.get("warmup", "") == str(warmup)):
                    # the launch pairs the problem's class with the equality class behind a
                    # device flag (nmpc_create); the one that ran is the row with the counts
                    if float(row["value"]) >= vals.get(row["counter"], -1.0):
                        vals[row["counter"]] = float(row["value"])
                        run[row["counter"]] = {k: row.get(k) for k in ("ibar", "kernel_ms", "bench_value")}
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            break
    else:
        return None
    out = {"traffic": (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0,
           "source": os.path.relpath(path, ROOT), "profiled_runs": run}
    if vals.get("SQ_WAVE_CYCLES"):
        wc = vals["SQ_WAVE_CYCLES"]
        out["sq"] = {"wait_any_frac": vals.get("SQ_WAIT_ANY", 0) / wc,
                     "valu_active_frac": vals.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                     "lds_active_frac": vals.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                     "wait_inst_frac": vals.get("SQ_WAIT_INST_ANY", 0) / wc}
    if vals.get("TCC_HIT_sum") is not None and vals.get("TCC_MISS_sum") is not None:
        out["l2_hit_rate"] = vals["TCC_HIT_sum"] / max(1.0, vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])
    return out


def cpu_baseline(spec_cfg, cfg, P, lbx, ubx, lbg, ubg, K, W=0, p_step=None, budget_s=15.0, cold=True):
    """Time the compiled CPU restatement (oracle/cpu_ipopt.cpp: C++/OpenMP, the same
    IPOPT restatement with a Riccati Newton step, pinned to the numpy oracle's
    fixtures by tests/test_cpu_restatement.py) on the bench's own workload and window:
    the same scenarios advanced by the same W untimed warm-up MPC steps from w = 0,
    then the same K timed warm-started closed-loop steps (solve + shift) from there --
    the (scenario, step) window of the GPU's timed launch -- one scenario per OpenMP
    thread at a time, until the budget runs out (scenarios split across
    cores).  p_step (W + K, np): the moving obstacles' per-step displacement (config 5)."""
    sys.path.insert(0, ROOT)
    from oracle import cpu_ipopt, nmpc_oracle as orc

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    nthr = max(1, min(16, ncpu))  # the GPU box's CPU share is 16
    # the oracle's description of the same problem (nmpc_amd.config_spec's layouts)
    layout, dynamic = {0: ("nmpc_tt", False), 1: (None, False), 2: (None, False), 3: ("race_track_2", False),
                       4: ("race_track_2", False), 5: ("dynamic", True)}[cfg]
    prob = orc.make_problem(layout, N=spec_cfg.N, T=spec_cfg.T, dynamic=dynamic, model=spec_cfg.model)
    assert prob.np_ == spec_cfg.np and prob.n_obs == spec_cfg.n_obs, "CPU baseline problem differs from the bench's"
    # the W warm-up steps, untimed (the GPU runs them as W per-step launches), for as many
    # scenarios as a warm-up budget allows (all 4,096 of config 3 take ~1 s; config 5's
    # N = 50 solves are ~5x dearer): the timed window runs on the fully warmed ones
    P1, W1 = P, None
    sel = np.arange(P.shape[0])
    if W > 0:
        r0 = cpu_ipopt.closed_loop(prob, P, W, lbx, ubx, lbg, ubg, orc.REFERENCE_OPTS, vt=12.0, wt=0.01,
                                   p_step=None if p_step is None else p_step[:W], threads=nthr,
                                   budget_s=budget_s)
        sel = np.flatnonzero(r0["steps"] == W)
        P1, W1 = r0["p"][sel], r0["w"][sel]
    cpu_baseline.start = (P1, W1, sel)
    t0 = time.perf_counter()
    r = cpu_ipopt.closed_loop(prob, P1, K, lbx, ubx, lbg, ubg, orc.REFERENCE_OPTS, vt=12.0, wt=0.01,
                              p_step=None if p_step is None else p_step[W:W + K], budget_s=budget_s,
                              threads=nthr, W0=W1)
    wall = time.perf_counter() - t0
    done = r["steps"]
    n = int(done.sum())
    rows = np.flatnonzero(done > 0)
    # records keyed by the row of the timed sample (P1 / W1 order)
    recs = [(int(b), k, int(r["status"][b, k]), r["u0"][b, k].copy(), float(r["f"][b, k]))
            for b in rows for k in range(int(done[b]))]
    cpu_baseline.records = recs
    cpu_baseline.sample_rows = int(rows.max()) + 1 if len(rows) else 0
    its = np.concatenate([r["iter"][b, :done[b]] for b in rows]) if len(rows) else np.zeros(0)
    sts = np.concatenate([r["status"][b, :done[b]] for b in rows]) if len(rows) else np.zeros(0, int)
    tsv = np.concatenate([r["solve_s"][b, :done[b]] for b in rows]) if len(rows) else np.zeros(0)
    def pct(v):
        return {"p50_ms": float(np.percentile(v, 50) * 1e3), "p99_ms": float(np.percentile(v, 99) * 1e3),
                "max_ms": float(v.max() * 1e3)} if len(v) else None
    out = {"value": n / wall, "unit": "MPC steps/s", "cores": nthr, "kind": "port",
           "sample": f"{n} warm-started closed-loop MPC steps (solve + shift) of the GPU's timed window -- "
                     f"steps {W}..{W + K - 1} after the same {W} untimed warm-up steps, up to {K} per scenario, "
                     f"{len(rows)} of the bench's config-{cfg} scenarios ({len(sel)} warmed within the budget) -- "
                     f"by oracle/cpu_ipopt.cpp (CPU "
                     f"restatement, not CasADi: C++/OpenMP IPOPT restatement with a Riccati step), "
                     f"{nthr} threads, budget {budget_s:.0f}s, wall {wall:.1f}s",
           "mean_ip_iterations": float(its.mean()) if n else None,
           "iterations_per_s_per_core": float(its.sum() / wall / nthr) if n else None,
           "per_solve_wall": pct(tsv),
           "status_histogram": {int(k): int(v) for k, v in zip(*np.unique(sts, return_counts=True))}}
    if not cold:
        return out
    # cold-start leg (cold u = 0 and warm-started): every scenario's NLP of
    # the timed window's first step from u = 0, the same threads
    t1 = time.perf_counter()
    rc = cpu_ipopt.solve_batch(prob, np.zeros((P1.shape[0], spec_cfg.nw)), P1, lbx, ubx, lbg, ubg,
                               orc.REFERENCE_OPTS, threads=nthr)
    cwall = time.perf_counter() - t1

    cold = {"value": P1.shape[0] / cwall, "unit": "NLP solves/s", "solves": int(P1.shape[0]), "wall_s": cwall,
            "mean_ip_iterations": float(rc["iter"].mean()), "per_solve_wall": pct(rc["solve_s"]),
            "status_histogram": {int(k): int(v) for k, v in zip(*np.unique(rc["status"], return_counts=True))},
            "sample": f"cold solves (u = 0) of the timed window's first step, {P1.shape[0]} scenarios, {nthr} threads"}
    out["cold_start"] = cold
    return out


def parity_sample(solver, spec, start, K, records, bnd, dev, p_step=None, tol=1e-6):
    """GPU vs the CPU leg on the same (scenario, step) pairs: the CPU leg's scenarios
    rerun through nmpc_closed_loop_dev from the CPU leg's own start of the timed window
    (its p and warm start after the W warm-up steps, the same target controls and
    obstacle motion), compared step by step until a chain first disagrees -- status, and
    for converged steps u0 and f within tol (1 + |ref|) (the north-star 1e-6)."""
    import torch

    rows = sorted({r[0] for r in records})
    if not rows:
        return None
    idx = {r: j for j, r in enumerate(rows)}
    B = len(rows)
    P1, W1, _ = start
    f64 = dict(dtype=torch.float64, device=dev)
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device=dev)}
    w0 = torch.zeros(B, spec.nw, **f64) if W1 is None else torch.tensor(W1[rows], **f64).contiguous()
    solver.closed_loop_device(K, *bnd, torch.tensor(P1[rows], **f64).contiguous(), w0,
                              torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64), hist,
                              p_step=None if p_step is None else torch.tensor(p_step, **f64).contiguous())
    H = {k: v.cpu().numpy() for k, v in hist.items()}
    by = {}
    for row, k, st, u0, f in records:
        by.setdefault(row, []).append((k, st, u0, f))
    compared = agree_status = before_div = chains_same = 0
    max_u, max_f = 0.0, 0.0
    for row, steps in by.items():
        j, same = idx[row], True
        for k, st, u0, f in sorted(steps, key=lambda t: t[0]):
            compared += 1
            gs = int(H["status"][k, j])
            agree_status += gs == st
            if not same:
                continue
            ok = gs == st
            if ok and st in (0, 1):
                eu = float(np.max(np.abs(H["u"][k, j, :len(u0)] - u0) / (1 + np.abs(u0))))
                ef = abs(float(H["f"][k, j]) - f) / (1 + abs(f))
                ok = eu <= tol and ef <= tol
                if ok:
                    max_u, max_f = max(max_u, eu), max(max_f, ef)
            if ok:
                before_div += 1
            else:
                same = False
        chains_same += same
    return {"scenarios": len(by), "steps_compared": compared,
            "status_agreement": agree_status / max(1, compared),
            "steps_before_first_divergence": before_div, "chains_identical": chains_same,
            "max_u0_relerr": max_u, "max_f_relerr": max_f, "tol": tol,
            "reference": "oracle/cpu_ipopt.cpp (the cpu_baseline leg's own solves; pinned to oracle/nmpc_oracle.py by tests/test_cpu_restatement.py)"}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_cmd(n, argv, port):
    """The command bench.py --gpus N runs when no launcher started it: one process per GPU
    through torch.distributed.run on this node (127.0.0.1 rendezvous), each rank running
    this same script with the same arguments (WORLD_SIZE is then set, so no rank relaunches)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def launch_ranks(n, argv):
    """Parent of an N-rank run: starts the ranks as a child process (never exec: this
    process stays the parent and has touched no GPU), streams every non-JSON line to
    stderr as it arrives, and prints rank 0's JSON line last on stdout.  Returns the
    launcher's exit code (non-zero also when no JSON line came back)."""
    import subprocess
    import threading

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the host driver's only mode)
    proc = subprocess.Popen(rank_launch_cmd(n, argv, _free_port()), stdout=subprocess.PIPE, env=env, text=True,
                            bufsize=1)
    lines = []

    def pump():
        for ln in proc.stdout:
            if ln.lstrip().startswith("{"):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()
    t = threading.Thread(target=pump, daemon=True)
    t.start()
    rc = proc.wait()
    t.join()
    if lines:
        print(lines[-1], flush=True)
    elif rc == 0:
        sys.stderr.write("bench.py: the ranks exited without a JSON line\n")
        rc = 1
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="closed-loop MPC steps per scenario (timed)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="scenarios per GPU")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--mode", choices=["fused", "per_step", "cold"], default="fused",
                    help="fused: K closed-loop steps per scenario in one launch (nmpc_closed_loop_dev); "
                         "per_step: one solve launch + shift launch per step; cold: per step, u=0 each step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true", help="skip the per-step-launch comparison line")
    ap.add_argument("--in-order", action="store_true",
                    help="fused mode: dispatch scenarios in index order (no longest-first order)")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the config-5 side leg (N=50, 10 obstacles of which 6 move; N=1 only)")
    ap.add_argument("--config5-batch", type=int, default=8192, help="config-5 leg: scenarios (BASELINE config 5)")
    ap.add_argument("--config5-cpu-scenarios", type=int, default=2048,
                    help="config-5 leg: scenarios in the CPU baseline's bounded sample")
    ap.add_argument("--config5-cpu-budget", type=float, default=8.0)
    ap.add_argument("--dump-rows", default="",
                    help="fused mode: rank 0 saves the gathered (scenarios, 8K) per-step rows (u0, f, status) "
                         "of the timed launch to this .npy (multi-rank rehearsal test)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher around us: start the N rank processes ourselves (before any GPU call
        # of this process, which never initialises the GPU) and relay rank 0's line
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} does not match the launcher's WORLD_SIZE={env_world}; "
                         f"the line would be mislabelled")

    import torch
    import torch.distributed as dist
    from nmpc_amd import config_spec, draw_scenarios

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    spec = config_spec(args.config)
    B, K, W = args.batch, args.steps, args.warmup
    # the config-5 side leg (BASELINE config 5, Dynamic Obstacle avoidance.m:211-231): N=1 only
    leg5 = world == 1 and args.config != 5 and args.mode == "fused" and not args.no_config5
    cpu_res = cpu5 = None
    if world == 1 and not args.no_cpu_baseline:  # OpenMP threads, before the GPU is initialised
        lb = spec.bounds()
        cpu_res = cpu_baseline(spec, args.config, draw_scenarios(spec, B, seed=1000 + args.config), *lb, K, W,
                               p_step=obstacle_pstep(spec, W + K), budget_s=args.cpu_budget)
        cpu_res_start, cpu_res_records = cpu_baseline.start, cpu_baseline.records
        if leg5:
            s5 = config_spec(5)
            cpu5 = cpu_baseline(s5, 5, draw_scenarios(s5, args.config5_batch, seed=1005)[:args.config5_cpu_scenarios],
                                *s5.bounds(), K, W, p_step=obstacle_pstep(s5, W + K), budget_s=args.config5_cpu_budget,
                                cold=False)
    # NMPC_BENCH_BACKEND=gloo rehearses the multi-rank path on one GPU (all ranks on
    # cuda:0); the measured configuration is one process per GPU over RCCL ("nccl")
    backend = os.environ.get("NMPC_BENCH_BACKEND", "nccl")
    dev_idx = local_rank % max(1, torch.cuda.device_count()) if world > 1 else 0
    if world > 1:
        torch.cuda.set_device(dev_idx)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", dev_idx)
    ctx = dict(world=world, rank=rank, backend=backend, dev=dev, dist=dist)

    m = measure(args, ctx, args.config, B, K, W, args.mode, per_step_side=(args.mode == "fused" and not args.no_per_step),
                dump_rows=args.dump_rows)
    m5 = measure(args, ctx, 5, args.config5_batch, K, W, "fused", per_step_side=False) if leg5 else None

    if rank == 0:
        res = result_line(args, m, world)
        if m["side"] is not None:
            res["per_step_launch"] = m["side"]
        if cpu_res is not None:
            res["cpu_baseline"] = cpu_res
            if world == 1 and cpu_res_records:
                res["parity_sample"] = parity_sample(m["solver"], m["spec"], cpu_res_start, K, cpu_res_records,
                                                     m["bnd"], dev, p_step=m["ps_np"][W:W + K] if m["ps_np"] is not None
                                                     else None)
        if m5 is not None:
            r5 = result_line(args, m5, world)
            leg = {k: r5[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup", "config", "roofline",
                                      "mean_ip_iterations", "status_histogram", "dispatch", "scheduler_error",
                                      "steps_done") if k in r5}
            leg["note"] = ("BASELINE config 5 (N=50, 10 obstacles of which 6 move per MATLAB/Dynamic Obstacles/"
                           "Dynamic Obstacle avoidance.m:211-231), timed like the headline: W warm-up MPC steps, "
                           "then K closed-loop steps per scenario in one launch (HIP events on the launch stream); "
                           "a side leg, not the headline value")
            if cpu5 is not None:
                leg["cpu_baseline"] = cpu5
            res["config5"] = leg
        print(json.dumps(res))
        if args.dump_rows and args.mode == "fused":
            np.save(args.dump_rows, m["rows"].cpu().numpy())
    if world > 1:
        dist.destroy_process_group()


def obstacle_pstep(spec, n):
    """Moving obstacles (config 5: MATLAB/Dynamic Obstacles/Dynamic Obstacle avoidance.m:213-230,
    from MPC iteration 195 as in the config-5 fixtures; the W warm-up steps come first):
    (n, np) per-step parameter increments, or None for a static layout."""
    if spec.np <= spec.np_min:
        return None
    from nmpc_amd.targets import obstacle_steps
    return obstacle_steps(195, n, spec.np)


def measure(args, ctx, cfg, B, K, W, mode, per_step_side=False, dump_rows=""):
    """One configuration on this rank's GPU: W warm-up MPC steps, then exactly K timed steps
    bracketed by barrier + synchronize (fused: one launch, timed twice over -- once on scratch
    copies of the same state, then the timed launch); HIP events on the launch stream give the
    kernel time.  Returns the raw measurements."""
    import torch
    from nmpc_amd import nlpsol, config_spec, draw_scenarios, REFERENCE_OPTS
    from nmpc_amd.dist import shard, pack_result, gather_rows, gather_closed_loop, pack_closed_loop
    from nmpc_amd.schedule import longest_first

    world, rank, backend, dev, dist = ctx["world"], ctx["rank"], ctx["backend"], ctx["dev"], ctx["dist"]
    spec = config_spec(cfg)
    ps_np = obstacle_pstep(spec, W + K)

    def all_reduce(t, op):
        if backend == "nccl":
            dist.all_reduce(t, op=op)
        else:
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)
    # global scenario stream, sliced per rank (results independent of world size)
    P_all = draw_scenarios(spec, B * world, seed=1000 + cfg)
    P = P_all[shard(B * world, world, rank)]
    lbx, ubx, lbg, ubg = spec.bounds()
    solver = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)

    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)
    bnd = [torch.tensor(v, **f64) for v in (lbx, ubx, lbg, ubg)]
    p0 = torch.tensor(P, **f64).contiguous()
    w0 = torch.zeros(B, spec.nw, **f64)
    v_t = torch.full((B,), 12.0, **f64)   # target speed, Python/NMPC_TT.py:25
    w_t = torch.full((B,), 0.01, **f64)   # target turn rate
    stream = torch.cuda.current_stream()
    pstep = None if ps_np is None else torch.tensor(ps_np, **f64)

    def hist_bufs(k):
        return {"u": torch.empty(k, B, 6, **f64), "f": torch.empty(k, B, **f64), "fov": torch.zeros(k, B, **f64),
                "status": torch.empty(k, B, **i32), "iters": torch.empty(k, B, **i32)}

    out = {"x": torch.empty(B, spec.nw, **f64), "f": torch.empty(B, **f64),
           "status": torch.empty(B, **i32), "iters": torch.empty(B, **i32)}

    def per_step(p, w, hist, k, cold, timed_events=None, g=None):
        """One batched step: solve launch (+ shift launch) (+ per-step gather)."""
        if timed_events is not None:
            timed_events[0].record(stream)
        solver.solve_device(torch.zeros_like(w) if cold else w, *bnd, p, out, stream=stream)
        if timed_events is not None:
            timed_events[1].record(stream)
        if not cold:
            solver.shift_device(p, out["x"], w, v_t, w_t, stream=stream)
            if pstep is not None:  # obstacle coordinates move after the step (nmpc_closed_loop_dev's p_step)
                p[:, spec.np_min:] += pstep[k if g is None else g, spec.np_min:]
        if world > 1:  # per-step gather of (u0, f, status)
            gather_rows(pack_result(out["x"], out["f"], out["status"], spec.nu), world, total=B * world)
        hist["u"][k].zero_(); hist["u"][k][:, :spec.nu].copy_(out["x"][:, :spec.nu]); hist["f"][k].copy_(out["f"])
        hist["iters"][k].copy_(out["iters"]); hist["status"][k].copy_(out["status"])

    def fused(p, w, hist, k_steps, timed_events=None, order=None):
        if timed_events is not None:
            timed_events[0].record(stream)
        solver.closed_loop_device(k_steps, *bnd, p, w, v_t, w_t, hist, stream=stream, order=order, check=False,
                                  p_step=None if pstep is None else pstep[W:W + k_steps].contiguous())
        if timed_events is not None:
            timed_events[1].record(stream)
        if world > 1:  # the only exchange: final gather of every step's (u0, f, status)
            rows = gather_closed_loop(hist, world, total=B * world)
        else:
            rows = pack_closed_loop(hist) if dump_rows else None
        if timed_events is not None:
            fused.rows = rows

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed_run(mode, p, w):
        """Warmup W steps (advancing the closed loop), then time exactly K steps."""
        hw, ht = hist_bufs(max(W, 1)), hist_bufs(K)
        # warmup: W MPC steps advance the closed loop (one solve + shift launch per step)
        for k in range(W):
            per_step(p, w, hw, k, mode == "cold")
        order = None
        if mode == "fused" and W > 0 and not args.in_order:
            # longest-expected-first dispatch from the iterations of the W warm-up
            # steps, which precede the timed steps (nmpc_amd.schedule)
            order = longest_first(hw["iters"][:W])
        if mode == "fused":
            # the timed launch once on scratch copies of the same state (code objects,
            # workspace): the fused kernel then runs exactly twice with identical work
            fused(p.clone(), w.clone(), hist_bufs(K), K, order=order)
        barrier_sync()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(1 if mode == "fused" else K)]
        t0 = time.perf_counter()
        if mode == "fused":
            fused(p, w, ht, K, evs[0], order=order)
        else:
            for k in range(K):
                per_step(p, w, ht, k, mode == "cold", evs[k], g=W + k)
        barrier_sync()
        elapsed = time.perf_counter() - t0
        if mode == "fused":  # every (scenario, step) ran: raises otherwise (after the timed region)
            timed_run.info = solver.check_closed_loop(B, K)
        kern_ms = [a.elapsed_time(b) for a, b in evs]
        el_t = torch.tensor([elapsed], **f64)
        tot = torch.stack([ht["iters"].sum().double(), torch.tensor(float(B * K), **f64)])
        if world > 1:
            all_reduce(el_t, dist.ReduceOp.MAX)
            all_reduce(tot, dist.ReduceOp.SUM)
        sts = ht["status"].cpu().numpy()
        hist = {int(s_): int((sts == s_).sum()) for s_ in np.unique(sts)}
        timed_run.fov = float(ht["fov"].mean().item())
        timed_run.chain = ht["iters"].sum(0).cpu().numpy()
        return float(el_t.item()), kern_ms, float(tot[0].item() / tot[1].item()), hist

    elapsed, kern_ms, ibar, status_hist = timed_run(mode, p0.clone(), w0.clone())
    res = {"cfg": cfg, "spec": spec, "B": B, "K": K, "W": W, "mode": mode, "elapsed": elapsed, "kern_ms": kern_ms,
           "ibar": ibar, "status_hist": status_hist, "solver": solver, "bnd": bnd, "ps_np": ps_np,
           "pstep": pstep, "fov": timed_run.fov if mode == "fused" else None,
           "chain": timed_run.chain, "info": timed_run.info if mode == "fused" else None,
           "rows": getattr(fused, "rows", None), "side": None}
    if per_step_side:
        e2, km2, ib2, h2 = timed_run("per_step", p0.clone(), w0.clone())
        res["side"] = {"mode": "per_step (one solve launch + one shift launch per MPC step)",
                       "value": B * world * K / e2, "ms_per_step": e2 / K * 1e3,
                       "kernel_avg_ms": float(np.mean(km2)), "kernel_max_ms": float(np.max(km2)),
                       "mean_ip_iterations": ib2, "status_histogram": h2}
    return res


def result_line(args, m, world):
    """The bench JSON fields of one measured configuration (BASELINE.json metric)."""
    spec, B, K, W, mode = m["spec"], m["B"], m["K"], m["W"], m["mode"]
    elapsed, kern_ms, ibar = m["elapsed"], m["kern_ms"], m["ibar"]
    total_steps = B * world * K
    value = total_steps / elapsed
    ms_per_step = elapsed / K * 1e3
    n_launch = len(kern_ms)
    kern_avg_s = float(np.mean(kern_ms)) / 1e3
    steps_per_launch = K if mode == "fused" else 1
    kname = "nmpc_closed_loop_kernel" if mode == "fused" else "nmpc_solve_kernel"
    if mode == "fused" and m["info"]["policy"] == "step_queues":
        kname = "nmpc_closed_loop_sched_kernel"
    flops_launch = B * steps_per_launch * ibar * (spec.N + 1) * KFLOP_PER_STAGE_ITER * 1e3
    achieved_tf = flops_launch / kern_avg_s / 1e12
    bps, s_stage, b_iter, io = survey_bytes_per_step(spec, ibar)
    achieved_gbs = B * steps_per_launch * bps / kern_avg_s / 1e9
    pmc = pmc_summary(kname, K if mode == "fused" else None, B, W)
    traffic = pmc["traffic"] if pmc else None
    mode_txt = {"fused": f"{K} warm-started closed-loop MPC steps per scenario in one launch",
                "per_step": "warm-started closed-loop MPC steps, one launch per step",
                "cold": "cold-start (u=0) solves, one launch per step"}[mode]
    res = {
        "metric": METRIC,
        "value": value, "unit": "MPC steps/s", "n_gpus": world, "steps": K,
        "warmup": W, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": (f"config 4 family: {B * world} scenarios sharded {B}/GPU over {world} GPUs, "
                                if world > 1 and m["cfg"] == 3 else "")
                               + f"config {m['cfg']}: batch={B}/GPU, "
                               f"{'no-gimbal 5-state' if spec.model == 'uav5' else '8-state UAV+gimbal'}, "
                               f"N={spec.N}, {spec.n_obs} obstacles"
                               + (" (moving per MATLAB/Dynamic Obstacles schedule)" if m["pstep"] is not None
                                  else " static (Race Track 2.py layout)" if spec.n_obs else "")
                               + f", T={spec.T}, "
                               f"reference IPOPT opts, {mode_txt}",
                   "global_batch": B * world, "seq_len": spec.N, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_unit": "bytes per launch between L2 and the fabric (Infinity Cache or HBM): "
                                     "2*FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC (calibrated x2 for 8 and 16 B/lane "
                                     "reads, scripts/fetch_calib.hip)",
                     "traffic_source": pmc["source"] if pmc else None,
                     "counter_bytes_frac": (traffic / kern_avg_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                     "pmc_runs": pmc["profiled_runs"] if pmc else None,
                     "sq": pmc.get("sq") if pmc else None,
                     "l2_hit_rate": pmc.get("l2_hit_rate") if pmc else None,
                     "kernel": kname, "kernel_avg_ms": kern_avg_s * 1e3, "launches": n_launch,
                     "model": f"SURVEY 8(d) streamed-KKT bytes: I_bar x B_iter + IO = {bps:.0f} B per "
                              f"MPC step (I_bar={ibar:.2f}, B_iter={b_iter} B, IO={io} B) x B={B} x "
                              f"{steps_per_launch} step(s) per launch / kernel time",
                     "fp64": {"achieved_tflops": achieved_tf, "peak_tflops": FP64_PEAK_TFLOPS,
                              "frac": achieved_tf / FP64_PEAK_TFLOPS,
                              "model": f"{KFLOP_PER_STAGE_ITER} kflop/stage-iteration x (N+1) x I_bar"},
                     "io_only_GBs": B * steps_per_launch * io / kern_avg_s / 1e9},
        "mean_ip_iterations": ibar,
        "status_histogram": m["status_hist"],
    }
    if mode == "fused":
        # the launch is bounded by its longest scenario chain (K steps of up to max_iter
        # iterations each) and by the total work over the persistent slots
        ch = m["chain"]
        info = m["info"]
        slots = info["launched_waves"] if info["policy"] == "step_queues" else B
        res["roofline"]["chain"] = {
            "max_chain_iterations": int(ch.max()), "mean_chain_iterations": float(ch.mean()),
            "total_iterations": int(ch.sum()), "slots": int(min(slots, B)),
            "ms_per_chain_iteration": kern_avg_s * 1e3 / float(ch.max()),
            "work_bound_iterations_per_slot": float(ch.sum()) / min(slots, B),
            "note": "launch >= max(max_chain, total/slots) x per-iteration time"}
        first = ("index order" if (args.in_order or W == 0) else
                 "longest-expected-first by the iterations of the "
                 f"{W} warm-up MPC steps that precede the timed steps (nmpc_amd.schedule)")
        if info["policy"] == "step_queues":
            res["dispatch"] = (f"step queues: {info['launched_waves']} persistent waves claim (scenario, step) "
                               f"pairs whose previous step is done, lowest step first, scenarios pinned to an "
                               f"XCD; initial order {first}")
        else:
            res["dispatch"] = f"one workgroup per scenario, {first}"
        res["scheduler_error"] = info["scheduler_error"]
        res["steps_done"] = info["steps_done"]
        if m["fov"] is not None:
            res["closed_loop_fov_error_mean_m"] = m["fov"]  # Python/NMPC_TT.py:433-437 metric, per step
    return res


if __name__ == "__main__":
    main()
