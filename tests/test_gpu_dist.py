"""GPU test of bench.py's multi-rank fused path at world size 2 (gloo, both ranks on
cuda:0): each rank runs nmpc_closed_loop_dev on its contiguous shard of the global
scenario stream, then the single exchange of the fused mode (dist.gather_closed_loop,
an all-gather of every step's u0, f and status) assembles the whole batch.  The
gathered rows must equal a single-rank launch over the whole batch bitwise: results
do not depend on the GPU count (SURVEY 8(e), weak scaling by scenario shards)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOTAL, K = 96, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _closed_loop(P, K):
    import torch
    from nmpc_amd import nlpsol, config_spec, REFERENCE_OPTS

    spec = config_spec(3)
    s = nlpsol("solver", "ipopt", spec, REFERENCE_OPTS)
    f64 = dict(dtype=torch.float64, device="cuda")
    B = P.shape[0]
    bnd = [torch.tensor(v, **f64) for v in spec.bounds()]
    hist = {"u": torch.empty(K, B, 6, **f64), "f": torch.empty(K, B, **f64),
            "status": torch.empty(K, B, dtype=torch.int32, device="cuda")}
    s.closed_loop_device(K, *bnd, torch.tensor(P, **f64), torch.zeros(B, spec.nw, **f64),
                         torch.full((B,), 12.0, **f64), torch.full((B,), 0.01, **f64), hist)
    return hist


def _rank(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
    import torch
    import torch.distributed as dist
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.dist import shard, gather_closed_loop

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P_all = draw_scenarios(config_spec(3), TOTAL, seed=1003)
    hist = _closed_loop(P_all[shard(TOTAL, world, rank)], K)
    rows = gather_closed_loop(hist, world)
    if rank == 0:
        q.put(rows.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_fused_gather_equals_single_rank():
    import torch.multiprocessing as mp
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.dist import pack_closed_loop

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = pack_closed_loop(_closed_loop(draw_scenarios(config_spec(3), TOTAL, seed=1003), K)).cpu().numpy()
    assert got.shape == ref.shape == (TOTAL, 8 * K)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.timeout(600)
def test_config4_eight_rank_bench_rehearsal_equals_single_rank():
    """BASELINE config 4's global batch through bench.py's own multi-rank fused path,
    started exactly as the driver starts it -- `python bench.py --gpus 8 ...` with no
    launcher around it: bench.py starts its 8 ranks itself (torch.distributed.run as a
    child process), 32,768 scenarios sharded 4,096 per rank (gloo backend via
    NMPC_BENCH_BACKEND, every rank on cuda:0 of this one-GPU box), W = 1 warm-up step,
    K = 2 timed closed-loop steps, then the fused mode's single all-gather.  The relayed
    line must say 8 GPUs and 32,768 scenarios, and rank 0's gathered rows must equal one
    single-rank bench run over all 32,768 scenarios bitwise (results do not
    depend on the GPU count)."""
    import subprocess
    import sys

    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    multi, single = os.path.join(out, "cfg4_rows_8rank.npy"), os.path.join(out, "cfg4_rows_1rank.npy")
    common = ["--steps", "2", "--warmup", "1", "--no-per-step", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(NMPC_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--batch", "4096", *common,
                        "--dump-rows", multi], cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    print(r.stdout[-2000:], r.stderr[-3000:])
    assert r.returncode == 0
    assert r.stdout.strip().splitlines()[-1].startswith("{")  # the relayed line is the last stdout line
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    import json
    res = json.loads(line)
    assert res["n_gpus"] == 8 and res["config"]["global_batch"] == 32768
    assert res["config"]["parallelism"] == "dp8" and res["steps"] == 2
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "32768", *common,
                         "--dump-rows", single], cwd=ROOT, capture_output=True, text=True, timeout=300)
    print(r1.stdout[-1000:], r1.stderr[-2000:])
    assert r1.returncode == 0
    a, b = np.load(multi), np.load(single)
    assert a.shape == b.shape == (32768, 8 * 2)
    np.testing.assert_array_equal(a, b)


def _rccl_rank(port, q):
    """World size 1 over RCCL (backend "nccl") on cuda:0, the process group created before
    any other GPU call of this process: gather_rows / gather_closed_loop take their
    all_gather_into_tensor branch; a gloo group of the same rank gives the reference."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "mpc-implementation_amd"))
    import torch
    import torch.distributed as dist
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.dist import gather_rows, gather_closed_loop, pack_result

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    gloo = dist.new_group(backend="gloo")
    assert dist.get_backend() == "nccl" and dist.get_backend(gloo) == "gloo"
    P = draw_scenarios(config_spec(3), TOTAL, seed=1003)
    hist = _closed_loop(P, K)
    torch.cuda.synchronize()
    out = {}
    for name, g in (("nccl", None), ("gloo", gloo)):
        rows = gather_closed_loop(hist, 1, group=g, total=TOTAL)
        res = gather_rows(pack_result(hist["u"][-1].contiguous(), hist["f"][-1], hist["status"][-1]), 1, group=g,
                          total=TOTAL)
        torch.cuda.synchronize()
        out[name] = (rows.cpu().numpy(), res.cpu().numpy(), rows.device.type)
    q.put(out)
    dist.destroy_process_group(gloo)
    dist.destroy_process_group()


def test_rccl_world_size_one_gather_equals_gloo():
    """The RCCL branch of nmpc_amd.dist (all_gather_into_tensor on device tensors, the
    path bench.py takes on a multi-GPU node) runs on this one-GPU box at world size 1 and
    gives bitwise the rows of the gloo branch (host-staged all_gather) and of the local
    packing."""
    import torch.multiprocessing as mp
    from nmpc_amd.dist import pack_closed_loop

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    proc.start()
    out = q.get(timeout=240)
    proc.join(timeout=60)
    assert proc.exitcode == 0
    (rn, sn, dev_n), (rg, sg, _) = out["nccl"], out["gloo"]
    assert dev_n == "cuda"
    assert rn.shape == (TOTAL, 8 * K) and sn.shape == (TOTAL, 8)
    np.testing.assert_array_equal(rn, rg)
    np.testing.assert_array_equal(sn, sg)
    np.testing.assert_array_equal(rn[:, 6 * K:7 * K][:, -1], sn[:, 6])  # f of the last step, both packings
