"""CPU multi-process test of the N>1 path (gloo, world size 2): scenario
sharding of the global stream + the per-step result gather reproduce the
single-process result exactly.  The per-rank solve here is the CPU oracle
(test infrastructure) because this container has no GPU; on the GPU box the
same helpers carry the HIP results over RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _solve_rows(P, spec):
    from oracle import nmpc_oracle as orc

    prob = orc.make_problem("race_track_2", N=spec.N, T=spec.T)
    lbx, ubx, lbg, ubg = orc.bounds(prob)
    sol = orc.IpoptDense(prob, orc.REFERENCE_OPTS)
    rows = []
    for p in P:
        r = sol.solve(np.zeros(prob.nw), lbx, ubx, lbg, ubg, p)
        rows.append(np.concatenate([r["x"][:6], [r["f"], r["status"]]]))
    return np.array(rows)


def _worker_uneven(rank, world, port, total, q):
    """Rows tagged with their global scenario index, sharded unevenly (total % world != 0)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "mpc-implementation_amd"))
    from nmpc_amd.dist import shard, gather_rows, gather_closed_loop

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sl = shard(total, world, rank)
    idx = torch.arange(sl.start, sl.stop, dtype=torch.float64)
    local = torch.stack([idx, idx * 10 + 1, -idx], dim=1)
    allr = gather_rows(local, world, total=total)
    # the fused closed loop's packed histories (K steps of u0, f, status) over the same shards
    K, B = 3, sl.stop - sl.start
    hist = {"u": idx[None, :, None].repeat(K, 1, 6) + torch.arange(K, dtype=torch.float64)[:, None, None],
            "f": idx[None, :].repeat(K, 1) * 2, "status": torch.zeros(K, B, dtype=torch.int32)}
    cl = gather_closed_loop(hist, world, total=total)
    try:
        # a block that is not this rank's shard is refused (on every rank, before any collective)
        gather_rows(torch.cat([local, torch.zeros(1, 3, dtype=local.dtype)]), world, total=total)
        bad = False
    except ValueError:
        bad = True
    if rank == 0:
        q.put((allr.numpy(), cl.numpy(), bad))
    dist.barrier()
    dist.destroy_process_group()


def _worker(rank, world, port, total, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "mpc-implementation_amd"))
    from nmpc_amd import make_spec, draw_scenarios
    from nmpc_amd.dist import shard, gather_rows

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec = make_spec("race_track_2", N=5, T=0.2)
    P_all = draw_scenarios(spec, total, seed=99)
    sl = shard(total, world, rank)
    local = torch.tensor(_solve_rows(P_all[sl], spec))
    allr = gather_rows(local, world)
    if rank == 0:
        q.put(allr.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partitions_range():
    from nmpc_amd.dist import shard

    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                s = shard(total, world, r)
                covered += list(range(s.start, s.stop))
            assert covered == list(range(total))


@pytest.mark.timeout(300)
def test_gloo_world2_gather_matches_serial():
    from nmpc_amd import make_spec, draw_scenarios

    total, world = 4, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    spec = make_spec("race_track_2", N=5, T=0.2)
    want = _solve_rows(draw_scenarios(spec, total, seed=99), spec)
    np.testing.assert_array_equal(got, want)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("total,world", [(10, 3), (7, 3), (2, 3)])
def test_gloo_world3_uneven_shards_gather(total, world):
    """total % world != 0: shard() gives unequal blocks; the gather pads to the largest
    block and returns exactly the global rows in order (bench.py's fused-mode exchange)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_uneven, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    allr, cl, bad = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    idx = np.arange(total, dtype=np.float64)
    np.testing.assert_array_equal(allr, np.stack([idx, idx * 10 + 1, -idx], axis=1))
    assert cl.shape == (total, 8 * 3)
    np.testing.assert_array_equal(cl[:, 0], idx)            # step 0's u0[0] = scenario index
    np.testing.assert_array_equal(cl[:, 6 * 3], idx * 2)    # step 0's f
    assert bad
