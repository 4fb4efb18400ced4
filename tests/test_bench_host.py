"""bench.py's host-side legs on the CPU (no GPU): the CPU baseline times the GPU's own
window (the same W warm-up steps, then K timed steps) on the oracle description of the
bench's config -- config 5 with its moving obstacles (np = 17) -- and the roofline's PMC
summary is read from the profiles file whose rows match the run's kernel, batch, steps and
warm-up."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    argv, sys.argv = sys.argv, ["bench.py"]
    try:
        import bench as b
    finally:
        sys.argv = argv
    return b


@pytest.mark.parametrize("cfg", [3, 5])
def test_cpu_baseline_times_the_gpu_window(bench, cfg):
    from nmpc_amd import config_spec, draw_scenarios
    from nmpc_amd.targets import obstacle_steps
    spec = config_spec(cfg)
    W, K, B = 2, 2, 8
    ps = obstacle_steps(195, W + K, spec.np) if spec.np > spec.np_min else None
    r = bench.cpu_baseline(spec, cfg, draw_scenarios(spec, B, seed=1000 + cfg), *spec.bounds(), K, W, p_step=ps,
                           budget_s=30.0)
    P1, W1, sel = bench.cpu_baseline.start
    assert len(sel) == B and P1.shape == (B, spec.np) and W1.shape == (B, spec.nw)
    assert r["kind"] == "port" and r["value"] > 0 and f"steps {W}..{W + K - 1}" in r["sample"]
    assert len(bench.cpu_baseline.records) == B * K
    # the window starts after the warm-up: the first timed p is not the drawn one
    assert not np.allclose(P1[:, :8], draw_scenarios(spec, B, seed=1000 + cfg)[:, :8])


def test_pmc_summary_picks_the_matching_profile(bench):
    p3 = bench.pmc_summary("nmpc_closed_loop_sched_kernel", 20, 4096, 5)
    p5 = bench.pmc_summary("nmpc_closed_loop_sched_kernel", 20, 8192, 5)
    assert p3 and p5 and p3["source"] != p5["source"]
    assert "cfg5" in p5["source"] and "cfg5" not in p3["source"]
    assert bench.pmc_summary("nmpc_closed_loop_sched_kernel", 20, 1234, 5) is None


def test_gpus_n_launches_its_own_ranks(bench):
    """bench.py --gpus N without a launcher starts torch.distributed.run with N ranks of
    this same script and arguments (127.0.0.1 rendezvous); the ranks then see WORLD_SIZE."""
    cmd = bench.rank_launch_cmd(8, ["--gpus", "8", "--steps", "2"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "2"] and cmd[-5].endswith("bench.py")


def test_launch_ranks_relays_rank0_line(bench, monkeypatch, capsys):
    """The parent relays the ranks' JSON line as its last stdout line, forwards everything
    else to stderr, and passes the launcher's exit code on (non-zero without a line)."""
    prog = "print('rank log'); print('{\"value\": 1}')"
    monkeypatch.setattr(bench, "rank_launch_cmd", lambda n, argv, port: [sys.executable, "-c", prog])
    assert bench.launch_ranks(2, []) == 0
    out, err = capsys.readouterr()
    assert out.strip().splitlines()[-1] == '{"value": 1}' and "rank log" in err
    monkeypatch.setattr(bench, "rank_launch_cmd", lambda n, argv, port: [sys.executable, "-c", "print('x')"])
    assert bench.launch_ranks(2, []) != 0
    monkeypatch.setattr(bench, "rank_launch_cmd",
                        lambda n, argv, port: [sys.executable, "-c", "import sys; sys.exit(3)"])
    assert bench.launch_ranks(2, []) == 3


def test_gpus_must_match_launcher_world_size():
    """Under a launcher, --gpus must equal WORLD_SIZE (checked before any GPU call)."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "does not match" in r.stderr
