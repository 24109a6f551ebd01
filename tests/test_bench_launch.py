"""bench.py's launcher plumbing (no GPU): `bench.py --gpus N` outside a launcher relaunches itself under
torch.distributed.run with N ranks (a child process, not an exec), a rank refuses a world size that differs from
--gpus, and the ranks the driver's command starts really form an N-rank group (gloo, --launch-check)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_relaunch_command():
    import bench
    assert bench.relaunch_command(None, [], {}) is None
    assert bench.relaunch_command(1, ["--gpus", "1"], {}) is None
    assert bench.relaunch_command(4, ["--gpus", "4"], {"WORLD_SIZE": "4"}) is None   # already a rank
    cmd = bench.relaunch_command(8, ["--gpus", "8", "--steps", "5"], {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert os.path.basename(cmd[-5]) == "bench.py"
    # `--n` is a prefix of torch.distributed.run's --nnodes / --nproc-per-node: passed on as --gaussians
    cmd = bench.relaunch_command(2, ["--gpus", "2", "--n", "5000", "--n=6000"], {})
    assert cmd[-4:] == ["2", "--gaussians", "5000", "--gaussians=6000"]


def test_world_mismatch_refused():
    import bench
    bench.check_world(None, 3)
    bench.check_world(2, 2)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1)


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_starts_n_ranks(n):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line == {"n_gpus": n, "rank_sum": n * (n - 1) // 2, "gpus_arg": n}


def test_driver_command_world_checked():
    """The driver's own form (torch.distributed.run ... bench.py --gpus N) with a mismatched N fails loudly."""
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", "0", os.path.join(ROOT, "bench.py"),
                        "--gpus", "3", "--launch-check"], capture_output=True, text=True, env=env, timeout=240,
                       cwd=ROOT)
    assert r.returncode != 0
    assert "--gpus 3" in r.stderr
