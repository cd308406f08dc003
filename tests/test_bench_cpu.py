"""bench.py's launcher contract, on CPU (no GPU is touched).

`python bench.py --gpus N` without a launcher must start N ranks itself (torch.distributed.run
as a child process) and must refuse, with a non-zero exit, to measure fewer ranks than asked.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def test_launcher_spawns_n_ranks_dry_run():
    for n in (2, 4, 8):
        out = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "20", "--warmup", "5",
                              "--dry-run-launch"], capture_output=True, text=True, env=_env(), timeout=120)
        assert out.returncode == 0, out.stderr
        d = json.loads(out.stdout.strip().splitlines()[-1])
        cmd = d["launch"]
        assert cmd[1:3] == ["-m", "torch.distributed.run"]
        assert cmd[cmd.index("--nproc-per-node") + 1] == str(n)
        assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
        assert os.path.samefile(cmd[cmd.index("--master-port") + 2], BENCH)
        # the ranks get the same flags, so their world-size check sees --gpus N
        assert cmd[cmd.index("--gpus") + 1] == str(n) and "--dry-run-launch" not in cmd
        assert d["nproc"] == n


def test_launcher_refuses_without_enough_gpus():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "2"], capture_output=True,
                         text=True, env=_env(), timeout=120)
    assert out.returncode == 2
    assert "refusing" in out.stderr


def test_rank_world_mismatch_is_an_error():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--steps", "2"], capture_output=True,
                         text=True, env=env, timeout=120)
    assert out.returncode == 2
    assert "WORLD_SIZE=1" in out.stderr
