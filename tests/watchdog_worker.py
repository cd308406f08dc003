"""One rank of tests/test_watchdog_cpu.py (gloo, CPU only): every rank arms glx.watchdog, then
joins a sum all-reduce that one rank never enters (it sleeps in place of the call), so every rank
but that one blocks inside the collective until the watchdog's deadline passes."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "convex-optimization_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--deadline", type=float, default=5.0)
    ap.add_argument("--stall-rank", type=int, default=1)
    a = ap.parse_args()
    from glx.watchdog import Watchdog
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    done = {"collectives": 0}
    # the stalled rank's deadline is later: the blocked rank's diagnostic is the one under test
    dl = a.deadline * (3 if rank == a.stall_rank else 1)
    wd = Watchdog(dl, "watchdog_worker", rank=rank, world=world).start()
    wd.probe("progress", lambda: dict(done))
    wd.phase = "all-reduce loop"
    t = torch.ones(4)
    for _ in range(3):
        if rank == a.stall_rank and done["collectives"] == 1:
            time.sleep(600)   # this rank never joins the second all-reduce
        dist.all_reduce(t)
        done["collectives"] += 1
    wd.stop()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
