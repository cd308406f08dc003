"""glx.watchdog (round 6) on the CPU: two gloo ranks, one of which never
joins the second all-reduce. The other rank blocks inside the collective; at its deadline its
watchdog prints the diagnostic (rank, phase, the registered progress record, every thread's
stack) and the process leaves with exit code 3, so the launcher fails fast instead of hanging
until an outer time limit. The same module is armed by bench.py for N > 1 runs (RCCL or host
transport), with libglx's glx_session_progress / glx_comm_progress as its probes."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_stalled_rank_fails_fast_with_diagnostic():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "watchdog_worker.py"), "--deadline", "5"]
    t0 = time.monotonic()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    elapsed = time.monotonic() - t0
    err = p.stderr
    assert p.returncode != 0
    assert elapsed < 60, elapsed
    # the blocked rank's diagnostic: who, what, the progress record, and the stack in the collective
    assert "glx watchdog: rank 0 of 2: watchdog_worker passed its deadline of 5 s" in err, err[-3000:]
    assert "phase all-reduce loop" in err
    assert "progress: {'collectives': 1}" in err
    assert "all_reduce" in err   # faulthandler's stack shows where rank 0 is blocked
    assert "exitcode  : 3" in err or "exit code: 3" in err or "exitcode: 3" in err, err[-2000:]
