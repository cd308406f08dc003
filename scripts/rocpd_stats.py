"""Per-kernel statistics from a rocprofv3 rocpd database (the default output format when
--output-format csv is not given): name, calls, total and average duration, share of GPU time.
Optionally restricted to the last N dispatches of each kernel (the timed window)."""
import sqlite3
import sys


def stats(path, top=25):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{path}: {len(rows)} kernels, {tot / 1e6:.1f} ms")
    for n, cnt, s, a in rows[:top]:
        print(f"  {s / tot * 100:5.1f}%  {cnt:7d}  avg {a / 1e3:8.2f} us  {n[:110]}")


for p in sys.argv[1:]:
    stats(p)
