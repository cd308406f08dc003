"""Per-kernel summary (calls, average and total duration) of a rocprofv3 run_results.db (the
rocpd SQLite output of `rocprofv3 --kernel-trace`), sorted by total time."""
import sqlite3
import sys

for path in sys.argv[1:]:
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels "
                     "group by name order by sum(end-start) desc limit 16").fetchall()
    print("==", path)
    print("name,calls,avg_us,total_ms")
    for r in rows:
        print('"%s",%d,%.2f,%.2f' % (r[0][:110], r[1], r[2], r[3]))
