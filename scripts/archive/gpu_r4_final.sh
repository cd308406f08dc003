#!/bin/bash
# Round 4 closing evidence at HEAD: the GPU suite, smoke(), the driver's bench command twice, and
# the same command under a rocprofv3 kernel trace (stats) for the bench/trace agreement.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_final; rm -rf $O; mkdir -p $O
bash scripts/gpu_verify.sh r4_final/verify "--gpus 1 --steps 20 --warmup 5" "--gpus 1 --steps 20 --warmup 5" > $O/verify.txt 2>&1 || { tail -30 $O/verify.txt; exit 1; }
tail -4 $O/verify.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || { tail -20 $O/drv.err; exit 1; }
python3 - $O/drv/run_kernel_stats.csv $O/drv.json <<'PY'
import csv, json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1]); r = d["roofline"]
print("bench under rocprof: %.1f it/s, events: ax %.1f atr %.1f us" % (d["value"], r["avg_launch_us"], r["atr_avg_launch_us"]))
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:6]:
    print("%-60s calls %5s avg %7.1f us" % (row["Name"][:60], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
