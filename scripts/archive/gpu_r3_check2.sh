#!/bin/bash
# Round 3 closing check: the whole GPU suite (the world-8 test in its own step), smoke, the
# driver's command twice, its kernel trace (event/trace agreement, gaps of the timed region).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_check2}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 250 --timeout-method thread -k "world8" > $O/world8.log 2>&1 || exit 1
tail -2 $O/world8.log >> $O/status.txt
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_r$r.json 2> $O/driver_r$r.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/driver_cmd_kernel_stats.csv \;
python3 - $O <<'PY' | tee -a $O/status.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*.json")):
    t = [x for x in open(f) if x.startswith('{"')]
    if not t: continue
    d = json.loads(t[-1])
    if "roofline" in d:
        r = d["roofline"]
        print(os.path.basename(f), "%.1f it/s ax %.1f atr %.1f ga %s pair4 %.3f frac %.3f n %d cpu %s" % (d["value"], r["avg_launch_us"], r["atr_avg_launch_us"], r.get("gather_avg_launch_us"), r["pair4_frac"] or 0, r["frac"], r["launches_timed"], (d.get("cpu_baseline") or {}).get("value")))
PY
cat $O/agree.json $O/prof_gaps.txt >> $O/status.txt
echo done >> $O/status.txt
