#!/bin/bash
# Round 3 final evidence: the whole GPU suite (world-8 in its own step), smoke, the driver's
# command twice (with the CPU baseline and the whole-solve figure), its rocprofv3 kernel trace
# + stats (event/trace agreement, gaps), a host-staged 2-rank rehearsal of the N > 1 bench path,
# and C1 (512,1024,2) with and without device control.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_final}; rm -rf $O; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 250 --timeout-method thread -k "world8" > $O/world8.log 2>&1 || exit 1
tail -2 $O/world8.log >> $O/status.txt
fi
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_r$r.json 2> $O/driver_r$r.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/driver_cmd_kernel_stats.csv \;
timeout -k 10 300 python3 bench.py --gpus 2 --comm host --steps 10 --warmup 3 > $O/host2.json 2> $O/host2.err || exit 1
for w in -1 8; do
  GLX_DC_BATCH=$w timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 20 --m 512 --n 1024 --l 2 --no-cpu-baseline > $O/c1_dc$w.json 2> $O/c1_dc$w.err || exit 1
done
python3 - $O <<'PY' | tee -a $O/status.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*.json")):
    t = [x for x in open(f) if x.startswith('{"')]
    if not t: continue
    d = json.loads(t[-1])
    if "roofline" in d:
        r = d["roofline"]
        print(os.path.basename(f), "n_gpus %d %.1f it/s ax %.1f atr %.1f ga %s pair4 %.3f frac %.3f traffic %s n %d cpu %s whole %s" % (d["n_gpus"], d["value"], r["avg_launch_us"], r["atr_avg_launch_us"], r.get("gather_avg_launch_us"), r["pair4_frac"] or 0, r["frac"], r.get("traffic"), r["launches_timed"], (d.get("cpu_baseline") or {}).get("value"), d.get("whole_solve") and "%d it %.1f it/s" % (d["whole_solve"]["k"], d["whole_solve"]["iters_per_s"])))
PY
cat $O/agree.json $O/prof_gaps.txt >> $O/status.txt
echo done >> $O/status.txt
