#!/bin/bash
# Round 4 batch 3: timing events without the system-scope fence against plain events, in the
# driver's command form, and the event/trace agreement of the new form under rocprofv3.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_evt; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for v in nofence fence; do
    f=""; [ $v = fence ] && f=1
    GLX_EVENT_FENCE=$f timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_$v.$r.json 2> $O/drv_$v.$r.err || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/driver_cmd_kernel_stats.csv \;
rm -rf $O/trace
python3 - $O <<'PY' | tee $O/summary.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/drv_*.json")) + [O + "/prof.json"]:
    d = json.loads([x for x in open(f) if x.startswith('{"')][-1])
    r = d["roofline"]
    print(os.path.basename(f), "%.1f it/s pair4 %.3f dom %s frac %.3f ax %.1f atr %.1f ga %s" % (d["value"], r["pair4_frac"], r["dominant"], r["frac"], r["kernels"]["ax"]["avg_launch_us"], r["kernels"]["atr"]["avg_launch_us"], r.get("gather_avg_launch_us")))
PY
cat $O/agree.json $O/prof_gaps.txt >> $O/summary.txt
