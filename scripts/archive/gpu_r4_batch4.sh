#!/bin/bash
# Round 4 batch 4: the driver's command with the timed session created before the pre-warm (no
# idle gap before the window) against the previous bench flow on the same library, interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_flow; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/new.$r.json 2> $O/new.$r.err || exit 1
  ( cd abtree/oldbench && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > ../../$O/old.$r.json 2> ../../$O/old.$r.err ) || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 2 --comm host --steps 10 --warmup 3 > $O/host2.json 2> $O/host2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/driver_cmd_kernel_stats.csv \;
rm -rf $O/trace
python3 - $O <<'PY' | tee $O/summary.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*.json")):
    t = [x for x in open(f) if x.startswith('{"')]
    if not t or "roofline" not in t[-1]: continue
    d = json.loads(t[-1]); r = d["roofline"]
    k = r.get("kernels", {})
    print(os.path.basename(f), "%.1f it/s pair4 %.3f frac %.3f ax %.1f atr %.1f ga %s" % (d["value"], r["pair4_frac"], r["frac"], r["avg_launch_us"], r["atr_avg_launch_us"], r.get("gather_avg_launch_us")))
PY
cat $O/agree.json $O/prof_gaps.txt >> $O/summary.txt
