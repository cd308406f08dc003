#!/bin/bash
# Full GPU suite after the shard-shape planner change; m = 1024 shard iteration profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r34; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 30"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
run m1024_f64 $B --m 1024 || exit 1
run m1024_f32 $B --m 1024 --dtype f32 --method gl_FProxGD_primal || exit 1
run m1024_f32_old env GLX_AXB_VARIANT=52324 $B --m 1024 --dtype f32 --method gl_FProxGD_primal || exit 1
run m1024_fista $B --m 1024 --method gl_FProxGD_primal || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --m 1024 --profile 0 > $O/prof.log 2>&1; echo "prof rc=$?" >> $O/status.txt
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-18s %8.1f it/s  ax %.1fus atr %.1fus %s' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r.get('atr_avg_launch_us', -1), r['kernel']))"; done
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv; rows=list(csv.DictReader(open('{}')))
for r in rows[:12]: print('%-60s %8s %10.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
cat $O/status.txt | tr '\n' ' '
