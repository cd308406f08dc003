#!/bin/bash
# Grouped-slab finalize: kernel tests (forced splits 1..64), GPU suite, benches at m = 1024 and NS,
# kernel trace at m = 1024.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r36; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 30"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
run m1024_f64 $B --m 1024 || exit 1
run m1024_f32 $B --m 1024 --dtype f32 --method gl_FProxGD_primal || exit 1
run m2048_f64 $B --m 2048 || exit 1
run ns_f64 $B || exit 1
run ns_f64b $B || exit 1
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-18s %8.1f it/s  ax %.1fus atr %.1fus %s' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r.get('atr_avg_launch_us', -1), r['kernel']))"; done
for m in 1024 8192; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$m -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --m $m --profile 0 > $O/b$m.json 2> $O/tr$m.err; rc=$?; echo "trace rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
python scripts/trace_gaps.py $(find $O/tr$m -name "*kernel_trace.csv" | head -1) --last 1000 | head -6
done
cat $O/status.txt | tr '\n' ' '
