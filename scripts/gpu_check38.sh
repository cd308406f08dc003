#!/bin/bash
# Sampled event timing (--profile 16 default) vs none, NS and m = 1024; profile test.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r38; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_profile.py tests/test_gpu_kernels.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 30"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
for rep in 1 2; do
run m1024_p16.$rep $B --m 1024 || exit 1
run m1024_p0.$rep $B --m 1024 --profile 0 || exit 1
run ns_p16.$rep $B || exit 1
run ns_p0.$rep $B --profile 0 || exit 1
done
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-18s %8.1f it/s  ax %.1fus (%s timed) atr %.1fus' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r.get('launches_timed'), r.get('atr_avg_launch_us', -1)))"; done
cat $O/status.txt | tr '\n' ' '
