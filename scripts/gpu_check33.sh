#!/bin/bash
# main.py-parity driver on the GPU; A@X tile/split choice at the per-rank shard shapes of the
# 2/4/8-GPU scaling runs (m = 4096/2048/1024 rows of A per rank), single GPU, no comm.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r33; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_driver.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "driver tests rc=$rc" >> $O/status.txt
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 300 --warmup 30"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
for m in 1024 2048 4096; do
  run m${m}_default $B --m $m || exit 1
  for vb in 52228:128 52224:256 52224:512 52214:256 52214:512 54214:512 54214:1024; do
    v=${vb%:*}; blk=${vb#*:}
    run m${m}_${v}_b$blk env GLX_AXB_VARIANT=$v GLX_AXL_BLOCKS=$blk $B --m $m || exit 1
  done
done
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-22s %8.1f it/s  ax %.1fus atr %.1fus %s' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r.get('atr_avg_launch_us', -1), r['kernel']))"; done
cat $O/status.txt | tr '\n' ' '
