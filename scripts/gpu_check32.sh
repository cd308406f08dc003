#!/bin/bash
# MT4 8-wave LDS tiles (more MFMAs per LDS X read) vs the defaults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r32; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "batch" > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
for rep in 1 2; do
  for v in 52228 54228 54218; do run pgd_$v.$rep env GLX_AXB_VARIANT=$v $B || exit 1; done
  for v in 52324 54228 54218; do run f32_$v.$rep env GLX_AXB_VARIANT=$v $B --method gl_FProxGD_primal --dtype f32 || exit 1; done
done
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-18s %8.1f it/s  ax %.1fus %.1f TF  %s' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['mfma_tflops'], r['kernel']))"; done
cat $O/status.txt | tr '\n' ' '
