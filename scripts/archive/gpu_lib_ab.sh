#!/bin/bash
# Same-box A/B of two builds of libglx: gpuab/libglx_old.so vs the tree's glx/libglx.so.
#   bash scripts/gpu_lib_ab.sh TAG "bench args (;-separated configs)"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; CONFIGS=$2
O=gpurun_out/$TAG; rm -rf $O; mkdir -p $O
L=convex-optimization_amd/glx/libglx.so
cp $L gpuab/libglx_new.so
IFS=';' read -ra CFG <<< "$CONFIGS"
for rep in 1 2; do for ci in "${!CFG[@]}"; do for v in old new; do
  cp gpuab/libglx_$v.so $L
  f=$O/c${ci}_${v}.$rep
  timeout -k 10 200 python bench.py --no-cpu-baseline ${CFG[$ci]} > $f.out 2> $f.err || { echo "bench [${CFG[$ci]}] $v failed"; tail -5 $f.err; cp gpuab/libglx_new.so $L; exit 1; }
  python -c "
import json; d=json.loads(open('$f.out').read().strip().splitlines()[-1]); r=d['roofline']
print('[${CFG[$ci]}] $v rep $rep: %.1f it/s  ax %.1fus atr %.1fus' % (d['value'], r['avg_launch_us'], r['atr_avg_launch_us']))" | tee -a $O/summary.txt
done; done; done
cp gpuab/libglx_new.so $L
