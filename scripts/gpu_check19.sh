#!/bin/bash
# A@X ablation (what limits k_ax_lds) + interleaved end-to-end tile comparison.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r19; mkdir -p $O
for abl in 0 1 2 3 4 0; do
  GLX_AXL_ABL=$abl timeout -k 10 200 python scripts/kbench.py --ax 52228 --splits 0 --atr 102 --axb 52224 --reps 30 > $O/abl_$abl.jsonl 2>> $O/abl.err; rc=$?; echo "abl_$abl rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
done
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
for rep in 1 2; do for v in 52224 52228 52324 52214 54214; do
  GLX_AXB_VARIANT=$v $B > $O/b_$v.$rep.json 2>> $O/bench.err; rc=$?; echo "b_$v.$rep rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
done; done
for abl in 0 1 2 3 4; do echo "abl $abl: $(grep ax_batch2 $O/abl_$abl.jsonl)"; done
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-20s %8.1f it/s  ax %.1fus' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us']))"; done
cat $O/status.txt
