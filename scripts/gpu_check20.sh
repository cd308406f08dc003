#!/bin/bash
# Branch-free, copy-free k_ax_lds ring: kernel tests, ablation, interleaved tiles end to end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r20; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
for abl in 0 2 3; do
  GLX_AXL_ABL=$abl timeout -k 10 200 python scripts/kbench.py --ax 52228 --splits 0 --atr 102 --axb 52224,52324 --reps 30 > $O/abl_$abl.jsonl 2>> $O/abl.err; rc=$?; echo "abl_$abl rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
done
timeout -k 10 300 python scripts/kbench.py --dtype f32 --ax 21410,52228 --splits 0 --atr 1102 --axb 52224,52324,52214 --reps 20 > $O/kb_f32.jsonl 2>> $O/abl.err; echo "kb_f32 rc=$?" >> $O/status.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
for rep in 1 2; do for v in 52224 52324 52228; do
  GLX_AXB_VARIANT=$v $B > $O/b_$v.$rep.json 2>> $O/bench.err; rc=$?; echo "b_$v.$rep rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
done; done
for v in 52224 52324; do GLX_AXB_VARIANT=$v $B --method gl_FProxGD_primal --dtype f32 > $O/b32_$v.json 2>> $O/bench.err; echo "b32_$v rc=$?" >> $O/status.txt; done
for abl in 0 2 3; do grep ax_batch2 $O/abl_$abl.jsonl | python -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('abl $abl', d['variant'], '%.1f us %.1f TF'%(d['us'], d['TFs']))"; done
grep -h "ax_batch2\|\"ax\"" $O/kb_f32.jsonl | python -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('f32', d['kernel'], d['variant'], '%.1f us'%d['us'], d.get('TFs',''))"
for f in $O/b_*.json $O/b32_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-20s %8.1f it/s  ax %.1fus %.1f TF' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['mfma_tflops']))"; done
cat $O/status.txt
