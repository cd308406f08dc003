#!/bin/bash
# In-place A^T R ring: tests, ring-depth sweep, end to end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r22; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/kbench.py --ax 52228 --splits 0 --atr 102,103,104,106,108,114,1102,1104,1106,1108 --reps 20 > $O/kb_f64.jsonl 2>> $O/kb.err; echo "kb_f64 rc=$?" >> $O/status.txt
timeout -k 10 300 python scripts/kbench.py --dtype f32 --ax 21410 --splits 0 --atr 102,104,106,108,1102,1104,1106,1108,1114 --reps 20 > $O/kb_f32.jsonl 2>> $O/kb.err; echo "kb_f32 rc=$?" >> $O/status.txt
timeout -k 10 300 python scripts/kbench.py --ax 52228 --splits 1,2,4,8 --atr 104,106,1104 --reps 20 > $O/kb_f64s.jsonl 2>> $O/kb.err; echo "kb_f64s rc=$?" >> $O/status.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
$B > $O/b_pgd.json 2>> $O/bench.err; echo "b_pgd rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32.json 2>> $O/bench.err; echo "b_fpgd32 rc=$?" >> $O/status.txt
$B --method gl_SGD_primal --m 65536 --n 8192 --l 1 > $O/b_c4.json 2>> $O/bench.err; echo "b_c4 rc=$?" >> $O/status.txt
for f in $O/kb_*.jsonl; do echo == $f; python -c "
import json
for l in open('$f'):
    d=json.loads(l)
    if d['kernel'] in ('atr','torch_sum_A'): print(d['kernel'], d.get('variant',''), 'S=%s'%d.get('split',''), '%.1f us %.0f GB/s'%(d['us'], d['GBs']))"; done
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-14s %8.1f it/s ax %.1fus atr %.1fus %.0fGB/s' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], r['atr_GBs']))"; done
cat $O/status.txt | tr '\n' ' '
