#!/bin/bash
# DVFS probe (MFMA beside HBM streaming) + end-to-end bench with the LDS batched tiles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r13; mkdir -p $O
timeout -k 10 180 scripts/mfma_peak > $O/mfma_peak.jsonl 2> $O/mfma_peak.err; echo "mfma_peak rc=$?" >> $O/status.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
for v in 21420 54214 52324 52224; do GLX_AXB_VARIANT=$v $B > $O/b_pgd_$v.json 2>> $O/bench.err; echo "b_pgd_$v rc=$?" >> $O/status.txt; done
for v in 21410 52214 52324; do GLX_AXB_VARIANT=$v $B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32_$v.json 2>> $O/bench.err; echo "b_fpgd32_$v rc=$?" >> $O/status.txt; done
cat $O/mfma_peak.jsonl
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['value'],1), 'ax %.1fus %.1fTF frac %.3f pair %.3f atr %.1fus' % (r['avg_launch_us'], r['mfma_tflops'], r['frac'], r['pair_frac'], r['atr_avg_launch_us']))"; done
cat $O/status.txt
