#!/bin/bash
# Speculative gradient: full GPU tests, then A/B (GLX_SPEC_GRAD=0) benches in one run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r18; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_comm.py tests/test_gpu_parity.py tests/test_gpu_cabi.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
for sp in 0 1; do
  GLX_SPEC_GRAD=$sp $B > $O/b_pgd_s$sp.json 2>> $O/bench.err; echo "b_pgd_s$sp rc=$?" >> $O/status.txt
  GLX_SPEC_GRAD=$sp $B --method gl_FProxGD_primal > $O/b_fpgd_s$sp.json 2>> $O/bench.err; echo "b_fpgd_s$sp rc=$?" >> $O/status.txt
  GLX_SPEC_GRAD=$sp $B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32_s$sp.json 2>> $O/bench.err; echo "b_fpgd32_s$sp rc=$?" >> $O/status.txt
  GLX_SPEC_GRAD=$sp $B --m 4096 --n 8192 --l 16 > $O/b_c2_s$sp.json 2>> $O/bench.err; echo "b_c2_s$sp rc=$?" >> $O/status.txt
done
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; w=d['work']; print('%-32s %8.1f it/s  ax %.1fus atr %.1fus atr/it %.2f' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], w['atr_per_iter']))"; done
cat $O/status.txt
