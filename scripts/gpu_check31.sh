#!/bin/bash
# Fused ProxGD trial in A^T r: all GPU tests, then A/B end to end, kernel stats.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r31; mkdir -p $O
timeout -k 10 900 python -m pytest tests/test_gpu_fused.py tests/test_gpu_kernels.py tests/test_gpu_comm.py tests/test_gpu_parity.py tests/test_gpu_cabi.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
run() { local tag=$1; shift; "$@" > $O/$tag.json 2>> $O/bench.err; local rc=$?; echo "$tag rc=$rc" >> $O/status.txt; return $rc; }
for rep in 1 2; do
run pgd.$rep $B || exit 1
run nofuse.$rep env GLX_FUSED_TRIAL=0 $B || exit 1
run fpgd.$rep $B --method gl_FProxGD_primal || exit 1
run fpgd_nofuse.$rep env GLX_FUSED_TRIAL=0 $B --method gl_FProxGD_primal || exit 1
run f32.$rep $B --method gl_FProxGD_primal --dtype f32 || exit 1
run f32_nofuse.$rep env GLX_FUSED_TRIAL=0 $B --method gl_FProxGD_primal --dtype f32 || exit 1
done
run exact $B --exact 1 || exit 1
run c5shard $B --method gl_FProxGD_primal --m 16384 || exit 1
run c2 $B --m 4096 --n 8192 --l 16 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err; echo "prof rc=$?" >> $O/status.txt
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; w=d['work']; print('%-18s %8.1f it/s ax %.1fus atr(+trial) %.1fus atr/it %.2f' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], w['atr_per_iter']))"; done
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r31/prof/bench_kernel_stats.csv')))
for r in rows[:9]: print(r['Name'][:60], r['Calls'], '%.1f'%(float(r['AverageNs'])/1e3))
PY
cat $O/status.txt | tr '\n' ' '
