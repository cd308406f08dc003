set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r17; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_comm.py -m gpu -q --maxfail=5 > $O/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> $O/status.txt
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=20 > $O/pytest_parity.log 2>&1 ; echo "parity rc=$?" >> $O/status.txt
tail -3 $O/pytest_kernels.log; tail -3 $O/pytest_parity.log
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
$B > $O/b_pgd.json 2> $O/bench.err ; echo "b_pgd rc=$?" >> $O/status.txt
$B --exact 1 > $O/b_pgd_exact.json 2>> $O/bench.err ; echo "b_pgd_exact rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal > $O/b_fpgd.json 2>> $O/bench.err ; echo "b_fpgd rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32.json 2>> $O/bench.err ; echo "b_fpgd32 rc=$?" >> $O/status.txt
$B --m 4096 --n 8192 --l 16 > $O/b_c2.json 2>> $O/bench.err ; echo "b_c2 rc=$?" >> $O/status.txt
$B --method gl_SGD_primal --m 65536 --n 8192 --l 1 > $O/b_c4.json 2>> $O/bench.err ; echo "b_c4 rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal --m 16384 > $O/b_c5shard.json 2>> $O/bench.err ; echo "b_c5shard rc=$?" >> $O/status.txt
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2>> $O/bench.err ; echo "bench_default rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err ; echo "prof rc=$?" >> $O/status.txt
for f in $O/b_*.json $O/bench_default.json; do echo $f; python -c "
import json,sys; d=json.load(open('$f')); r=d['roofline']; w=d['work']
print(' it/s=%.1f ms=%.3f ax=%.0fus(%.1f%s,rhs=%.1f,frac=%.2f,pair=%.2f) atr=%.0fus(%.0fGB/s) passes=%.2f' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['achieved'], r['unit'], r['rhs_per_launch'], r['frac'], r['pair_frac'] or 0, r['atr_avg_launch_us'], r['atr_GBs'], w['passes_over_A_per_iter']), d.get('cpu_baseline'))"; done
cat $O/status.txt
