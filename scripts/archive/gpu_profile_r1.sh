#!/bin/bash
# Round-1 evidence: rocprofv3 kernel stats of the default bench command (same steps/warmup as
# the bench line), its agreement with the live HIP-event timing, and per-launch HBM traffic
# from separate FETCH_SIZE / WRITE_SIZE PMC passes (gfx950 correction in scripts/pmc_traffic.py)
# for the north-star, C3, C2 and C4 configurations.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p1; rm -rf $O; mkdir -p $O
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- $B > $O/bench_stats.json 2> $O/stats.err; rc=$?; echo "stats rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
python scripts/prof_agree.py --trace $O/stats --bench $O/bench_stats.json --out $O/agree.json > $O/agree.log 2>&1; echo "agree rc=$?" >> $O/status.txt
run_pmc() {   # name key args...
  local name=$1 key=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$name -o run -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $O/b_fetch_$name.json 2> $O/fetch_$name.err; local rc=$?; echo "fetch_$name rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || return 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write_$name -o run -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $O/b_write_$name.json 2> $O/write_$name.err; rc=$?; echo "write_$name rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || return 1
  python scripts/pmc_traffic.py --fetch $O/fetch_$name --write $O/write_$name --key $key --out $O/pmc_traffic.json >> $O/pmc.log 2>&1
}
run_pmc ns gl_ProxGD_primal_f64_8192x16384x32_g1 || exit 1
run_pmc c3 gl_FProxGD_primal_f32_8192x16384x32_g1 --method gl_FProxGD_primal --dtype f32 || exit 1
run_pmc c2 gl_ProxGD_primal_f64_4096x8192x16_g1 --m 4096 --n 8192 --l 16 || exit 1
run_pmc c4 gl_SGD_primal_f64_65536x8192x1_g1 --method gl_SGD_primal --m 65536 --n 8192 --l 1 || exit 1
cat $O/agree.log; cat $O/status.txt | tr "\n" " "
cat $O/status.txt
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > $O/bench_default.json 2> $O/bench_default.err; echo "bench_default rc=$?" >> $O/status.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
$B --exact 1 > $O/b_pgd_exact.json 2>> $O/bench.err; echo "b_pgd_exact rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal > $O/b_fpgd.json 2>> $O/bench.err; echo "b_fpgd rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32.json 2>> $O/bench.err; echo "b_fpgd32 rc=$?" >> $O/status.txt
$B --m 4096 --n 8192 --l 16 > $O/b_c2.json 2>> $O/bench.err; echo "b_c2 rc=$?" >> $O/status.txt
$B --method gl_SGD_primal --m 65536 --n 8192 --l 1 > $O/b_c4.json 2>> $O/bench.err; echo "b_c4 rc=$?" >> $O/status.txt
$B --method gl_FProxGD_primal --m 16384 > $O/b_c5shard.json 2>> $O/bench.err; echo "b_c5shard rc=$?" >> $O/status.txt
for f in $O/bench_default.json $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-18s %8.1f it/s  %s %.1f %s frac %.3f pair %.3f  ax %.1fus atr %.1fus' % ('$f'.split('/')[-1], d['value'], r['bound'], r['achieved'], r['unit'], r['frac'], r['pair_frac'] or 0, r['avg_launch_us'], r['atr_avg_launch_us']), d.get('cpu_baseline', {}).get('value'))"; done
