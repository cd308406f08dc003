#!/bin/bash
# Round 3 (closing): BASELINE.md §3 re-measured at HEAD without the PMC passes — every BASELINE config in driver form (20 timed / 5 warmup, with the
# CPU baseline), a 200-step window, and a whole solve to the solver's own stop rule; then the
# PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes) of the dominant kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_table3}; rm -rf $O; mkdir -p $O
run() {   # tag, bench args
  local tag=$1; shift
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $O/${tag}_d.json 2> $O/${tag}_d.err || return 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline "$@" > $O/${tag}_w.json 2> $O/${tag}_w.err || return 1
  python3 -c "
import json,sys
for s in ('d','w'):
    l=[x for x in open('$O/${tag}_'+s+'.json') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
    cb=d.get('cpu_baseline',{}) or {}
    print('$tag', s, '%.1f it/s' % d['value'], 'ax %.1f atr %.1f ga %s' % (r['avg_launch_us'], r['atr_avg_launch_us'], r.get('gather_avg_launch_us')),
          'pair4 %.3f frac %.3f' % (r['pair4_frac'] or 0, r['frac'] or 0), 'syncs/it %.3f' % d['work']['syncs_per_iter'], 'cpu %s' % cb.get('value'))
" | tee -a $O/status.txt
}
solve() {   # tag, full_solve args
  local tag=$1; shift
  timeout -k 10 200 python3 scripts/full_solve.py "$@" > $O/${tag}_full.json 2> $O/${tag}_full.err || return 1
  python3 -c "
import json; d=json.loads(open('$O/${tag}_full.json').read().strip().splitlines()[-1])
print('$tag full solve: k %d  %.1f it/s  fval %.10g' % (d['k'], d['its'], d['fval']))" | tee -a $O/status.txt
}
run ns   || exit 1
solve ns || exit 1
run nsf --method gl_FProxGD_primal || exit 1
solve nsf --method gl_FProxGD_primal || exit 1
run c2 --m 4096 --n 8192 --l 16 || exit 1
solve c2 --m 4096 --n 8192 --l 16 || exit 1
run c3 --method gl_FProxGD_primal --dtype f32 || exit 1
solve c3 --method gl_FProxGD_primal --dtype f32 || exit 1
run c4 --method gl_SGD_primal --m 65536 --n 8192 --l 1 || exit 1
solve c4 --method gl_SGD_primal --m 65536 --n 8192 --l 1 || exit 1
run c1 --m 512 --n 1024 --l 2 || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline --m 16384 --method gl_FProxGD_primal --force-comm > $O/c5shard_w.json 2> $O/c5shard_w.err || exit 1
echo "bench ok" >> $O/status.txt
echo done >> $O/status.txt
