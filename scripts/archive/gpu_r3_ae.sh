#!/bin/bash
# Round 3: A e fused into the LDS-DMA dense pass (split-candidate mode 2). Its tests, the
# split-candidate / FISTA / device-control suites, then NS driver form, 200-step windows and
# whole solves, mode 2 against mode 1 (GLX_SPLIT_AE=0), two interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_ae}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ae.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ae.log 2>&1; rc=$?
echo "ae tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_ae.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_dc_dist.py tests/test_gpu_dist.py tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size or FProx or world3 or dc" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline"
one() {   # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "
import json
d=json.loads([x for x in open('$O/$tag.json') if x.startswith('{\"')][-1])
if 'roofline' in d:
    r=d['roofline']
    print('%-14s %8.1f it/s ax %6.1f atr %6.1f ga %s' % ('$tag', d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], r.get('gather_avg_launch_us')))
else:
    print('%-14s k %d %.1f it/s fval %.10g' % ('$tag', d['k'], d['its'], d['fval']))" | tee -a $O/status.txt
}
for r in 1 2; do
  for a in 1 0; do
    one d_ae${a}_r$r GLX_SPLIT_AE=$a timeout -k 10 200 $B --steps 20 --warmup 5 || exit 1
    one w_ae${a}_r$r GLX_SPLIT_AE=$a timeout -k 10 200 $B --steps 200 --warmup 20 || exit 1
    one f_ae${a}_r$r GLX_SPLIT_AE=$a timeout -k 10 200 python3 scripts/full_solve.py || exit 1
    one ff_ae${a}_r$r GLX_SPLIT_AE=$a timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal || exit 1
  done
done
echo done >> $O/status.txt
