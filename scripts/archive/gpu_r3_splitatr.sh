#!/bin/bash
# Round 3: K-split fused A^T R + trial without the identity partials (grid_reduce nparts):
# the fused-trial tests (S = 2/4/8, host and device control), then C2 and NS at several S,
# interleaved rounds of 200-step windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_splitatr}; rm -rf $O; mkdir -p $O
GLX_ATR_SPLIT_MAJOR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
B="python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
one() {   # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "
import json
d=json.loads([x for x in open('$O/$tag.json') if x.startswith('{')][-1]); r=d['roofline']
print('%-22s %8.1f it/s ax %6.1f atr %6.1f syncs/it %.3f' % ('$tag', d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], d['work']['syncs_per_iter']))" | tee -a $O/status.txt
}
for r in 1 2; do
  for s in 2 4 8; do
    for o in 0 1; do
      one c2_s${s}_o${o}_r$r GLX_ATR_S=$s GLX_ATR_SPLIT_MAJOR=$o timeout -k 10 120 $B --m 4096 --n 8192 --l 16 || exit 1
    done
  done
  for o in 0 1; do
    one c2f_s8_o${o}_r$r GLX_ATR_S=8 GLX_ATR_SPLIT_MAJOR=$o timeout -k 10 120 $B --m 4096 --n 8192 --l 16 --method gl_FProxGD_primal || exit 1
    one ns_s2_o${o}_r$r GLX_ATR_S=2 GLX_ATR_SPLIT_MAJOR=$o timeout -k 10 120 $B || exit 1
  done
  one ns_s1_r$r timeout -k 10 120 $B || exit 1
done
echo done >> $O/status.txt
