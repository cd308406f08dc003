#!/bin/bash
# Round 3: software-pipelined A e gather; split-candidate / FISTA tests, then NS windows and
# whole solves, and the finalize workgroup size at NS (GLX_FIN_PER_BLOCK), two rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_gpipe}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_dist.py tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size or FProx or world3 or dc" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline"
one() {   # tag, env...
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
  one d_r$r GLX_NONE=1 timeout -k 10 200 $B --steps 20 --warmup 5 || exit 1
  one w_r$r GLX_NONE=1 timeout -k 10 200 $B --steps 200 --warmup 20 || exit 1
  for f in 512 1024; do
    one w_fin${f}_r$r GLX_FIN_PER_BLOCK=$f timeout -k 10 200 $B --steps 200 --warmup 20 || exit 1
  done
  one f_r$r GLX_NONE=1 timeout -k 10 200 python3 scripts/full_solve.py || exit 1
  one ff_r$r GLX_NONE=1 timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
cat $O/prof_gaps.txt >> $O/status.txt
echo done >> $O/status.txt
