#!/bin/bash
# Round 3: C3 (FProxGD fp32, 8192 x 16384 x 32) fused A^T R + FISTA trial: load policy x prefetch
# depth x K splits (the session plan's default is NTL, PF 4, S = 2), 200-step windows, two rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_c3atr}; rm -rf $O; mkdir -p $O
B="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 --method gl_FProxGD_primal --dtype f32"
one() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 150 $B > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "
import json
d=json.loads([x for x in open('$O/$tag.json') if x.startswith('{\"')][-1]); r=d['roofline']
print('%-16s %8.1f it/s ax %6.1f atr %6.1f' % ('$tag', d['value'], r['avg_launch_us'], r['atr_avg_launch_us']))" | tee -a $O/status.txt
}
for r in 1 2; do
  one def_r$r GLX_NONE=1 || exit 1
  for v in 1004 1008 8 4; do for s in 1 2 4; do
    one v${v}_s${s}_r$r GLX_ATR_VARIANT=$v GLX_ATR_S=$s || exit 1
  done; done
done
echo done >> $O/status.txt
