#!/bin/bash
# Round 3: NS knob sweep at HEAD (200-step windows, two interleaved rounds): A@X K splits, the
# Infinity-Cache hand-off sizes, XCD grouping / rotation of the DMA tile's K walk.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_nssweep}; rm -rf $O; mkdir -p $O
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-whole-solve --steps 200 --warmup 20"
one() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 150 $B > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "
import json
d=json.loads([x for x in open('$O/$tag.json') if x.startswith('{\"')][-1]); r=d['roofline']
print('%-16s %8.1f it/s ax %6.1f atr %6.1f ga %s' % ('$tag', d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], r.get('gather_avg_launch_us')))" | tee -a $O/status.txt
}
for r in 1 2; do
  one def_r$r GLX_NONE=1 || exit 1
  one axs4_r$r GLX_AX_S=4 || exit 1
  one axs16_r$r GLX_AX_S=16 || exit 1
  one keep128_r$r GLX_AX_KEEP_MIB=128 GLX_ATR_KEEP_MIB=128 || exit 1
  one keep256_r$r GLX_AX_KEEP_MIB=256 GLX_ATR_KEEP_MIB=256 || exit 1
  one axkeep0_r$r GLX_AX_KEEP_MIB=0 || exit 1
  one xcd0_r$r GLX_AX_XCD=0 || exit 1
  one rot0_r$r GLX_AX_ROT=0 || exit 1
done
echo done >> $O/status.txt
