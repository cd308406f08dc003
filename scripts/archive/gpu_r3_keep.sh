#!/bin/bash
# Round 3: Infinity-Cache hand-off between the passes (GLX_AX_KEEP_MIB / GLX_ATR_KEEP_MIB): NS
# ProxGD bench lines, arms interleaved, two rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_keep; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for arm in "0 0" "192 0" "0 192" "192 192" "128 128" "96 224"; do
    set -- $arm
    GLX_AX_KEEP_MIB=$1 GLX_ATR_KEEP_MIB=$2 timeout -k 10 120 python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/k_${1}_${2}_r$r.json 2> $O/k_${1}_${2}_r$r.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/k_${1}_${2}_r$r.json')); r=d['roofline']
print('ax_keep $1 atr_keep $2 round $r: %.1f it/s  ax %.1f  atr %.1f  gather %.1f' % (d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], r['gather_avg_launch_us'] or 0))"
  done
done
echo done
