#!/bin/bash
# Round 5: the Infinity-Cache hand-off sizes re-checked at NS with the bitmap gather and the
# deferred reductions (200-step windows, two interleaved rounds).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_keep}; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for k in "192 192" "224 224" "160 160" "256 128" "128 256"; do
    set -- $k
    GLX_AX_KEEP_MIB=$1 GLX_ATR_KEEP_MIB=$2 timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/k$1_$2.$rep.json 2> $O/k$1_$2.$rep.err || exit 1
    echo -n "keep ax $1 atr $2 ($rep): " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/k$1_$2.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
