#!/bin/bash
# Round 5: the bitmap gather's loads in flight early in a solve (the driver's 20-step window,
# ~570 flagged rows): U = 8 (default) against 16, three interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_gu}; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
  for v in "8,256,1" "16,256,1" "16,128,1"; do
    GLX_GATHER_BM=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/$v.$rep.json 2> $O/$v.$rep.err || exit 1
    echo -n "bm=$v ($rep): " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$v.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
