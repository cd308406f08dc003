#!/bin/bash
# Round 6: FProxGD's dense [xc | y_next] batch (two right-hand sides, l = 32, NS) on the LDS-DMA
# tiles (GLX_AXB_VARIANT=92278 / 92268) against the planner's kind-5 tile (52228): NS FProxGD in the
# driver's form with the whole solve (where the dense batches dominate), 2 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_axb}; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for v in "k5:GLX_AXB_VARIANT=52228" "d78:GLX_AXB_VARIANT=92278" "d68:GLX_AXB_VARIANT=92268"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name failed"; tail -5 $O/$name.$rep.err; exit 1; }
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
