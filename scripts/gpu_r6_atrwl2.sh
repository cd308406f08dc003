#!/bin/bash
# Round 6: the 1024-row shard's A^T r on the eight-wave panel (WL 2, code 1028: two waves per
# SIMD, no K split) against the planner's WL 0 (code 8), 3 interleaved rounds of the model.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_atrwl2}; rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8"
for rep in 1 2 3; do
  for v in "wl0:GLX_ATR_KEEP_MIB=192" "wl2:GLX_ATR_VARIANT=1028"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name failed"; tail -5 $O/$name.$rep.err; exit 1; }
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
