#!/bin/bash
# Round 6: the fused shard pass's K splits (GLX_AX_S; the planner's 32 = 256 dense workgroups)
# with its extra p_thr / A e workgroups, 1024-row model, 3 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_drvs}; rm -rf $O; mkdir -p $O
B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8"
for rep in 1 2 3; do
  for v in "s32:GLX_AX_S=32" "s24:GLX_AX_S=24" "s28:GLX_AX_S=28"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name failed"; tail -5 $O/$name.$rep.err; exit 1; }
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
