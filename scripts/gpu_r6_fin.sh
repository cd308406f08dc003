#!/bin/bash
# Round 6: NS ProxGD's finalize width (GLX_FIN_PER_BLOCK work items per workgroup) in the
# driver's window, 3 interleaved rounds, kernel time from the bench's own events and it/s.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_fin}; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
  for v in "f256:GLX_FIN_PER_BLOCK=256" "f128:GLX_FIN_PER_BLOCK=128" "f512:GLX_FIN_PER_BLOCK=512"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name failed"; exit 1; }
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
