#!/bin/bash
# Round 6: NS ProxGD whole solves (the bench's whole_solve) with the bitmap gather's loads in flight
# U = 8 (default) and 16, and with A e fused into the dense pass (GLX_AE_FUSED=1); 3 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_gws}; rm -rf $O; mkdir -p $O
for rep in 1 2 3; do
  for v in "u8:GLX_GATHER_BM=8,256,1" "u16:GLX_GATHER_BM=16,256,1" "egat:GLX_AE_FUSED=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.$rep.json 2> $O/$name.$rep.err || exit 1
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
