#!/bin/bash
# Round 2: one-RHS A@X tile A/B inside the solver (200-step bench, same box).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_axtile; rm -rf $O; mkdir -p $O
B="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
for i in 1 2; do
  timeout -k 10 200 $B > $O/def_$i.json 2> $O/def_$i.err || exit 1
  GLX_AX_VARIANT=51328 timeout -k 10 200 $B > $O/v51328_$i.json 2> $O/v51328_$i.err || exit 1
  GLX_AX_VARIANT=52324 GLX_AX_S=4 timeout -k 10 200 $B > $O/v52324s4_$i.json 2> $O/v52324s4_$i.err || exit 1
  GLX_AX_VARIANT=52328 timeout -k 10 200 $B > $O/v52328_$i.json 2> $O/v52328_$i.err || exit 1
done
echo done
