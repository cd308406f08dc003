#!/bin/bash
# Round 2: C5's per-rank shape (FProxGD fp64, 16384 x 16384 x 32 per rank) through the comm path
# on one GPU: split-candidate FISTA against the dense batch, and the A^T R policy.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_c5; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 100 --warmup 10 --method gl_FProxGD_primal --m 16384 --force-comm"
run() { name=$1; shift; env "$@" timeout -k 10 300 $D > $O/$name.json 2> $O/$name.err || exit 1; }
run split; run dense GLX_SPLIT_FISTA=0; run atr_old GLX_ATR_VARIANT=8
timeout -k 10 300 python3 bench.py --gpus 1 --no-cpu-baseline --steps 100 --warmup 10 --method gl_FProxGD_primal --m 16384 > $O/nocomm.json 2> $O/nocomm.err || exit 1
echo done
