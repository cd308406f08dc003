#!/bin/bash
# Round 2: where the split-candidate trial pays — default against GLX_SPLIT_CAND=0 at NS, C2 and
# the comm-path shards of the strong-scaling bench (m = 4096, 2048, 1024 rows per rank).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_splitgate; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D $EXTRA > $O/$name.json 2> $O/$name.err || exit 1; }
EXTRA=""; run ns_sc; run ns_dense GLX_SPLIT_CAND=0
EXTRA="--m 4096 --n 8192 --l 16"; run c2_sc; run c2_dense GLX_SPLIT_CAND=0
EXTRA="--m 4096 --force-comm"; run s4096_sc; run s4096_dense GLX_SPLIT_CAND=0
EXTRA="--m 2048 --force-comm"; run s2048_sc; run s2048_dense GLX_SPLIT_CAND=0
EXTRA="--m 1024 --force-comm"; run s1024_sc; run s1024_dense GLX_SPLIT_CAND=0
EXTRA="--m 4096"; run m4096_sc; run m4096_dense GLX_SPLIT_CAND=0
echo done
