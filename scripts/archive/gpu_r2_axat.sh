#!/bin/bash
# Round 2: (1) A@X through the A^T R panel kernel on At, at several row splits; (2) the
# non-temporal A^T R default against the old default-policy code (GLX_ATR_VARIANT=8) at NS, C2
# and the 1024-row shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_axat; rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 scripts/ax_via_at.py > $O/axat_def.json 2> $O/axat_def.err || exit 1
for s in 1 2 4 8; do GLX_ATR_S=$s timeout -k 10 120 python3 scripts/ax_via_at.py > $O/axat_s$s.json 2> $O/axat_s$s.err || exit 1; done
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D $EXTRA > $O/$name.json 2> $O/$name.err || exit 1; }
EXTRA="" ; run ns_nt; run ns_old GLX_ATR_VARIANT=8
EXTRA="--m 4096 --n 8192 --l 16"; run c2_nt; run c2_old GLX_ATR_VARIANT=8
EXTRA="--m 1024 --force-comm"; run sh_nt; run sh_old GLX_ATR_VARIANT=8
EXTRA="--method gl_FProxGD_primal"; run fi_nt; run fi_old GLX_ATR_VARIANT=8
echo done
