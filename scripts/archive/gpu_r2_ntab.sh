#!/bin/bash
# Round 2: A/B of the pass-level knobs the streaming probe points at — non-temporal A loads in
# A^T R (GLX_ATR_VARIANT=1008) and the A@X K split (GLX_AX_S) — on the 200-step NS bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_ntab; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D > $O/$name.json 2> $O/$name.err || exit 1; }
run base
run atr_nt GLX_ATR_VARIANT=1008
run base2
run atr_nt2 GLX_ATR_VARIANT=1008
for s in 4 8 16 32; do run axs$s GLX_AX_S=$s; done
echo done
