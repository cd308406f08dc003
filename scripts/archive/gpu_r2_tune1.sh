#!/bin/bash
# Round 2: one-RHS A@X tile sweep at NS, gather-kernel depth/grid A/B, bench windows later in the
# solve (how many rows the threshold touches there), whole solve.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_tune1; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 scripts/kbench.py --ax 52228,51228,51328,52328,54228,52224,52324,54224,21820 --splits 0,4,8,16 --atr 108 --reps 20 > $O/kbench_ax1.jsonl 2> $O/kbench.err || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $B --steps 200 --warmup 20 > $O/g_pf8.json 2> $O/g_pf8.err || exit 1
GLX_GATHER_PF=4 GLX_GATHER_BLOCKS=256 timeout -k 10 200 $B --steps 200 --warmup 20 > $O/g_pf4.json 2> $O/g_pf4.err || exit 1
GLX_GATHER_PF=8 GLX_GATHER_BLOCKS=256 timeout -k 10 200 $B --steps 200 --warmup 20 > $O/g_pf8_256.json 2> $O/g_pf8_256.err || exit 1
GLX_GATHER_PF=4 GLX_GATHER_BLOCKS=1024 timeout -k 10 200 $B --steps 200 --warmup 20 > $O/g_pf4_1024.json 2> $O/g_pf4_1024.err || exit 1
for w in 1000 2000 2600; do
  timeout -k 10 200 $B --steps 200 --warmup $w > $O/w$w.json 2> $O/w$w.err || exit 1
  GLX_SPLIT_CAND=0 timeout -k 10 200 $B --steps 200 --warmup $w > $O/w${w}_dense.json 2> $O/w${w}_dense.err || exit 1
done
timeout -k 10 200 python3 scripts/full_solve.py > $O/full.json 2> $O/full.err || exit 1
echo done
