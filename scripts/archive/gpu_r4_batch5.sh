#!/bin/bash
# Round 4 batch 5: C2's fused A^T R on the eight-wave panel (WL 2) with 2 / 4 K splits; the
# 20-step window's clock (the probe build) against a 200-step one.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C2="--steps 200 --warmup 20 --m 4096 --n 8192 --l 16"
OUT=r4_c2atr REPS=2 BENCH="$C2" bash scripts/gpu_ab.sh "c2|.|GLX_X=1" "w8s2|.|GLX_ATR_VARIANT=28 GLX_ATR_S=2" "w8p4s2|.|GLX_ATR_VARIANT=24 GLX_ATR_S=2" "w8s4|.|GLX_ATR_VARIANT=28 GLX_ATR_S=4" || exit 1
cd abtree/probe && timeout -k 10 120 python3 ../../scripts/clock_probe.py --steps 20 --warmup 5 > ../../gpurun_out/r4_clk8.json 2> ../../gpurun_out/r4_clk8.err && timeout -k 10 120 python3 ../../scripts/clock_probe.py --steps 200 --warmup 20 > ../../gpurun_out/r4_clk9.json 2>> ../../gpurun_out/r4_clk8.err || exit 1
echo batch5 done
