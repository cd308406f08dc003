#!/bin/bash
# Round 4 batch: tests of the epilogue/gather changes, base-vs-head A/B (NS, C2), the gather's
# workgroup size over whole solves, and C3's fp32 A^T R on the eight-wave panel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_dc.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_pt3.log 2>&1 || { tail -30 gpurun_out/r4_pt3.log; exit 1; }
OUT=r4_ab3 REPS=2 bash scripts/gpu_ab.sh "base|abtree/base|GLX_X=1" "head|.|GLX_X=1" || exit 1
OUT=r4_ab3c2 REPS=2 BENCH="--steps 200 --warmup 20 --m 4096 --n 8192 --l 16" bash scripts/gpu_ab.sh "base|abtree/base|GLX_X=1" "head|.|GLX_X=1" || exit 1
WHOLE=1 OUT=r4_gw REPS=2 LAST=3000 bash scripts/gpu_ab.sh "gw4|.|GLX_GATHER_WAVES=4" "gw2|.|GLX_GATHER_WAVES=2" "gw1|.|GLX_GATHER_WAVES=1" || exit 1
C3="--steps 200 --warmup 20 --method gl_FProxGD_primal --dtype f32"
OUT=r4_c3atr REPS=2 BENCH="$C3" bash scripts/gpu_ab.sh "c3|.|GLX_X=1" "c3w8s1|.|GLX_ATR_VARIANT=1028 GLX_ATR_S=1" "c3w8s2|.|GLX_ATR_VARIANT=1028 GLX_ATR_S=2" "c3w8p4s1|.|GLX_ATR_VARIANT=1024 GLX_ATR_S=1" || exit 1
echo batch1 done
