#!/bin/bash
# Round 4 batch 2: the 16-B gather (GLX_GATHER_VEC) against the 8-B one over whole NS solves,
# C3 with the fp32 eight-wave A^T R default, and the driver's command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_pt4.log 2>&1 || { tail -30 gpurun_out/r4_pt4.log; exit 1; }
WHOLE=1 OUT=r4_gvec REPS=2 LAST=3000 bash scripts/gpu_ab.sh "vec|.|GLX_GATHER_VEC=1" "scalar|.|GLX_GATHER_VEC=0" "vec_gdef_k0|.|GLX_GATHER_NT=0 GLX_AX_KEEP_MIB=0 GLX_ATR_KEEP_MIB=0" "vec_gdef_k64|.|GLX_GATHER_NT=0 GLX_AX_KEEP_MIB=64 GLX_ATR_KEEP_MIB=64" || exit 1
OUT=r4_c3 REPS=1 BENCH="--steps 200 --warmup 20 --method gl_FProxGD_primal --dtype f32" bash scripts/gpu_ab.sh "c3|.|GLX_X=1" || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_drv_b2_$r.json 2> gpurun_out/r4_drv_b2_$r.err || exit 1
done
echo batch2 done
