#!/bin/bash
# Round 4 batch 6: kind-8 LDS-DMA tiles (one row tile per wave) for the batched right-hand sides:
# kernel tests, then NS FProxGD with the dense [xc | y_next] batch on each tile (GLX_SPLIT_FISTA=0:
# every batch dense) and the default whole solve.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "residual" > gpurun_out/r4_pt6.log 2>&1 || { tail -30 gpurun_out/r4_pt6.log; exit 1; }
F="--steps 200 --warmup 20 --method gl_FProxGD_primal"
OUT=r4_fdense REPS=2 BENCH="$F" bash scripts/gpu_ab.sh "k5|.|GLX_SPLIT_FISTA=0" "k8s2|.|GLX_SPLIT_FISTA=0 GLX_AXB_VARIANT=82278" "k8s3|.|GLX_SPLIT_FISTA=0 GLX_AXB_VARIANT=83278" "k8s3d|.|GLX_SPLIT_FISTA=0 GLX_AXB_VARIANT=83268" || exit 1
echo batch6 done
