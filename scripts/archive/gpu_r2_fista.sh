#!/bin/bash
# Round 2: split-candidate FProxGD — parity subset, then bench / full solve A/B against the dense
# [xc | y_next] batch (GLX_SPLIT_FISTA=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_fista; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_dist.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --method gl_FProxGD_primal"
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200_split.json 2> $O/b200_split.err || exit 1
GLX_SPLIT_FISTA=0 timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200_dense.json 2> $O/b200_dense.err || exit 1
timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal > $O/full_split.json 2> $O/full_split.err || exit 1
GLX_SPLIT_FISTA=0 timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal > $O/full_dense.json 2> $O/full_dense.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --method gl_FProxGD_primal --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
echo done
