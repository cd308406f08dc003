#!/bin/bash
# Round 2: split-candidate FProxGD with the nnz budget — parity subset, whole solves at several
# budgets against the dense batch, the 200-step bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_fista2; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_dist.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
F="python3 scripts/full_solve.py --method gl_FProxGD_primal"
GLX_SPLIT_FISTA=0 timeout -k 10 200 $F > $O/full_dense.json 2> $O/full_dense.err || exit 1
for b in 0.35 0.2 0.5 10; do
  GLX_SPLIT_NNZ=$b timeout -k 10 200 $F > $O/full_$b.json 2> $O/full_$b.err || exit 1
done
D="python3 bench.py --gpus 1 --no-cpu-baseline --method gl_FProxGD_primal"
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200_split.json 2> $O/b200_split.err || exit 1
GLX_SPLIT_FISTA=0 timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200_dense.json 2> $O/b200_dense.err || exit 1
echo done
