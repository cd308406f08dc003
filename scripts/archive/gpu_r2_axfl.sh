#!/bin/bash
# Round 2: full-line non-temporal A loads in the single-RHS A@X tile (k_ax_lds FL) — parity
# (default suites + the forced split-candidate golden cases with FL forced at small shapes),
# then the NS bench A/B against GLX_AX_FL=0 and a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_axfl; rm -rf $O; mkdir -p $O
GLX_AX_FL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "split_candidate_forced" -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_forced.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_fused.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D $EXTRA > $O/$name.json 2> $O/$name.err || exit 1; }
EXTRA=""; run fl; run nofl GLX_AX_FL=0; run fl2; run nofl2 GLX_AX_FL=0
EXTRA="--method gl_FProxGD_primal"; run fi_fl; run fi_nofl GLX_AX_FL=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
echo done
