#!/bin/bash
# Round 2: non-temporal A in the l = 1 one-pass GEMV (C4) — its tests, then the C4 bench A/B
# against GLX_GEMV_NT=0 and a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_gemvnt; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemv_fused.py tests/test_gpu_parity.py -k "gemv or SGD or GD" -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --method gl_SGD_primal --m 65536 --n 8192 --l 1 --steps 100 --warmup 10"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D > $O/$name.json 2> $O/$name.err || exit 1; }
run nt; run def GLX_GEMV_NT=0; run nt2; run def2 GLX_GEMV_NT=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $D > $O/prof.json 2> $O/prof.err || exit 1
echo done
