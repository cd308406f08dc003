#!/bin/bash
# Round 2: A^T R with contiguous 256-B load pieces (atr_col) — full GPU parity subset, bench A/B
# of the load policy (GLX_ATR_VARIANT=1008: non-temporal), kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_atrcol; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_dist.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D > $O/$name.json 2> $O/$name.err || exit 1; }
run base
run atr_nt GLX_ATR_VARIANT=1008
run base2
run atr_nt2 GLX_ATR_VARIANT=1008

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
GLX_ATR_VARIANT=1008 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_nt -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/prof_nt.json 2> $O/prof_nt.err || exit 1
echo done
