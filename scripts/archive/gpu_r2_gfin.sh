#!/bin/bash
# Round 2: the split-candidate finalize fused into the A e gather — parity (forced split golden
# cases, full-size NS, sharded forced split), NS bench A/B against GLX_GATHER_FIN=0, kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_gfin; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_fused.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D $EXTRA > $O/$name.json 2> $O/$name.err || exit 1; }
EXTRA=""; run fin; run nofin GLX_GATHER_FIN=0; run fin2; run nofin2 GLX_GATHER_FIN=0
timeout -k 10 200 python3 bench.py --gpus 1 --no-cpu-baseline --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
echo done
