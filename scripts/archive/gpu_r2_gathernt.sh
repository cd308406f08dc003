#!/bin/bash
# Round 2: non-temporal At loads in the A e gather — split-candidate parity, NS A/B
# (GLX_GATHER_NT=0), kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_gathernt; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split_candidate or full_size" -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
run() { name=$1; shift; env "$@" timeout -k 10 200 $D > $O/$name.json 2> $O/$name.err || exit 1; }
run nt; run def GLX_GATHER_NT=0; run nt2; run def2 GLX_GATHER_NT=0
timeout -k 10 200 python3 scripts/full_solve.py > $O/full.json 2> $O/full.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $D > $O/prof.json 2> $O/prof.err || exit 1
echo done
