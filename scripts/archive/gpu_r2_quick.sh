#!/bin/bash
# Round 2 quick check: the split-candidate parity subset and the bench lines (no profile).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_quick; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_dist.py tests/test_gpu_comm.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $D --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200.json 2> $O/b200.err || exit 1
timeout -k 10 200 python3 scripts/full_solve.py > $O/full.json 2> $O/full.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $D --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
echo done
