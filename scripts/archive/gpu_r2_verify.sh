#!/bin/bash
# Round 2 HEAD verification: GPU suite + smoke, the driver's exact bench command, and its kernel
# trace under rocprofv3.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2_verify}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200.json 2> $O/b200.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --m 1024 --force-comm > $O/s1024.json 2> $O/s1024.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.json 2> $O/prof.err || exit 1
echo "all rc=0" >> $O/status.txt
echo done
