#!/bin/bash
# Round 2 closing check: GPU suite + smoke + the driver's bench command + C2 at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_last; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 --m 4096 --n 8192 --l 16 > $O/c2.json 2> $O/c2.err || exit 1
echo "all rc=0" >> $O/status.txt
