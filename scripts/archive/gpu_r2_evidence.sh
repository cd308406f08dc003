#!/bin/bash
# Round 2 evidence at HEAD: GPU suite, smoke, driver-form and 200-step bench lines, the rocprofv3
# kernel trace of the driver's exact command, the one-pass kernel against two passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_evidence; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
D="python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 200 $D > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 200 $D --no-cpu-baseline > $O/driver2.json 2> $O/driver2.err || exit 1
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/b200.json 2> $O/b200.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $D --no-cpu-baseline > $O/driver_prof.json 2> $O/driver_prof.err || exit 1
timeout -k 10 120 python3 scripts/rg_bench.py > $O/rg.jsonl 2> $O/rg.err || exit 1
echo done
