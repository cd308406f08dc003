#!/bin/bash
# Round 2: fused residual-gradient kernel — numerics test, then timing against two passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_resgrad; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_resgrad.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 scripts/rg_bench.py > $O/rg.jsonl 2> $O/rg.err || exit 1
timeout -k 10 120 python3 scripts/rg_bench.py --m 1024 > $O/rg_1024.jsonl 2>> $O/rg.err || exit 1
echo done
