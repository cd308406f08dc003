#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_probe; rm -rf $O; mkdir -p $O
for kb in 8; do
  timeout -k 10 60 ./scripts/rg_probe_kb$kb > $O/kb$kb.txt 2>&1 || exit 1
done
timeout -k 10 60 ./scripts/rg_probe_kb8 1024 16384 > $O/kb8_m1024.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_resgrad.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/rg_bench.py > $O/rg.jsonl 2> $O/rg.err || exit 1
GLX_RG_XCD=0 timeout -k 10 120 python3 scripts/rg_bench.py > $O/rg_sc1.jsonl 2>> $O/rg.err || exit 1
echo done
