#!/bin/bash
# Round 5 closing table at HEAD (after the row-sharded schedule and the deferred reductions): the
# new row-sharded tests, then scripts/gpu_r5_table.sh into r5_table2 plus the row-sharded shard
# models (GLX_SHARD_MODEL = G).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py -k "other_modes" \
  > gpurun_out/r5_table2_pytest.log 2>&1 || { tail -30 gpurun_out/r5_table2_pytest.log; exit 1; }
tail -1 gpurun_out/r5_table2_pytest.log
OUT=r5_table2 bash scripts/gpu_r5_table.sh || exit 1
O=gpurun_out/r5_table2
for pair in "1024 8" "2048 4" "4096 2"; do
  set -- $pair
  GLX_SHARD_MODEL=$2 timeout -k 10 300 python3 bench.py --m $1 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/rows$1.json 2> $O/rows$1.err || exit 1
  echo -n "rows-sharded model $1 (x$2): " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/rows$1.json | tee -a $O/status.txt
done
