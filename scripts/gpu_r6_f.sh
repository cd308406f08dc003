#!/bin/bash
# Round 6: the row-sharded derive fused into the dense pass (k_ax_lds DRV): parity, per-rank model
set -o pipefail
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations 10 \
  tests/test_gpu_dist.py -k "row_sharded_split_candidate or ns_world8 or test_row_sharded_proxgd" \
  > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8"
for v in "fused:" "nocomb:GLX_DRV_PROBE=4" "split:GLX_SHARD_DERIVE=0" "fused2:"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 $B > $OUT/pg1024_$name.json 2> $OUT/pg1024_$name.err || { echo "pg1024 $name failed"; tail -5 $OUT/pg1024_$name.err; exit 1; }
done
echo "model ok"
cd /tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pg -o pg -- python bench.py --steps 200 --warmup 20 \
  --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8 > $OUT/prof_pg.json 2> $OUT/prof_pg.err || { echo "prof pg failed"; exit 1; }
echo "prof ok"
