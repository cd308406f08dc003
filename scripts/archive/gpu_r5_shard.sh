#!/bin/bash
# Round 5: the row-sharded ProxGD schedule. Parity tests (host-staged
# world 2 / 3 / 8, the collectives, the world-1 RCCL identities and timing model), then the per-rank
# model at the 8 / 4 / 2-GPU shards of NS: the all-reduce schedule (--force-comm) against the
# row-sharded one (GLX_SHARD_MODEL = G: the trial on n / G rows), and a kernel trace of each at 1024 rows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_shard}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_comm.py \
  tests/test_gpu_dist.py -k "row_sharded or host_reduce or world1 or matches_oracle" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for pair in "1024 8" "2048 4" "4096 2"; do
  set -- $pair
  for mode in ar shard; do
    if [ $mode = shard ]; then export GLX_SHARD_MODEL=$2; else unset GLX_SHARD_MODEL; fi
    timeout -k 10 300 python3 bench.py --m $1 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve \
      > $O/m$1.$mode.json 2> $O/m$1.$mode.err || exit 1
    echo -n "m=$1 $mode: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/m$1.$mode.json | tee -a $O/status.txt
  done
done
unset GLX_SHARD_MODEL
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_ar -o run -- python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr_ar.log 2>&1 || exit 1
export GLX_SHARD_MODEL=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_shard -o run -- python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr_shard.log 2>&1 || exit 1
python3 scripts/trace_db_summary.py $(find $O -name "*.db") | tee -a $O/status.txt
echo done >> $O/status.txt
