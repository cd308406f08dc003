#!/bin/bash
# Round 5: the row-sharded per-rank model at 1024 rows (GLX_SHARD_MODEL=8: this rank's rows of p
# copied into the other chunks, so e's flagged rows are realistic) under a few launch-shape knobs,
# and its kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_shard2}; rm -rf $O; mkdir -p $O
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve \
    > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
run ar GLX_X=0 || exit 1
run shard GLX_SHARD_MODEL=8 || exit 1
run shard_fin512 GLX_SHARD_MODEL=8 GLX_FIN_PER_BLOCK=512 || exit 1
run shard_fin1024 GLX_SHARD_MODEL=8 GLX_FIN_PER_BLOCK=1024 || exit 1
run shard_rb1024 GLX_SHARD_MODEL=8 GLX_ROW_BLOCKS=1023 || exit 1
run ar2 GLX_X=0 || exit 1
run shard2 GLX_SHARD_MODEL=8 || exit 1
export GLX_SHARD_MODEL=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_shard -o run -- python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr_shard.log 2>&1 || exit 1
python3 scripts/trace_db_summary.py $(find $O/tr_shard -name "*.db") | tee -a $O/status.txt
echo done >> $O/status.txt
