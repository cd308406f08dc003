#!/bin/bash
# Round 6: the row-sharded derive pass reading p unthresholded (A p; finalize chain 2,
# GLX_SHARD_DRV_AP=1) against the thresholded operands (A p_thr): the NS world-8 whole solve and
# the row-sharded ProxGD tests with it, then the 1024-row model, 3 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_ap}; rm -rf $O; mkdir -p $O
GLX_SHARD_DRV_AP=1 timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_dist.py \
  -k "ns_world8 or test_row_sharded_proxgd" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8"
for rep in 1 2 3; do
  for v in "thr:GLX_SHARD_DRV_AP=0" "ap:GLX_SHARD_DRV_AP=1" "split:GLX_SHARD_DERIVE=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 120 $B > $O/$name.$rep.json 2> $O/$name.$rep.err || { echo "$name failed"; exit 1; }
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
