#!/bin/bash
# Round 5: the bitmap gather's variants at the multi-GPU shards (few rows of A per workgroup
# column: 64 workgroups at 1024 rows with the 16-B row form), all-reduce schedule, 200 steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_gsweep}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist.py -k "row_sharded" \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in 1024 2048 4096; do
  for v in "8,256,1" "8,256,0" "8,128,0" "16,256,0"; do
    GLX_GATHER_BM=$v timeout -k 10 300 python3 bench.py --m $m --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/m$m.$v.json 2> $O/m$m.$v.err || exit 1
    echo -n "m=$m bm=$v: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/m$m.$v.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
