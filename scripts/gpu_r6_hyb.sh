#!/bin/bash
# Round 6: ProxGD's per-trial A e form (gather below GLX_AE_HYB_ROWS flagged rows, fused above):
# the egat tests, then NS whole solves (bench whole_solve) over thresholds, 2 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_hyb}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_egat.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in "h0:GLX_AE_HYB_ROWS=0" "h1000:GLX_AE_HYB_ROWS=1000" "h1500:GLX_AE_HYB_ROWS=1500" "h2000:GLX_AE_HYB_ROWS=2000" "h2500:GLX_AE_HYB_ROWS=2500" "egat:GLX_AE_FUSED=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.$rep.json 2> $O/$name.$rep.err || exit 1
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
