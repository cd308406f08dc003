#!/bin/bash
# Round 6: FProxGD's over-budget split batches in the fused form (GLX_AE_HYB_ROWS = the gather's
# count from which they take it; 0 = off: the dense batch as before): the egat tests, then NS
# FProxGD whole solves (bench whole_solve) over thresholds, 2 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_fhyb}; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_egat.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in "f0:GLX_AE_HYB_ROWS=0" "f2000:GLX_AE_HYB_ROWS=2000" "f4000:GLX_AE_HYB_ROWS=4000" "f6000:GLX_AE_HYB_ROWS=6000"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.$rep.json 2> $O/$name.$rep.err || exit 1
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
