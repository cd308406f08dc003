#!/bin/bash
# Round 6: the gather form's A e and its finalize in one launch (k_at_gather_fin) against two
# launches (GLX_GATHER_FIN=0): the split-candidate / device-control / golden tests, then NS
# ProxGD in the driver's form (20 + 5, whole solve included), 3 interleaved rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_gf}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ragged_split.py \
  tests/test_gpu_egat.py tests/test_gpu_dc.py tests/test_gpu_ns_golden.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in "gf1:GLX_GATHER_FIN=1" "gf0:GLX_GATHER_FIN=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$name.$rep.json 2> $O/$name.$rep.err || exit 1
    echo -n "$name ($rep): " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/$name.$rep.json | tee -a $O/status.txt
  done
done
echo done >> $O/status.txt
