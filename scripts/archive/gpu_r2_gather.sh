#!/bin/bash
# Round 2: split-candidate ProxGD, gather form (A e from a transposed copy of A): GPU suite, bench
# windows and a whole NS solve, each against GLX_SPLIT_CAND=0 / sp on the same box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_gather; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 $B --steps 200 --warmup 20 > $O/sc_$i.json 2> $O/sc_$i.err || exit 1
  GLX_SPLIT_CAND=0 timeout -k 10 200 $B --steps 200 --warmup 20 > $O/dense_$i.json 2> $O/dense_$i.err || exit 1
  timeout -k 10 200 $B --steps 20 --warmup 5 > $O/scd_$i.json 2> $O/scd_$i.err || exit 1
  GLX_SPLIT_CAND=0 timeout -k 10 200 $B --steps 20 --warmup 5 > $O/densed_$i.json 2> $O/densed_$i.err || exit 1
done
GLX_SPLIT_CAND=sp timeout -k 10 200 $B --steps 200 --warmup 20 > $O/sp.json 2> $O/sp.err || exit 1
timeout -k 10 200 python3 scripts/full_solve.py > $O/full_sc.json 2> $O/full_sc.err || exit 1
GLX_SPLIT_CAND=0 timeout -k 10 200 python3 scripts/full_solve.py > $O/full_dense.json 2> $O/full_dense.err || exit 1
echo done
