#!/bin/bash
# Round 2: split-candidate ProxGD (A @ [e | p_thr]) — GPU suite, then A/B bench against the dense
# [z | p_thr] batch (GLX_SPLIT_CAND=0) on the same box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_split; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
B="python3 bench.py --gpus 1 --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 200 $B --steps 200 --warmup 20 > $O/sc_$i.json 2> $O/sc_$i.err || exit 1
  GLX_SPLIT_CAND=0 timeout -k 10 200 $B --steps 200 --warmup 20 > $O/dense_$i.json 2> $O/dense_$i.err || exit 1
done
timeout -k 10 200 $B --steps 20 --warmup 5 > $O/sc_driver.json 2> $O/sc_driver.err || exit 1
timeout -k 10 200 $B --steps 200 --warmup 20 --method gl_FProxGD_primal > $O/fista.json 2> $O/fista.err || exit 1
echo done
