#!/bin/bash
# Round 5: deferred trial / finalize reductions (single GPU ProxGD): the ProxGD parity suites, then
# NS and C2 in driver form and 200-step windows with GLX_DEFER_RED=0 / 1 interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_defer}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_ns_golden.py tests/test_gpu_comm.py tests/test_gpu_rows.py tests/test_gpu_dc.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for rep in 1 2; do
  for d in 0 1; do
    run ns_w_d$d.$rep GLX_DEFER_RED=$d --steps 200 --warmup 20 --no-cpu-baseline || exit 1
    run c2_w_d$d.$rep GLX_DEFER_RED=$d --steps 200 --warmup 20 --no-cpu-baseline --m 4096 --n 8192 --l 16 || exit 1
  done
done
run ns_drv GLX_X=0 --steps 20 --warmup 5 || exit 1
run c2_drv GLX_X=0 --steps 20 --warmup 5 --m 4096 --n 8192 --l 16 || exit 1
echo done >> $O/status.txt
