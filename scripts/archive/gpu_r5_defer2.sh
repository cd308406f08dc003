#!/bin/bash
# Round 5: deferred reductions extended to FProxGD: the FISTA / ProxGD parity, golden, device-
# control and fused suites, then NS FProxGD / C3 with GLX_DEFER_RED=0 / 1 interleaved.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_defer2}; rm -rf $O; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_ns_golden.py tests/test_gpu_comm.py tests/test_gpu_dc.py tests/test_gpu_fused.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for rep in 1 2; do
  for d in 0 1; do
    run nsf_w_d$d.$rep GLX_DEFER_RED=$d --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline || exit 1
    run c3_w_d$d.$rep GLX_DEFER_RED=$d --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
  done
done
echo done >> $O/status.txt
