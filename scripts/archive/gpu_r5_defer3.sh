#!/bin/bash
# Round 5: deferred reductions only ahead of a carried packet: parity suites, the rejection-heavy
# probe, then NS / C2 / NS FProxGD / C3 200-step windows with GLX_DEFER_RED=0 / 1.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_defer3}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_ns_golden.py tests/test_gpu_comm.py tests/test_gpu_dc.py tests/test_gpu_fused.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for meth in gl_ProxGD_primal gl_FProxGD_primal; do
  for d in 0 1; do
    GLX_DEFER_RED=$d timeout -k 10 200 python3 scripts/defer_probe.py $meth 2.5 >> $O/probe.jsonl 2> $O/probe.err || exit 1
  done
done
cat $O/probe.jsonl
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for d in 0 1; do
  run ns_d$d GLX_DEFER_RED=$d || exit 1
  run c2_d$d GLX_DEFER_RED=$d --m 4096 --n 8192 --l 16 || exit 1
  run nsf_d$d GLX_DEFER_RED=$d --method gl_FProxGD_primal || exit 1
  run c3_d$d GLX_DEFER_RED=$d --method gl_FProxGD_primal --dtype f32 || exit 1
done
echo done >> $O/status.txt
