#!/bin/bash
# Round 5: ProxGD plans without the fused trial on the communicator form of the speculative
# trial, and device control on it: dc / parity / comm suites, then C1 (512, 1024, 2) in driver
# form and 200-step windows: rounds-1-4 form (GLX_UNFUSED_SPEC=0), the new form with host
# control, and with device control (GLX_DC_BATCH=8).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_unfused}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dc.py \
  tests/test_gpu_parity.py tests/test_gpu_comm.py tests/test_gpu_logs.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 --m 512 --n 1024 --l 2 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for rep in 1 2; do
  run old_w.$rep GLX_UNFUSED_SPEC=0 --steps 200 --warmup 20 || exit 1
  run new_w.$rep GLX_DC_BATCH=0 --steps 200 --warmup 20 || exit 1
  run dc8_w.$rep GLX_DC_BATCH=8 --steps 200 --warmup 20 || exit 1
  run dc16_w.$rep GLX_DC_BATCH=16 --steps 200 --warmup 20 || exit 1
done
echo done >> $O/status.txt
