#!/bin/bash
# Round 5: the 32-column A^T R panel with eight waves (WL 4) against WL 3 (four waves) at C2:
# kernel / fused parity tests, then C2 200-step windows interleaved and whole solves.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_wl4}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "atr_codes" \
  tests/test_gpu_fused.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for rep in 1 2; do
  run c2_wl3.$rep GLX_ATR_NARROW=1 --m 4096 --n 8192 --l 16 || exit 1
  run c2_wl4.$rep GLX_ATR_NARROW=8 --m 4096 --n 8192 --l 16 || exit 1
done
echo done >> $O/status.txt
