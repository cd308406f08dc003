#!/bin/bash
# Round 3: split-candidate / FProxGD parity with the mask-fed column lists (incl. the world-2 twins),
# the device-control A/B and the C2 A^T R sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_combo2; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dc_dist.py tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_fused.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_env_sweep.sh r3_dcab scripts/sweep_dc_r3.txt || exit 1
bash scripts/gpu_env_sweep.sh r3_c2atr scripts/sweep_c2atr.txt || exit 1
echo done
