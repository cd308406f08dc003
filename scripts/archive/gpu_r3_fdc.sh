#!/bin/bash
# Round 3: device-controlled FProxGD (N = 1 and host-staged world 2), then the suites the FISTA
# refactor touches (parity, fused trial, dist, C ABI stub).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_fdc}; rm -rf $O; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_dc.py tests/test_gpu_dc_dist.py -x -v --timeout 150 --timeout-method thread > $O/pytest_dc.log 2>&1; rc=$?
echo "dc tests rc=$rc" >> $O/status.txt; tail -5 $O/pytest_dc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_cabi.py tests/test_gpu_dist.py tests/test_gpu_logs.py tests/test_gpu_driver.py -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest_p.log 2>&1; rc=$?
echo "parity tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_p.log
[ $rc -eq 0 ] || exit 1
echo done
