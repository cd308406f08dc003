#!/bin/bash
# Round 5: the finalize with every source's slab loads issued first: parity suites, then C2 / NS
# 200-step windows and a C2 kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_fin}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_ns_golden.py tests/test_gpu_comm.py tests/test_gpu_dc.py tests/test_gpu_kernels.py \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {   # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
run c2.1 --m 4096 --n 8192 --l 16 || exit 1
run ns.1 || exit 1
run c2.2 --m 4096 --n 8192 --l 16 || exit 1
run ns.2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2tr -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --m 4096 --n 8192 --l 16 > $O/c2tr.json 2> $O/c2tr.err || exit 1
python3 scripts/trace_db_summary.py $(find $O/c2tr -name "*.db") | head -8 | tee -a $O/status.txt
echo done >> $O/status.txt
