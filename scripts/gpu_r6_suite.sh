#!/bin/bash
# Round 6: new tests, smoke, the driver-form bench line and the A/B pairs (NS fused A e, C3 ring).
set -o pipefail
OUT=gpurun_out/${1:-r6a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest -v --timeout 120 --timeout-method thread --maxfail=3 \
  tests/test_gpu_egat.py tests/test_gpu_ragged_split.py tests/test_gpu_comm.py \
  "tests/test_gpu_dist.py::test_stalled_rank_watchdog_host_transport" \
  "tests/test_gpu_dist.py::test_row_sharded_ns_world8_whole_solve" \
  "tests/test_gpu_ns_golden.py::test_whole_solve_c3_fp32" > $OUT/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -3 $OUT/pytest_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
echo "bench ok"
for f in 0 1; do   # NS: A e fused into the dense pass (round 6) against the gather form
  GLX_AE_FUSED=$f timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
    > $OUT/ns_fused$f.json 2> $OUT/ns_fused$f.err || { echo "ns fused$f failed"; exit 1; }
done
echo "ns ab ok"
for pf in 8 16; do   # C3: the f32 A^T R ring depth
  GLX_ATR_PF32=$pf timeout -k 10 120 python bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 \
    --no-cpu-baseline > $OUT/c3_pf$pf.json 2> $OUT/c3_pf$pf.err || { echo "c3 pf$pf failed"; exit 1; }
done
echo "c3 ab ok"
