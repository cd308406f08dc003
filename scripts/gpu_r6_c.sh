#!/bin/bash
# Round 6: the fused A e (A p on MFMA + A e on VALU) and the row-sharded FProxGD.
set -o pipefail
OUT=gpurun_out/${1:-r6c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 150 --timeout-method thread --maxfail=4 \
  tests/test_gpu_egat.py tests/test_gpu_ragged_split.py \
  "tests/test_gpu_dist.py::test_row_sharded_fprox" \
  "tests/test_gpu_dist.py::test_row_sharded_fprox_matches_allreduce_schedule" \
  "tests/test_gpu_dist.py::test_row_sharded_fprox_c5_shard_shape" \
  "tests/test_gpu_dist.py::test_sharded_matches_oracle" \
  tests/test_gpu_ns_golden.py > $OUT/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
for f in 0 1; do   # NS: A e fused into the dense pass against the gather form
  GLX_AE_FUSED=$f timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline \
    > $OUT/ns_fused$f.json 2> $OUT/ns_fused$f.err || { echo "ns fused$f failed"; exit 1; }
done
echo "ns ab ok"
# FProxGD per-rank model at the 8-GPU shard: row-sharded (timing model) against all-reduce + dc
timeout -k 10 150 python bench.py --method gl_FProxGD_primal --m 1024 --force-comm --shard-model 8 \
  --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $OUT/fi1024_shard.json 2> $OUT/fi1024_shard.err || { echo "fi shard failed"; exit 1; }
timeout -k 10 150 python bench.py --method gl_FProxGD_primal --m 1024 --force-comm \
  --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $OUT/fi1024_ar.json 2> $OUT/fi1024_ar.err || { echo "fi ar failed"; exit 1; }
echo "fi model ok"
