#!/bin/bash
# Round 3: sanity of the last library build (timed launches raise on failure): profile, fused,
# C ABI and GEMV tests, then one driver-form bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_sanity; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_profile.py tests/test_gpu_fused.py tests/test_gpu_cabi.py tests/test_gpu_gemv_fused.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
tail -2 $O/pytest.log > $O/status.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['launches_timed'], d['whole_solve']['iters_per_s'])" >> $O/status.txt
