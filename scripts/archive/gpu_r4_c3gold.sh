#!/bin/bash
# Round 4: C3 whole-solve parity against the reference's fp32 run (tests/golden/c3_*), margins
# for the split-candidate default and the dense batch.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_c3gold; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u scripts/c3_golden_margins.py > $O/margins.jsonl 2> $O/margins.err || { tail -20 $O/margins.err; exit 1; }
cat $O/margins.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_ns_golden.py -x -q --timeout 240 --timeout-method thread -k c3 > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "f32" > $O/pytest_f32.log 2>&1 || { tail -20 $O/pytest_f32.log; exit 1; }
tail -1 $O/pytest_f32.log
timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 20 --warmup 5 > $O/c3_d.json 2> $O/c3_d.err || exit 1
timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/c3_w.json 2> $O/c3_w.err || exit 1
for f in $O/c3_d.json $O/c3_w.json; do python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); r=d['roofline']; w=d.get('whole_solve') or {}; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0), 'whole', w.get('iters_per_s'))" $f; done
