#!/bin/bash
# Round 4 experiment 11: the A e gather with each column's list cut into GLX_GATHER_SPLIT pieces
# (one output slab each; default 4) — parity (split-candidate golden / full-size / NS golden /
# device-control twins, world-2 twins), then interleaved A/B 1 / 4 / 8: NS ProxGD driver form and
# 200-step (with whole solves), NS FProxGD whole solves, and a kernel trace of a whole NS solve.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp11; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ns_golden.py tests/test_gpu_dc.py tests/test_gpu_dc_dist.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -k "split or full_size or ns_golden or dc or dist" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); r=d['roofline']; w=d.get('whole_solve') or {}; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f gather %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0, r.get('gather_avg_launch_us') or 0), 'whole', w.get('iters_per_s'), w.get('fval'))" $1; }
for r in 1 2; do
  for sp in 1 4 8; do
    GLX_GATHER_SPLIT=$sp timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/drv_$sp.$r.json 2> $O/drv_$sp.$r.err || { tail -20 $O/drv_$sp.$r.err; exit 1; }
    summ $O/drv_$sp.$r.json
    GLX_GATHER_SPLIT=$sp timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_$sp.$r.json 2> $O/ns_$sp.$r.err || { tail -20 $O/ns_$sp.$r.err; exit 1; }
    summ $O/ns_$sp.$r.json
    GLX_GATHER_SPLIT=$sp timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fi_$sp.$r.json 2> $O/fi_$sp.$r.err || { tail -20 $O/fi_$sp.$r.err; exit 1; }
    summ $O/fi_$sp.$r.json
  done
done
for sp in 1 4; do
  GLX_GATHER_SPLIT=$sp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$sp -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/tr$sp.json 2> $O/tr$sp.err || { tail -20 $O/tr$sp.err; exit 1; }
  python3 - $O/tr$sp/run_kernel_stats.csv $sp <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("k_at_gather", "k_e_lists", "finalize")):
        print("split", sys.argv[2], r["Name"][:50], "calls", r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
