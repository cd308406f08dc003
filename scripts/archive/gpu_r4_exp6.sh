#!/bin/bash
# Round 4 experiment 6: the software-pipelined A e gather (GLX_GATHER_PIPE, default on) — parity
# (split-candidate golden / full-size / NS whole-solve golden / device-control twins), then an
# interleaved A/B against round 3's loop (GLX_GATHER_PIPE=0): NS ProxGD and FProxGD, C3, with
# whole solves; kernel traces of the driver command + whole solve for both.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp6; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ns_golden.py tests/test_gpu_dc.py -x -q --timeout 120 --timeout-method thread -k "split or full_size or ns_golden or dc" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; w=d.get('whole_solve') or {}; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f gather %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0, r.get('gather_avg_launch_us') or 0), 'whole', w.get('iters_per_s'), w.get('fval'))" $1; }
for r in 1 2; do
  for pp in 0 1; do
    GLX_GATHER_PIPE=$pp timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_p$pp.$r.json 2> $O/ns_p$pp.$r.err || { tail -20 $O/ns_p$pp.$r.err; exit 1; }
    summ $O/ns_p$pp.$r.json
    GLX_GATHER_PIPE=$pp timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fi_p$pp.$r.json 2> $O/fi_p$pp.$r.err || { tail -20 $O/fi_p$pp.$r.err; exit 1; }
    summ $O/fi_p$pp.$r.json
    GLX_GATHER_PIPE=$pp timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline > $O/c3_p$pp.$r.json 2> $O/c3_p$pp.$r.err || { tail -20 $O/c3_p$pp.$r.err; exit 1; }
    summ $O/c3_p$pp.$r.json
  done
done
for pp in 0 1; do
  GLX_GATHER_PIPE=$pp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$pp -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/tr$pp.json 2> $O/tr$pp.err || { tail -20 $O/tr$pp.err; exit 1; }
  python3 - $O/tr$pp/run_kernel_stats.csv $pp <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_at_gather" in r["Name"] or "k_e_lists" in r["Name"]:
        print("pipe", sys.argv[2], r["Name"][:60], "calls", r["Calls"], "avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
