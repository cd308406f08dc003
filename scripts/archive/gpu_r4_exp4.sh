#!/bin/bash
# Round 4 experiment 4: split-candidate column lists + A e gather on a side stream beside the
# dense pass (GLX_GATHER_OVERLAP=1) — parity (forced-split golden cases, NS whole-solve golden)
# and NS ProxGD / FProxGD throughput, interleaved A/B, driver form and 200-step windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp4; rm -rf $O; mkdir -p $O
GLX_GATHER_OVERLAP=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ns_golden.py -x -q --timeout 120 --timeout-method thread -k "split or ns_golden or full_size" > $O/pytest_ov.log 2>&1 || { tail -30 $O/pytest_ov.log; exit 1; }
tail -1 $O/pytest_ov.log
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; w=d.get('whole_solve') or {}; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f gather %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0, r.get('gather_avg_launch_us') or 0), 'whole', w.get('iters_per_s'), w.get('fval'))" $1; }
for r in 1 2; do
  for ov in 0 1; do
    GLX_GATHER_OVERLAP=$ov timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_ov$ov.$r.json 2> $O/drv_ov$ov.$r.err || { tail -20 $O/drv_ov$ov.$r.err; exit 1; }
    summ $O/drv_ov$ov.$r.json
    GLX_GATHER_OVERLAP=$ov timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/w200_ov$ov.$r.json 2> $O/w200_ov$ov.$r.err || { tail -20 $O/w200_ov$ov.$r.err; exit 1; }
    summ $O/w200_ov$ov.$r.json
    GLX_GATHER_OVERLAP=$ov timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fista_ov$ov.$r.json 2> $O/fista_ov$ov.$r.err || { tail -20 $O/fista_ov$ov.$r.err; exit 1; }
    summ $O/fista_ov$ov.$r.json
  done
done
GLX_GATHER_OVERLAP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
python3 - $O/tr/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print("%-70s calls %6s avg %8.1f us  %5.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
# C3 (fp32 FProxGD) A^T R with the 16-step ring (GLX_ATR_PF16=1), split-candidate batch
for r in 1 2; do
  for pf in 0 1; do
    GLX_AX_DMA32=1 GLX_SPLIT_F32=1 GLX_ATR_PF16=$pf timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/c3pf$pf.$r.json 2> $O/c3pf$pf.$r.err || { tail -20 $O/c3pf$pf.$r.err; exit 1; }
    summ $O/c3pf$pf.$r.json
  done
done
