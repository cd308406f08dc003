#!/bin/bash
# Round 4 experiments 3: the f32 LDS-DMA A@X tile (92478) — kernel numerics, C3 FProxGD dense
# vs split-candidate (GLX_SPLIT_F32=1) with it, a kernel trace of the split run, the fp32 drift
# margins; then k_resgrad2 with the deeper tile prefetch (lags 24, 12).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp3; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "92478 or f32_dma or 21410 or 52324" > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for r in 1 2; do
  for mode in dense split; do
    if [ $mode = split ]; then export GLX_SPLIT_F32=1; else unset GLX_SPLIT_F32; fi; export GLX_AX_DMA32=1
    timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline > $O/c3_$mode.$r.json 2> $O/c3_$mode.$r.err || { tail -20 $O/c3_$mode.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0), 'whole', d.get('whole_solve',{}).get('iters_per_s'), d.get('whole_solve',{}).get('fval'))" $O/c3_$mode.$r.json
  done
done
export GLX_SPLIT_F32=1 GLX_AX_DMA32=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
python3 - $O/tr/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("%-70s calls %6s avg %8.1f us  %5.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
unset GLX_SPLIT_F32
timeout -k 10 400 python3 -u scripts/f32_split_margins.py --c3 > $O/margins.jsonl 2> $O/margins.err || { tail -20 $O/margins.err; exit 1; }
cat $O/margins.jsonl
LAGS="24 12" OUT=r4_exp3/rg2 bash scripts/gpu_r4_rg2x.sh > $O/rg2.txt 2>&1 || { cat $O/rg2.txt; exit 1; }
grep resgrad2 $O/rg2/summary.txt
