#!/bin/bash
# Round 4 experiments 2: k_resgrad2 with the deeper A / B tile prefetch (lags 24, 12; XCD-local and
# agent-scope), then C3 fp32 FProxGD split-candidate (GLX_SPLIT_F32=1) with the one-source A@X
# tiles 21410 (direct) / 52324 / 52224 (kind 5), and a kernel trace of the split run.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp2; rm -rf $O; mkdir -p $O
LAGS="24 12" OUT=r4_exp2/rg2 bash scripts/gpu_r4_rg2x.sh > $O/rg2.txt 2>&1 || { cat $O/rg2.txt; exit 1; }
grep resgrad2 $O/rg2/summary.txt
export GLX_SPLIT_F32=1
for v in 21410 52324 52224; do
  GLX_AX_VARIANT=$v timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/c3s_$v.json 2> $O/c3s_$v.err || { tail -20 $O/c3s_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0))" $O/c3s_$v.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
python3 - $O/tr/run_kernel_stats.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print("%-70s calls %6s avg %8.1f us  %5.1f%%" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
