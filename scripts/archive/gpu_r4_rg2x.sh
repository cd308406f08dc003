#!/bin/bash
# k_resgrad2 with the XCD-local hand-off (GLX_RG_XCD=1, default) against the agent-scope form,
# B-wave lags 12/24/36, C2 shape, under a kernel trace (scripts/rg2_bench.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r4_rg2x}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rg2.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for x in 1 0; do
for lag in ${LAGS:-12 24 36}; do
  GLX_RG_XCD=$x GLX_RG2_LAG=$lag timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x${x}l$lag -o run -- python3 scripts/rg2_bench.py $ARGS > $O/x${x}l$lag.log 2>&1 || { echo "x $x lag $lag failed"; tail -5 $O/x${x}l$lag.log; exit 1; }
  python3 - "$O/x${x}l$lag/run_kernel_stats.csv" "xcd $x lag $lag" >> $O/summary.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "resgrad2" in n or "k_ax_dma" in n or "k_atr" in n or "finalize" in n or "sum_partials" in n:
        print("%s %-40s calls %s avg %.1f min %.1f us" % (sys.argv[2], n[:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
done
done
cat $O/summary.txt
