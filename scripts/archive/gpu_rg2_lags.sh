#!/bin/bash
# k_resgrad2 B-wave lag sweep under a kernel trace: avg k_resgrad2 / k_ax_dma / k_atr durations
# per lag (scripts/rg2_bench.py), C2 shape unless ARGS says otherwise.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r4_rg2lag}; rm -rf $O; mkdir -p $O
for lag in ${LAGS:-12 23 24 36}; do
  GLX_RG2_LAG=$lag timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l$lag -o run -- python3 scripts/rg2_bench.py $ARGS > $O/l$lag.log 2>&1 || { echo "lag $lag failed"; tail -5 $O/l$lag.log; exit 1; }
  python3 - "$O/l$lag/run_kernel_stats.csv" $lag >> $O/summary.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "resgrad2" in n or "k_ax_dma" in n or "k_atr" in n:
        print("lag %s %-40s calls %s avg %.1f min %.1f us" % (sys.argv[2], n[:40], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3))
PY
done
cat $O/summary.txt
