#!/bin/bash
# Verification on one MI355X: GPU test suite, smoke(), then bench lines.
#   bash scripts/gpu_verify.sh TAG ["bench args 1" "bench args 2" ...]   (default: one default bench)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-verify}; shift
O=gpurun_out/$TAG; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -80; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc" >> $O/status.txt
tail -1 $O/smoke.log
[ $rc -eq 0 ] || exit 1
[ $# -eq 0 ] && set -- ""
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python bench.py $args > $O/b$i.json 2> $O/b$i.err; rc=$?; echo "bench$i [$args] rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -20 $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]; w = d["work"]
k = r["kernels"]
print("[%s] %.1f it/s  ax %.1fus (%s %.3f) atr %.1fus pair %.3f iter %.3f  passes %.2f syncs %.2f cpu %s" % (
    sys.argv[2], d["value"], k["ax"]["avg_launch_us"], r["bound"], r["frac"], (k.get("atr") or {}).get("avg_launch_us") or 0,
    r["pair_frac"] or 0, r["iter_frac"], w["passes_over_A_per_iter"], w["syncs_per_iter"],
    (d.get("cpu_baseline") or {}).get("value")))
PY
done
cat $O/status.txt | tr '\n' ' '
