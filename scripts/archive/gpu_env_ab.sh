#!/bin/bash
# A/B of one environment knob end to end, alternating runs, optionally after a pytest subset.
#   bash scripts/gpu_env_ab.sh TAG VAR "values" "bench args (;-separated configs)" ["pytest files"]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2; VALS=$3; CONFIGS=$4; TESTS=$5
O=gpurun_out/$TAG; rm -rf $O; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log
  [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -120; exit 1; }
fi
IFS=';' read -ra CFG <<< "$CONFIGS"
for rep in 1 2; do for ci in "${!CFG[@]}"; do for v in $VALS; do
  f=$O/c${ci}_${v}.$rep
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline ${CFG[$ci]} > $f.out 2> $f.err || { echo "bench [${CFG[$ci]}] $VAR=$v failed"; tail -5 $f.err; exit 1; }
  python -c "
import json; d=json.loads(open('$f.out').read().strip().splitlines()[-1]); r=d['roofline']
print('[${CFG[$ci]}] $VAR=$v rep $rep: %.1f it/s  ax %.1fus atr %.1fus' % (d['value'], r['avg_launch_us'], r['atr_avg_launch_us']))" | tee -a $O/summary.txt
done; done; done
