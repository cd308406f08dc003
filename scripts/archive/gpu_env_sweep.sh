#!/bin/bash
# Environment-knob sweep of bench.py end to end: each line of $2 (a file) = "TAG|ENV=.. ENV=..|bench args".
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sweep}; rm -rf $O; mkdir -p $O
while IFS='|' read -r tag envs args; do
  [ -z "$tag" ] && continue
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$tag.err; exit 1; }
  python - "$O/$tag.json" "$tag" "$envs" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print("%-16s %-40s %8.1f it/s ax %6.1fus atr %6.1fus syncs/it %.3f  %s" % (sys.argv[2], sys.argv[3], d["value"], r["avg_launch_us"], r["atr_avg_launch_us"], d["work"]["syncs_per_iter"], r["kernel"]))
PY
done < "$2"
