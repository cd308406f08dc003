#!/bin/bash
# Like gpu_env_sweep.sh, but every config runs under rocprofv3 --kernel-trace --stats and the
# per-kernel average durations (glx kernels) are printed next to the bench value.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-trace}; rm -rf $O; mkdir -p $O
while IFS='|' read -r tag envs args; do
  [ -z "$tag" ] && continue
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python bench.py --no-cpu-baseline $args > $O/$tag.json 2> $O/$tag.err; rc=$?
  echo "$tag rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || { tail -5 $O/$tag.err; exit 1; }
  python - "$O/$tag.json" "$tag" "$envs" "$(find $O/$tag -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = []
for r in csv.DictReader(open(sys.argv[4])):
    name = r["Name"]
    if "glx::" not in name:
        continue
    short = name.split("glx::")[1].split("(")[0].split("<")[0]
    ks.append("%s %.1f" % (short, float(r["AverageNs"]) / 1e3))
print("%-14s %-36s %8.1f it/s | %s" % (sys.argv[2], sys.argv[3], d["value"], ", ".join(ks[:8])))
PY
done < "$2"
