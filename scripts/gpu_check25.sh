#!/bin/bash
# Attribution of the finalize slowdown: merged vs split loops x fused vs separate publish.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r25; mkdir -p $O
P="python bench.py --steps 100 --warmup 10 --no-cpu-baseline"
i=0
for split in 0 1; do for nofuse in 0 1; do
  i=$((i+1))
  E=""
  [ $split -eq 1 ] && export GLX_FIN_SPLIT=1 || unset GLX_FIN_SPLIT
  [ $nofuse -eq 1 ] && export GLX_NO_FUSED_PUBLISH=1 || unset GLX_NO_FUSED_PUBLISH
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_s${split}_n${nofuse} -o b -- $P > $O/b_s${split}_n${nofuse}.json 2>> $O/err.log; rc=$?; echo "s${split}_n${nofuse} rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
done; done
unset GLX_FIN_SPLIT GLX_NO_FUSED_PUBLISH
for d in $O/p_*; do echo "== $d $(python -c "import json; print(round(json.load(open('$O/b_'+'$d'.split('p_')[-1]+'.json'))['value'],1))")"; python - "$d" <<'PY'
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1]+'/b_kernel_stats.csv')))
for r in rows:
    if 'finalize' in r['Name'] or 'publish' in r['Name'] or 'prox' in r['Name']: print('   ', r['Name'][:50], r['Calls'], '%.1f'%(float(r['AverageNs'])/1e3))
PY
done
cat $O/status.txt | tr '\n' ' '
