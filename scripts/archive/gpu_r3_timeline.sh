#!/bin/bash
# Round 3: per-iteration kernel composition and inter-kernel gaps of the NS timed region (driver
# form and a 200-step window), from rocprofv3 kernel traces of bench.py.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_timeline}; rm -rf $O; mkdir -p $O
for w in "20 5" "200 20"; do
  set -- $w
  tag=s$1
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python3 bench.py --gpus 1 --steps $1 --warmup $2 --no-cpu-baseline ${BENCH_ARGS} > $O/$tag.json 2> $O/$tag.err || exit 1
  f=$(find $O/$tag -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_gaps.py $f --markers > $O/${tag}_gaps.txt || exit 1
  python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value'],1), 'it/s')" >> $O/status.txt
  cat $O/${tag}_gaps.txt >> $O/status.txt
done
echo done >> $O/status.txt
