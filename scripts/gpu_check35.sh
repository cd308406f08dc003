#!/bin/bash
# Kernel trace of the m = 1024 shard iteration and of NS: busy time per kernel and gaps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r35; mkdir -p $O
for m in 1024 8192; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$m -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --m $m --profile 0 > $O/b$m.json 2> $O/tr$m.err; rc=$?; echo "trace $m rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
  f=$(find $O/tr$m -name "*kernel_trace.csv" | head -1)
  python scripts/trace_gaps.py $f --last 1500 > $O/gaps$m.txt; cat $O/gaps$m.txt
done
cat $O/status.txt | tr '\n' ' '
