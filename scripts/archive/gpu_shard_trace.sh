#!/bin/bash
# Per-rank schedule of the 2/4/8-GPU runs modelled on one GPU: bench at the shard row counts,
# without and with the (world-1, identity) communicator path, under a rocprofv3 kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-shard}; rm -rf $O; mkdir -p $O
for m in 1024 2048; do for c in "" "--force-comm"; do
tag=m${m}${c:+_comm}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --m $m $c > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
python -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag %.1f it/s' % d['value'])"
python scripts/trace_gaps.py $(find $O/$tag -name "*kernel_trace.csv" | head -1) --last 2000
done; done
cat $O/status.txt | tr '\n' ' '
