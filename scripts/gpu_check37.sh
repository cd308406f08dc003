#!/bin/bash
# Finalize lane rule (>= 2^19 lanes) vs slabs-only grouping (GLX_FIN_LANES=1), NS and m = 1024.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r37; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -m gpu -q -x > $O/pytest.log 2>&1; rc=$?; echo "tests rc=$rc" >> $O/status.txt
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
for m in 1024 8192; do for lanes in 1 524288; do
tag=m${m}_l$lanes
GLX_FIN_LANES=$lanes timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- python bench.py --no-cpu-baseline --steps 300 --warmup 30 --m $m > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
python -c "
import json; d=json.load(open('$O/$tag.json')); print('$tag %.1f it/s' % d['value'])"
python scripts/trace_gaps.py $(find $O/$tag -name "*kernel_trace.csv" | head -1) --last 1000 | grep -i "finalize\|publish\|k_ax\|atr"
done; done
cat $O/status.txt | tr '\n' ' '
