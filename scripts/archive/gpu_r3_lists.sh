#!/bin/bash
# Round 3: column lists with the masks kept in registers (one load round): split-candidate and
# FISTA tests, then the NS 200-step kernel trace (k_e_lists average) and the driver form.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_lists}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_dist.py tests/test_gpu_dc_dist.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size or FProx or world3 or dc" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -2 $O/pytest_split.log >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/prof.json 2> $O/prof.err || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
cat $O/prof_gaps.txt >> $O/status.txt
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/driver_r$r.json 2> $O/driver_r$r.err || exit 1
  python3 -c "import json; d=json.loads([x for x in open('$O/driver_r$r.json') if x.startswith('{\"')][-1]); print('driver r$r', round(d['value'],1))" >> $O/status.txt
done
echo done >> $O/status.txt
