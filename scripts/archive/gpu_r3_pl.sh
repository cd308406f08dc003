#!/bin/bash
# Round 3: per-panel column lists (k_e_plists + LDS-concatenated gather). Split-candidate /
# FISTA / device-control / sharded suites and the profile / fused / C ABI tests, then the NS
# 200-step kernel trace and driver-form lines against GLX_PLISTS=0, two rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_pl}; rm -rf $O; mkdir -p $O
GLX_PLISTS=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_dist.py tests/test_gpu_dc_dist.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size or FProx or world3 or dc" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -2 $O/pytest_split.log >> $O/status.txt
[ $rc -eq 0 ] || exit 1
GLX_PLISTS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_profile.py tests/test_gpu_fused.py tests/test_gpu_cabi.py tests/test_gpu_gemv_fused.py -x -q --timeout 150 --timeout-method thread > $O/pytest_misc.log 2>&1 || exit 1
tail -1 $O/pytest_misc.log >> $O/status.txt
GLX_PLISTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/prof.json 2> $O/prof.err || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/prof_gaps.txt || exit 1
cat $O/prof_gaps.txt >> $O/status.txt
for r in 1 2; do for p in 1 0; do
  GLX_PLISTS=$p timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/d_pl${p}_r$r.json 2> $O/d_pl${p}_r$r.err || exit 1
  GLX_PLISTS=$p timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/w_pl${p}_r$r.json 2> $O/w_pl${p}_r$r.err || exit 1
  python3 -c "
import json
for t in ('d','w'):
    d=json.loads([x for x in open('$O/%s_pl${p}_r$r.json'%t) if x.startswith('{\"')][-1]); r=d['roofline']; ws=d.get('whole_solve')
    print('%s pl$p r$r %.1f it/s ga %s whole %s' % (t, d['value'], r.get('gather_avg_launch_us'), ws and round(ws['iters_per_s'],1)))" >> $O/status.txt
done; done
echo done >> $O/status.txt
