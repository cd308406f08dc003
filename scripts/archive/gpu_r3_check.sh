#!/bin/bash
# Round 3 check: the whole GPU suite (world-8 test apart), smoke, whole-solve A/B of device
# control for FProxGD (split-candidate batches with the nnz budget), the driver's command and
# its kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_check}; rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
for r in 1 2; do for w in 0 8; do
  GLX_DC_BATCH=$w timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal > $O/nsf_full_dc${w}_r$r.json 2> $O/nsf_full_dc${w}_r$r.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/nsf_full_dc${w}_r$r.json').read().strip().splitlines()[-1])
print('nsf full dc $w r $r: k %d %.1f it/s fval %.10g stats %s' % (d['k'], d['its'], d['fval'], d['stats']))" | tee -a $O/status.txt
done; done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/driver_cmd_kernel_stats.csv \;
echo done >> $O/status.txt
