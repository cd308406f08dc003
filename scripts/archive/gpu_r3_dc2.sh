#!/bin/bash
# Round 3: device control with a communicator after the gating fix (cancelled k_prox_pgd /
# k_fista_trial), the pruned A@X tile set, then the dist suite and the comm-path benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_dc2}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dc_dist.py tests/test_gpu_dc.py -x -v --timeout 150 --timeout-method thread > $O/pytest_dc.log 2>&1; rc=$?
echo "dc tests rc=$rc" >> $O/status.txt; tail -5 $O/pytest_dc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dist.py tests/test_gpu_comm.py -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest_k.log 2>&1; rc=$?
echo "kernel+dist tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_k.log
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --force-comm"
for r in 1 2; do
for m in 1024 2048; do
  for w in 0 8; do
    GLX_DC_BATCH=$w timeout -k 10 120 $D --steps 200 --warmup 20 --m $m > $O/s${m}_dc${w}_r$r.json 2> $O/s${m}_dc${w}_r$r.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/s${m}_dc${w}_r$r.json'))
print('m $m dc $w round $r: %.1f it/s syncs/iter %.3f ax %.1f atr %.1f' % (d['value'], d['work']['syncs_per_iter'], d['roofline']['avg_launch_us'], d['roofline']['atr_avg_launch_us']))" | tee -a $O/status.txt
  done
done
done
echo done
