#!/bin/bash
# Round 2: device-controlled ProxGD batches. The new bit-identity tests, the whole GPU suite,
# smoke, the driver's bench command, and same-box A/B lines (GLX_DC_BATCH=0 = host control)
# at NS, C2 and the 1024-row shard, then the driver command's kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r2_dc}; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dc.py -x -v --timeout 120 --timeout-method thread > $O/dc_tests.log 2>&1; rc=$?
echo "dc tests rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
for dc in 8 0; do
  GLX_DC_BATCH=$dc timeout -k 10 200 $D > $O/b200_dc$dc.json 2> $O/b200_dc$dc.err || exit 1
  GLX_DC_BATCH=$dc timeout -k 10 200 $D --m 4096 --n 8192 --l 16 > $O/c2_dc$dc.json 2> $O/c2_dc$dc.err || exit 1
  GLX_DC_BATCH=$dc timeout -k 10 200 $D --m 1024 > $O/m1024_dc$dc.json 2> $O/m1024_dc$dc.err || exit 1
done
echo "bench rc=0" >> $O/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.json 2> $O/prof.err || exit 1
echo "all rc=0" >> $O/status.txt
