#!/bin/bash
# Round 3: GPU suite (the world-8 C5 test last, on its own), smoke, bench lines with the LDS-DMA
# A@X default, and the kernel trace of the driver's command for the event/rocprof reconciliation.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_verify}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "not world8" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
D="python3 bench.py --gpus 1"
timeout -k 10 300 $D --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
timeout -k 10 300 $D --steps 20 --warmup 5 --no-cpu-baseline > $O/driver2.json 2> $O/driver2.err || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200.json 2> $O/b200.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --method gl_FProxGD_primal > $O/fista.json 2> $O/fista.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --m 4096 --n 8192 --l 16 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 200 $D --steps 100 --warmup 10 --m 16384 --method gl_FProxGD_primal --force-comm > $O/c5shard.json 2> $O/c5shard.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
echo "bench ok"
timeout -k 10 380 python -u -m pytest tests/test_gpu_dist.py -x -v --timeout 400 --timeout-method thread -k "world8" > $O/world8.log 2>&1; echo "world8 rc=$?" >> $O/status.txt
tail -3 $O/world8.log
echo done
