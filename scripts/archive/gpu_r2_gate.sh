#!/bin/bash
# Round 2: full GPU suite + smoke after the split-size gate and the A^T R load remap / nt rule,
# then the bench lines (NS driver form and 200 steps, C2, 1024-row comm shard, FProxGD) and a
# kernel trace of the NS 200-step line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_gate; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/status.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
D="python3 bench.py --gpus 1"
timeout -k 10 300 $D --steps 20 --warmup 5 > $O/driver.json 2> $O/driver.err || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline"
timeout -k 10 200 $D --steps 200 --warmup 20 > $O/b200.json 2> $O/b200.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --m 4096 --n 8192 --l 16 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --m 1024 --force-comm > $O/s1024.json 2> $O/s1024.err || exit 1
timeout -k 10 200 $D --steps 200 --warmup 20 --method gl_FProxGD_primal > $O/fista.json 2> $O/fista.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 > $O/prof.json 2> $O/prof.err || exit 1
echo done
