#!/bin/bash
# Multi-rank rehearsal on one GPU: sharded-solve tests (host transport), an RCCL probe with two
# ranks on one device, a 2-rank bench rehearsal, and the 1024-row shard proxy bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-dist}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "dist tests rc=$rc" >> $O/status.txt
tail -12 $O/pytest.log
[ $rc -eq 0 ] || exit 1
GLX_TEST_DEVICE=0 NCCL_DEBUG=WARN timeout -k 10 90 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tests/dist_gpu_worker.py --transport rccl --out $O/rccl_probe.json > $O/rccl_probe.log 2>&1; echo "rccl probe rc=$?" >> $O/status.txt
tail -5 $O/rccl_probe.log
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --comm host --steps 40 --warmup 5 > $O/bench_host2.json 2> $O/bench_host2.err; rc=$?; echo "bench host2 rc=$rc" >> $O/status.txt
cat $O/bench_host2.json
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --m 1024 --steps 300 --warmup 30 > $O/b_m1024.json 2> $O/b_m1024.err; echo "m1024 rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b_ns.json 2> $O/b_ns.err; echo "ns rc=$?" >> $O/status.txt
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('%-14s %8.1f it/s ax %.1fus atr %.1fus frac %.3f iter_frac %.3f' % ('$f'.split('/')[-1], d['value'], r['avg_launch_us'], r['atr_avg_launch_us'], r['frac'], r['iter_frac']), d['work'])"; done
cat $O/status.txt | tr '\n' ' '
