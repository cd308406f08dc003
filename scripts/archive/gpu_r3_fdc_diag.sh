#!/bin/bash
# Diagnose the world-2 FProxGD device-control twin at (256, 16384, 32): full per-rank records.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_fdc_diag; rm -rf $O; mkdir -p $O
for w in "0,8" "0,1"; do
timeout -k 10 200 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  tests/dc_dist_worker.py --shape 256,16384,32 --dtype f64 --alpha-scale 1.0 --opts '{"maxit": 300}' --env '{}' \
  --windows $w --slices 0 --out $O/twin_${w/,/_}.json --method gl_FProxGD_primal > $O/run_${w/,/_}.log 2>&1 || exit 1
done
OMP_NUM_THREADS=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 \
  tests/dc_dist_worker.py --shape 256,16384,32 --dtype f64 --alpha-scale 1.0 --opts '{"maxit": 300}' --env '{}' \
  --windows 0,8 --slices 0 --out $O/twin_w1.json --method gl_FProxGD_primal > $O/run_w1.log 2>&1 || exit 1
echo done
