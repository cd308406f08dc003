#!/bin/bash
# Round 5 step E: the per-rank schedule of the multi-GPU path, modelled on one GPU (--force-comm:
# the communicator code path with a world-1 RCCL communicator): the split-candidate trial with
# the bitmap gather (GLX_SPLIT_CAND=1) against the dense [z | p_thr] batch (the size gate's
# choice below 768 MiB) at the 8 / 4 / 2-GPU shards of NS, ProxGD and FProxGD; C5's 16384-row
# FProxGD shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_e; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for m in 1024 2048 4096; do
    for sc in 0 1; do
      for meth in gl_ProxGD_primal gl_FProxGD_primal; do
        GLX_SPLIT_CAND=$sc timeout -k 10 200 python3 bench.py --method $meth --m $m --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/s$m.$meth.$sc.$r.json 2> $O/s$m.$meth.$sc.$r.err || { tail -20 $O/s$m.$meth.$sc.$r.err; exit 1; }
        echo "m=$m split=$sc $meth"; python3 scripts/r5_summ.py $O/s$m.$meth.$sc.$r.json
      done
    done
  done
done
timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --m 16384 --force-comm --steps 100 --warmup 10 --no-cpu-baseline --no-whole-solve > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
echo C5shard; python3 scripts/r5_summ.py $O/c5.json
