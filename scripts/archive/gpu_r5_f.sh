#!/bin/bash
# Round 5 step F: the bitmap gather's loads in flight / segment (GLX_GATHER_BM) at NS; C2 and the
# (4096, 16384, 32) shape with the split-candidate trial forced; whole solves of the 8- and
# 2-GPU shard models (--force-comm) with and without the split-candidate trial.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_f; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for v in 8,256 16,256 8,128 16,128; do
    GLX_GATHER_BM=$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_$v.$r.json 2> $O/ns_$v.$r.err || { tail -20 $O/ns_$v.$r.err; exit 1; }
    echo "bm=$v"; python3 scripts/r5_summ.py $O/ns_$v.$r.json
  done
done
for sc in 0 1; do
  GLX_SPLIT_CAND=$sc timeout -k 10 300 python3 bench.py --m 4096 --n 8192 --l 16 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_$sc.json 2> $O/c2_$sc.err || { tail -20 $O/c2_$sc.err; exit 1; }
  echo "C2 split=$sc"; python3 scripts/r5_summ.py $O/c2_$sc.json
  GLX_SPLIT_CAND=$sc timeout -k 10 300 python3 bench.py --m 4096 --steps 200 --warmup 20 --no-cpu-baseline > $O/h_$sc.json 2> $O/h_$sc.err || { tail -20 $O/h_$sc.err; exit 1; }
  echo "4096x16384x32 split=$sc"; python3 scripts/r5_summ.py $O/h_$sc.json
  for m in 1024 4096; do
    for meth in gl_ProxGD_primal gl_FProxGD_primal; do
      GLX_SPLIT_CAND=$sc timeout -k 10 300 python3 bench.py --method $meth --m $m --force-comm --steps 100 --warmup 10 --no-cpu-baseline > $O/w$m.$meth.$sc.json 2> $O/w$m.$meth.$sc.err || { tail -20 $O/w$m.$meth.$sc.err; exit 1; }
      echo "shard m=$m split=$sc $meth"; python3 scripts/r5_summ.py $O/w$m.$meth.$sc.json
    done
  done
done
