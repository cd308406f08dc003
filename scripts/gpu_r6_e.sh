#!/bin/bash
# Round 6: per-rank models at the multi-GPU shards (bench.py --force-comm, world-1 RCCL).
set -o pipefail
OUT=gpurun_out/${1:-r6e}
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm"
# ProxGD 1024-row (8-GPU) shard, the row-sharded timing model: knobs of the small kernels
for v in "base:" "gbm_novec:GLX_GATHER_BM=8,256,0" "gbm_seg128:GLX_GATHER_BM=8,128,1" "axs16:GLX_AX_S=16" "fin512:GLX_FIN_PER_BLOCK=512" \
         "dma268:GLX_AX_VARIANT=92268" "atr38:GLX_ATR_VARIANT=38" "atrS2:GLX_ATR_S=2" "axl512:GLX_AXL_BLOCKS=512"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 $B --m 1024 --shard-model 8 > $OUT/pg1024_$name.json 2> $OUT/pg1024_$name.err || { echo "pg1024 $name failed"; exit 1; }
done
echo "pg1024 ok"
# FProxGD at the 4- and 2-GPU shards: row-sharded model against the all-reduce schedule + dc
for m in 2048 4096; do
  timeout -k 10 120 $B --method gl_FProxGD_primal --m $m --shard-model $((8192 / m)) > $OUT/fi${m}_shard.json 2> $OUT/fi${m}_shard.err || { echo "fi$m shard failed"; exit 1; }
  timeout -k 10 120 $B --method gl_FProxGD_primal --m $m > $OUT/fi${m}_ar.json 2> $OUT/fi${m}_ar.err || { echo "fi$m ar failed"; exit 1; }
done
echo "fi ok"
# kernel trace of the 1024-row ProxGD and FProxGD models
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_pg -o pg -- python bench.py --steps 200 --warmup 20 \
  --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8 > $OUT/prof_pg.json 2> $OUT/prof_pg.err || { echo "prof pg failed"; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_fi -o fi -- python bench.py --method gl_FProxGD_primal \
  --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8 > $OUT/prof_fi.json 2> $OUT/prof_fi.err || { echo "prof fi failed"; exit 1; }
echo "prof ok"
