#!/bin/bash
# Round 6: timing probe of the fused shard pass (GLX_DRV_PROBE: 1 = no A e work, 2 = no p_thr, 3 = neither)
set -o pipefail
OUT=gpurun_out/${1:-r6h}
mkdir -p $OUT
export TMPDIR=/tmp
B="python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8"
for v in "full:" "nothr3:GLX_DRV_THR=3" "nocomb:GLX_DRV_PROBE=4" "bare:GLX_DRV_THR=3 GLX_DRV_PROBE=7" "split:GLX_SHARD_DERIVE=0"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 $B > $OUT/pg1024_$name.json 2> $OUT/pg1024_$name.err || { echo "pg1024 $name failed"; tail -5 $OUT/pg1024_$name.err; exit 1; }
done
echo "model ok"
[ -n "$PROF" ] || exit 0
cd /tmp && cd $GRAFT_REPO_ROOT
for v in full nogat; do
  pr=0; [ $v = nogat ] && pr=1
  GLX_DRV_PROBE=$pr timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o pg -- python bench.py --steps 200 --warmup 20 \
    --no-cpu-baseline --no-whole-solve --force-comm --m 1024 --shard-model 8 > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { echo "prof $v failed"; exit 1; }
done
echo "prof ok"
