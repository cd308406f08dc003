#!/bin/bash
# Round 2: finalize work per workgroup 256 vs 512 (GLX_FIN_PER_BLOCK), it/s over 200 steps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_fin2; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
for pb in 256 512 256 512; do
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D >> $O/ns_$pb.json 2> $O/ns_$pb.err || exit 1
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D --m 4096 --n 8192 --l 16 >> $O/c2_$pb.json 2> $O/c2_$pb.err || exit 1
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D --m 1024 >> $O/m1024_$pb.json 2> $O/m1024_$pb.err || exit 1
done
echo done > $O/status.txt
