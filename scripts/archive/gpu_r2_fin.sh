#!/bin/bash
# Round 2: finalize workgroup-size sweep (GLX_FIN_PER_BLOCK) at NS, C2 and the 1024-row shape,
# it/s over 200 steps plus a kernel trace per setting at the 1024-row shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_fin; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20"
for pb in 512 1024 2048 4096 512; do
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D > $O/ns_$pb.json 2> $O/ns_$pb.err || exit 1
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D --m 4096 --n 8192 --l 16 > $O/c2_$pb.json 2> $O/c2_$pb.err || exit 1
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 200 $D --m 1024 > $O/m1024_$pb.json 2> $O/m1024_$pb.err || exit 1
done
for pb in 512 2048; do
  GLX_FIN_PER_BLOCK=$pb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$pb -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --steps 200 --warmup 20 --m 1024 > $O/prof_$pb.json 2> $O/prof_$pb.err || exit 1
done
echo done > $O/status.txt
