#!/bin/bash
# Round 4 experiment 7: C3 (fp32 FProxGD, split-candidate + f32 LDS-DMA tile) Infinity-Cache
# hand-off sizes (A is 512 MiB in fp32), interleaved, 200-step windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp7; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for k in 192 0 96 256; do
    GLX_AX_KEEP_MIB=$k GLX_ATR_KEEP_MIB=$k timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/k$k.$r.json 2> $O/k$k.$r.err || { tail -20 $O/k$k.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f gather %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0, r.get('gather_avg_launch_us') or 0))" $O/k$k.$r.json
  done
done
