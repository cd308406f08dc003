#!/bin/bash
# Round 4: the N-rank bench flow at HEAD, rehearsed on one GPU with the host-staged transport
# (ranks share cuda:0, all-reduces through gloo): NOT a performance number, only that the
# launcher, the sharding, the barriers and the max-over-ranks line work (bench.py --comm host).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_rehearse; rm -rf $O; mkdir -p $O
for g in 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $g --comm host --steps 10 --warmup 2 --no-cpu-baseline --no-whole-solve > $O/host$g.json 2> $O/host$g.err || { tail -20 $O/host$g.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[1], d['n_gpus'], '%.1f it/s' % d['value'], d['config']['parallelism'])" $O/host$g.json
done
