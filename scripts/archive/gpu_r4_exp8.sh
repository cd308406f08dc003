#!/bin/bash
# Round 4 experiment 8: the row kernels' grid (GLX_ROW_BLOCKS caps their work workgroups) at the
# 8-GPU shard model (1024 rows, the communicator code path with a world-1 RCCL communicator),
# where the replicated trial kernel runs every iteration; interleaved, with a kernel trace each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp8; rm -rf $O; mkdir -p $O
for meth in gl_ProxGD_primal gl_FProxGD_primal; do
  for rb in 0 512 256 128; do
    tag=${meth:3:3}_$rb
    GLX_ROW_BLOCKS=$rb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o run -- python3 bench.py --method $meth --m 1024 --force-comm --steps 400 --warmup 40 --no-cpu-baseline --no-whole-solve > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
    python3 - $O/$tag/run_kernel_stats.csv $O/$tag.json $tag <<'PY'
import csv, json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
ks = {r["Name"].split("(")[0][-40:]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
sel = {k: round(v, 1) for k, v in ks.items() if any(s in k for s in ("prox_pgd", "fista_trial", "finalize", "ax_", "atr", "ctl"))}
print(sys.argv[3], "%.1f it/s" % d["value"], sel)
PY
  done
done
