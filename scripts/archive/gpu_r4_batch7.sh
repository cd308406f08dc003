#!/bin/bash
# Round 4 batch 7: Infinity-Cache hand-off sizes in the driver's 20-step window (early
# iterations, small gather), interleaved, 3 reps each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_keepdrv; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for k in 192 224 256 160; do
    GLX_AX_KEEP_MIB=$k GLX_ATR_KEEP_MIB=$k timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/k$k.$r.json 2> $O/k$k.$r.err || exit 1
  done
done
python3 - $O <<'PY' | tee $O/summary.txt
import json, sys, glob, os, collections
O = sys.argv[1]
agg = collections.defaultdict(list)
for f in sorted(glob.glob(O + "/*.json")):
    d = json.loads([x for x in open(f) if x.startswith('{"')][-1]); r = d["roofline"]
    k = os.path.basename(f).split(".")[0]
    agg[k].append((d["value"], r["pair4_frac"], r["avg_launch_us"], r["atr_avg_launch_us"]))
    print(os.path.basename(f), "%.1f it/s pair4 %.3f ax %.1f atr %.1f" % agg[k][-1])
for k, v in agg.items():
    print(k, "mean %.1f it/s pair4 %.3f" % (sum(a[0] for a in v) / len(v), sum(a[1] for a in v) / len(v)))
PY
