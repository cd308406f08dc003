#!/bin/bash
# Round 5: K splits of the dense pass against the finalize's slab reads (the deferred reductions
# on): C2 (two right-hand sides, GLX_AXB_S) and NS (one, GLX_AX_S), 200-step windows, two rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_split_sweep}; rm -rf $O; mkdir -p $O
run() {   # tag, env, bench args
  local tag=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve "$@" > $O/$tag.json 2> $O/$tag.err || return 1
  echo -n "$tag: " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$tag.json | tee -a $O/status.txt
}
for rep in 1 2; do
  for s in 0 4 8 12; do
    run c2_s$s.$rep GLX_AXB_S=$s --m 4096 --n 8192 --l 16 || exit 1
  done
  for s in 0 4 6; do
    run ns_s$s.$rep GLX_AX_S=$s || exit 1
  done
done
grep -h "describe\|session_plan" $O/c2_s0.1.json | head -2 > /dev/null
python3 - $O <<'PY' >> $O/status.txt
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.1.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f, d["roofline"].get("session_plan"))
PY
echo done >> $O/status.txt
