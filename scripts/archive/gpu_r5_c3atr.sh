#!/bin/bash
# Round 5: C3's fp32 A^T R (+ FISTA trial) tiles re-swept (200-step windows, two rounds).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_c3atr}; rm -rf $O; mkdir -p $O
for rep in 1 2; do
  for v in default 1028 1024 1008 1006; do
    if [ $v = default ]; then unset GLX_ATR_VARIANT GLX_ATR_S; else export GLX_ATR_VARIANT=$v GLX_ATR_S=1; fi
    timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/$v.$rep.json 2> $O/$v.$rep.err || exit 1
    echo -n "atr $v ($rep): " | tee -a $O/status.txt; python3 scripts/r5_summ.py $O/$v.$rep.json | tee -a $O/status.txt
  done
done
unset GLX_ATR_VARIANT GLX_ATR_S
python3 - $O <<'PY' >> $O/status.txt
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.1.json")):
    d = json.loads([x for x in open(f) if x.startswith("{")][-1])
    print(f, d["roofline"].get("session_plan"))
PY
echo done >> $O/status.txt
