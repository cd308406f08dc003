#!/bin/bash
# Round 6: the N-rank bench path (the driver's SCALE flow) rehearsed on one GPU through the host
# transport: 8 ranks (1024 rows each: the fused derive pass) and 4 ranks, with the whole solve
# checked against the reference's run; NOT a performance number (ranks share cuda:0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_rehearse}; rm -rf $O; mkdir -p $O
for N in 8 4; do
  timeout -k 10 500 python3 bench.py --gpus $N --comm host --steps 10 --warmup 3 --no-cpu-baseline > $O/host$N.json 2> $O/host$N.err || { tail -30 $O/host$N.err; exit 1; }
  python3 - $O/host$N.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
w = d.get("whole_solve") or {}
print(d["n_gpus"], d["config"]["parallelism"], "| value", round(d["value"], 1), "| whole k", w.get("k"),
      "fval", w.get("fval"), "within_bar", (w.get("vs_reference") or {}).get("within_bar"))
PY
done
