#!/bin/bash
# Round 5: the N-rank bench path with the row-sharded schedule, rehearsed on one GPU through the
# host transport (2 and 4 ranks sharing cuda:0; not a performance number), short windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_rehearse}; rm -rf $O; mkdir -p $O
for N in 2 4; do
  timeout -k 10 400 python3 bench.py --gpus $N --comm host --steps 10 --warmup 3 --no-cpu-baseline > $O/host$N.json 2> $O/host$N.err || { tail -30 $O/host$N.err; exit 1; }
  python3 - $O/host$N.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
w = d.get("whole_solve") or {}
print(d["n_gpus"], d["config"]["parallelism"], "| value", round(d["value"], 1), "| whole k", w.get("k"),
      "fval", w.get("fval"), "within_bar", (w.get("vs_reference") or {}).get("within_bar"))
PY
done
