#!/bin/bash
# Round 5 step B: e / e_c distribution over whole NS solves (scripts/ec_distribution.py) and the
# driver's bench command with the new reference-instance fields (whole_solve.vs_reference,
# cpu_baseline.gpu_same_sample).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_b; rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 scripts/ec_distribution.py > $O/ec.jsonl 2> $O/ec.err || { tail -20 $O/ec.err; exit 1; }
cat $O/ec.jsonl
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || { tail -20 $O/drv.err; exit 1; }
python3 scripts/r5_summ.py $O/drv.json
python3 -c "import json; d=json.loads([x for x in open('$O/drv.json') if x.startswith('{')][-1]); print(json.dumps(d['cpu_baseline'])); print(d['data']); print(json.dumps(d['whole_solve']['vs_reference']))"
