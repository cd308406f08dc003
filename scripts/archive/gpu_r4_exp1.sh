#!/bin/bash
# Round 4 experiments: (1) k_resgrad2 XCD-local / lag sweep (gpu_r4_rg2x.sh); (2) fp32 FProxGD
# split-candidate batch drift (scripts/f32_split_margins.py); (3) C3 bench dense vs split.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp1; rm -rf $O; mkdir -p $O
OUT=r4_exp1/rg2 bash scripts/gpu_r4_rg2x.sh > $O/rg2.txt 2>&1 || { cat $O/rg2.txt; exit 1; }
tail -30 $O/rg2.txt
timeout -k 10 400 python3 -u scripts/f32_split_margins.py --c3 > $O/margins.jsonl 2> $O/margins.err || { tail -20 $O/margins.err; exit 1; }
cat $O/margins.jsonl
for r in 1 2; do
  for mode in dense split; do
    if [ $mode = split ]; then export GLX_SPLIT_F32=1; else unset GLX_SPLIT_F32; fi
    timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline > $O/c3_$mode.$r.json 2> $O/c3_$mode.$r.err || { tail -20 $O/c3_$mode.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0), 'whole', d.get('whole_solve',{}).get('iters_per_s'), d.get('whole_solve',{}).get('fval'))" $O/c3_$mode.$r.json
  done
done
