#!/bin/bash
# Round 3: the per-rank schedule of the N-GPU row shards at HEAD, modelled on one GPU through the
# communicator code path (--force-comm: world-1 RCCL communicator): ProxGD at 1024 / 2048 / 4096
# rows (8 / 4 / 2 GPUs of the NS problem) and FProxGD at C5's 16384-row shard, 200-step windows,
# plus the kernel trace of the 1024-row case.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_shards}; rm -rf $O; mkdir -p $O
B="python3 bench.py --gpus 1 --no-cpu-baseline --no-whole-solve --force-comm"
for m in 1024 2048 4096; do
  timeout -k 10 200 $B --steps 200 --warmup 20 --m $m > $O/pgd_m$m.json 2> $O/pgd_m$m.err || exit 1
done
timeout -k 10 200 $B --steps 100 --warmup 10 --m 16384 --method gl_FProxGD_primal > $O/fpgd_m16384.json 2> $O/fpgd_m16384.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --no-cpu-baseline --no-whole-solve --force-comm --steps 200 --warmup 20 --m 1024 > $O/prof_m1024.json 2> $O/prof_m1024.err || exit 1
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_gaps.py $f --markers > $O/gaps_m1024.txt || exit 1
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_m1024.csv \;
python3 - $O <<'PY' | tee -a $O/status.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*.json")):
    t = [x for x in open(f) if x.startswith('{"')]
    if not t: continue
    d = json.loads(t[-1]); r = d["roofline"]
    print(os.path.basename(f), "%.1f it/s ax %.1f atr %.1f syncs/it %.3f" % (d["value"], r["avg_launch_us"], r["atr_avg_launch_us"], d["work"]["syncs_per_iter"]))
PY
cat $O/gaps_m1024.txt >> $O/status.txt
echo done >> $O/status.txt
