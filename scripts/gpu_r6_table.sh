#!/bin/bash
# Round 6 (closing table): BASELINE.md §3 at HEAD — every BASELINE config in driver form (20 timed /
# 5 warmup, with the CPU baseline and its same-sample GPU check), a 200-step window, and the
# bench's whole solve (checked against the reference's own run where one is committed); the
# row-sharded per-rank timing models (--force-comm --shard-model G) and C5's shard.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_table}; rm -rf $O; mkdir -p $O
run() {   # tag, bench args
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $O/${tag}_d.json 2> $O/${tag}_d.err || return 1
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline "$@" > $O/${tag}_w.json 2> $O/${tag}_w.err || return 1
  python3 - $O $tag <<'PY' | tee -a $O/status.txt
import json, sys
O, tag = sys.argv[1], sys.argv[2]
for s in ("d", "w"):
    d = json.loads([x for x in open("%s/%s_%s.json" % (O, tag, s)) if x.startswith("{")][-1])
    r = d["roofline"]; k = r.get("kernels", {}); w = d.get("whole_solve") or {}; v = w.get("vs_reference") or {}
    cb = d.get("cpu_baseline") or {}
    print(tag, s, "%.1f it/s" % d["value"], "ax %.1f atr %.1f ga %s" % ((k.get("ax") or {}).get("avg_launch_us") or 0,
          (k.get("atr") or {}).get("avg_launch_us") or 0, r.get("gather_avg_launch_us")),
          "pair4 %.3f frac %.3f" % (r.get("pair4_frac") or 0, r.get("frac") or 0),
          "whole k=%s %.1f it/s ref_ok=%s" % (w.get("k"), w.get("iters_per_s") or 0, v.get("within_bar")),
          "cpu %s same_sample %s" % (cb.get("value"), (cb.get("gpu_same_sample") or {}).get("f_hist_max_rel_diff")))
PY
}
run ns || exit 1
run nsf --method gl_FProxGD_primal || exit 1
run c2 --m 4096 --n 8192 --l 16 || exit 1
run c3 --method gl_FProxGD_primal --dtype f32 || exit 1
run c4 --method gl_SGD_primal --m 65536 --n 8192 --l 1 || exit 1
run c1 --m 512 --n 1024 --l 2 || exit 1
for pair in "1024 8" "2048 4" "4096 2"; do
  set -- $pair
  for meth in gl_ProxGD_primal gl_FProxGD_primal; do
    timeout -k 10 300 python3 bench.py --method $meth --m $1 --force-comm --shard-model $2 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/shard$1.$meth.json 2> $O/shard$1.$meth.err || exit 1
    echo -n "row-sharded model $1 (x$2) $meth: " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/shard$1.$meth.json | tee -a $O/status.txt
  done
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 10 --no-cpu-baseline --no-whole-solve --m 16384 --method gl_FProxGD_primal --force-comm > $O/c5shard_w.json 2> $O/c5shard_w.err || exit 1
echo -n "c5shard: " | tee -a $O/status.txt; python3 scripts/bench_summary.py $O/c5shard_w.json | tee -a $O/status.txt
echo done >> $O/status.txt
