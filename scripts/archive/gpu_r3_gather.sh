#!/bin/bash
# Round 3: the gather with in-workgroup column lists (no side stream): split-candidate / FISTA /
# device-control parity, then the driver's command, 200-step windows and its kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r3_gather2}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_dc_dist.py tests/test_gpu_parity.py tests/test_gpu_dc.py tests/test_gpu_fused.py tests/test_gpu_dist.py -x -q --timeout 150 --timeout-method thread -k "split or gather or fista or full_size or FProx or world3" > $O/pytest_split.log 2>&1; rc=$?
echo "split tests rc=$rc" >> $O/status.txt; tail -3 $O/pytest_split.log
[ $rc -eq 0 ] || exit 1
D="python3 bench.py --gpus 1 --no-cpu-baseline"
for r in 1 2; do
timeout -k 10 300 $D --steps 20 --warmup 5 > $O/driver_r$r.json 2> $O/driver_r$r.err || exit 1
timeout -k 10 300 $D --steps 200 --warmup 20 > $O/b200_r$r.json 2> $O/b200_r$r.err || exit 1
timeout -k 10 300 $D --steps 200 --warmup 20 --method gl_FProxGD_primal > $O/fista_r$r.json 2> $O/fista_r$r.err || exit 1
timeout -k 10 200 python3 scripts/full_solve.py > $O/ns_full_r$r.json 2> $O/ns_full_r$r.err || exit 1
timeout -k 10 200 python3 scripts/full_solve.py --method gl_FProxGD_primal > $O/nsf_full_r$r.json 2> $O/nsf_full_r$r.err || exit 1
done
python3 - $O <<'PY' | tee -a $O/status.txt
import json, sys, glob, os
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*.json")):
    t = open(f).read().strip().splitlines()[-1]
    d = json.loads(t)
    if "roofline" in d:
        r = d["roofline"]
        print(os.path.basename(f), "%.1f it/s ax %.1f atr %.1f ga %s pair4 %.3f" % (d["value"], r["avg_launch_us"], r["atr_avg_launch_us"], r.get("gather_avg_launch_us"), r["pair4_frac"] or 0))
    else:
        print(os.path.basename(f), "k %d %.1f it/s fval %.10g" % (d["k"], d["its"], d["fval"]))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/prof_agree.py --trace $O/trace --bench $O/prof.json --out $O/agree.json > /dev/null || exit 1
echo done >> $O/status.txt
