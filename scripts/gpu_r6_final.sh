#!/bin/bash
# Round 6 evidence (OUT=r6_final): the driver's bench command under a rocprofv3 kernel trace
# (stats); PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes, corrected in scripts/pmc_traffic.py) of
# NS ProxGD merged into profiles/pmc_traffic.json under the bench's key; kernel traces of the
# 8-GPU shard models (1024 rows, --force-comm --shard-model 8) of ProxGD and FProxGD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_final}; rm -rf $O; mkdir -p $O
cp profiles/pmc_traffic.json $O/pmc_traffic.json
stats() {
python3 - $1 <<'PY'
import csv, sys
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:10]:
    print("%-70s calls %5s avg %7.1f us" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || { tail -20 $O/drv.err; exit 1; }
python3 scripts/bench_summary.py $O/drv.json
stats $O/drv/run_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/ns_$c -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/ns_$c.json 2> $O/ns_$c.err || { tail -5 $O/ns_$c.err; exit 1; }
done
key=$(python3 -c "import json,sys; print(json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])['roofline']['pmc_key'])" $O/ns_FETCH_SIZE.json)
python3 scripts/pmc_traffic.py --fetch $O/ns_FETCH_SIZE --write $O/ns_WRITE_SIZE --key "$key" --out $O/pmc_traffic.json --tag "round 6" > $O/ns_summary.json || exit 1
echo "ns $key"; head -c 900 $O/ns_summary.json; echo
for meth in gl_ProxGD_primal gl_FProxGD_primal; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard_$meth -o run -- python3 bench.py --method $meth --m 1024 --force-comm --shard-model 8 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/shard_$meth.json 2> $O/shard_$meth.err || { tail -20 $O/shard_$meth.err; exit 1; }
  python3 scripts/bench_summary.py $O/shard_$meth.json
  stats $O/shard_$meth/run_kernel_stats.csv
done
echo done
