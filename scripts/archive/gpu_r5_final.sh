#!/bin/bash
# Round 5 evidence (OUT=r5_final at the end of the round): the driver's bench command under a rocprofv3 kernel trace (stats); PMC HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes, corrected in scripts/pmc_traffic.py) of NS ProxGD,
# NS FProxGD and C3 merged into profiles/pmc_traffic.json under the bench's keys; a kernel trace
# of the 8-GPU shard model (1024 rows, --force-comm) with the split-candidate trial.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_final}; rm -rf $O; mkdir -p $O
cp profiles/pmc_traffic.json $O/pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || { tail -20 $O/drv.err; exit 1; }
python3 scripts/r5_summ.py $O/drv.json
python3 - $O/drv/run_kernel_stats.csv <<'PY'
import csv, sys
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:8]:
    print("%-70s calls %5s avg %7.1f us" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
pmc() {   # tag, bench args
  local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${tag}_$c -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve "$@" > $O/${tag}_$c.json 2> $O/${tag}_$c.err || { tail -5 $O/${tag}_$c.err; return 1; }
  done
  local key=$(python3 -c "import json,sys; print(json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])['roofline']['pmc_key'])" $O/${tag}_FETCH_SIZE.json)
  python3 scripts/pmc_traffic.py --fetch $O/${tag}_FETCH_SIZE --write $O/${tag}_WRITE_SIZE --key "$key" --out $O/pmc_traffic.json --tag "round 5" > $O/${tag}_summary.json || return 1
  echo "$tag $key"; head -c 900 $O/${tag}_summary.json; echo
}
pmc ns || exit 1
pmc fi --method gl_FProxGD_primal || exit 1
pmc c3 --method gl_FProxGD_primal --dtype f32 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard -o run -- python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/shard.json 2> $O/shard.err || { tail -20 $O/shard.err; exit 1; }
python3 scripts/r5_summ.py $O/shard.json
python3 - $O/shard/run_kernel_stats.csv <<'PY'
import csv, sys
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:12]:
    print("%-70s calls %5s avg %7.1f us" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
export GLX_SHARD_MODEL=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/shard_rows -o run -- python3 bench.py --m 1024 --force-comm --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/shard_rows.json 2> $O/shard_rows.err || { tail -20 $O/shard_rows.err; exit 1; }
unset GLX_SHARD_MODEL
python3 scripts/r5_summ.py $O/shard_rows.json
python3 - $O/shard_rows/run_kernel_stats.csv <<'PY'
import csv, sys
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:12]:
    print("%-70s calls %5s avg %7.1f us" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
echo done
