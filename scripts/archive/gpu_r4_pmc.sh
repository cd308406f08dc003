#!/bin/bash
# Round 4: PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# §HBM corrections in scripts/pmc_traffic.py) of the NS ProxGD driver command and C3 (fp32
# FProxGD, the f32 LDS-DMA tile), merged into profiles/pmc_traffic.json under the bench's keys.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_pmc; rm -rf $O; mkdir -p $O
cp profiles/pmc_traffic.json $O/pmc_traffic.json
pmc() {   # tag, bench args
  local tag=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${tag}_$c -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve "$@" > $O/${tag}_$c.json 2> $O/${tag}_$c.err || { tail -5 $O/${tag}_$c.err; return 1; }
  done
  local key=$(python3 -c "import json,sys; print(json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])['roofline']['pmc_key'])" $O/${tag}_FETCH_SIZE.json)
  python3 scripts/pmc_traffic.py --fetch $O/${tag}_FETCH_SIZE --write $O/${tag}_WRITE_SIZE --key "$key" --out $O/pmc_traffic.json --tag "round 4" > $O/${tag}_summary.json || return 1
  echo "$tag $key"; head -c 600 $O/${tag}_summary.json; echo
}
pmc ns || exit 1
pmc c3 --method gl_FProxGD_primal --dtype f32 || exit 1
