#!/bin/bash
# Round 2: PMC HBM traffic (FETCH_SIZE and WRITE_SIZE passes, each its own run) of the NS
# ProxGD line and the 1024 / 2048-row comm shards with the current kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_pmc; rm -rf $O; mkdir -p $O
cp profiles/pmc_traffic.json $O/pmc_traffic.json
pass() {  # name key args...
  name=$1; key=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${name}_fetch -o run -- python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 "$@" > $O/${name}_fetch.json 2> $O/${name}_fetch.err || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${name}_write -o run -- python3 bench.py --no-cpu-baseline --steps 30 --warmup 5 "$@" > $O/${name}_write.json 2> $O/${name}_write.err || exit 1
  python3 scripts/pmc_traffic.py --fetch $O/${name}_fetch --write $O/${name}_write --key $key --out $O/pmc_traffic.json > $O/${name}_summary.json || exit 1
}
pass ns gl_ProxGD_primal_f64_8192x16384x32_g1_sc
pass s1024 gl_ProxGD_primal_f64_1024x16384x32_g1 --m 1024 --force-comm
pass s2048 gl_ProxGD_primal_f64_2048x16384x32_g1 --m 2048 --force-comm
echo done
