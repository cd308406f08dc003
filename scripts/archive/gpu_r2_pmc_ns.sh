#!/bin/bash
# Round 2: PMC traffic of the NS ProxGD line without the pre-warm session, so the per-launch
# average covers the same iterations as the bench's timed window (the gather's bytes grow with
# the number of thresholded rows, which rises over a solve).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_pmc_ns; rm -rf $O; mkdir -p $O
cp profiles/pmc_traffic.json $O/pmc_traffic.json
A="--no-cpu-baseline --steps 20 --warmup 5 --prewarm-s 0"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python3 bench.py $A > $O/fetch.json 2> $O/fetch.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python3 bench.py $A > $O/write.json 2> $O/write.err || exit 1
python3 scripts/pmc_traffic.py --fetch $O/fetch --write $O/write --key gl_ProxGD_primal_f64_8192x16384x32_g1_sc --out $O/pmc_traffic.json > $O/ns_summary.json || exit 1
echo done
