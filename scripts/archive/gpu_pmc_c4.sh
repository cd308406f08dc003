#!/bin/bash
# PMC HBM traffic of the one-pass l = 1 kernel (config C4), FETCH_SIZE and WRITE_SIZE passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_c4; rm -rf $O; mkdir -p $O
A="--no-cpu-baseline --method gl_SGD_primal --m 65536 --n 8192 --l 1 --steps 30 --warmup 5"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- python bench.py $A > $O/b_fetch.json 2> $O/fetch.err || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o run -- python bench.py $A > $O/b_write.json 2> $O/write.err || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
python scripts/pmc_traffic.py --fetch $O/fetch --write $O/write --key gl_SGD_primal_f64_65536x8192x1_g1 --out $O/pmc_traffic.json
