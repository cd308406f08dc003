# Round-1 evidence: rocprofv3 kernel stats + PMC traffic of the default bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/p1; mkdir -p $O
CMD="python bench.py --steps 50 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 python -m pytest tests/test_gpu_comm.py -m gpu -q > $O/pytest_comm.log 2>&1 ; echo "comm rc=$?" >> $O/status.txt
tail -3 $O/pytest_comm.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- $CMD > $O/bench_stats.json 2> $O/stats.err ; echo "stats rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o bench -- $CMD > $O/bench_fetch.json 2> $O/fetch.err ; echo "fetch rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/write -o bench -- $CMD > $O/bench_write.json 2> $O/write.err ; echo "write rc=$?" >> $O/status.txt
python scripts/pmc_traffic.py --fetch $O/fetch --write $O/write --key gl_ProxGD_primal_f64_8192x16384x32_g1 --out $O/pmc_traffic.json > $O/pmc.log 2>&1 ; echo "pmc rc=$?" >> $O/status.txt
cat $O/pmc.log | head -30
ls -R $O | head -40
cat $O/status.txt
