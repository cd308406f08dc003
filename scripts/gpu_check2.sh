set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/r2
O=gpurun_out/r2
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > $O/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> $O/status.txt
tail -3 $O/pytest_kernels.log
timeout -k 10 300 python scripts/kbench.py > $O/kbench_f64.jsonl 2> $O/kbench.err ; echo "kbench64 rc=$?" >> $O/status.txt
timeout -k 10 300 python scripts/kbench.py --dtype f32 > $O/kbench_f32.jsonl 2>> $O/kbench.err ; echo "kbench32 rc=$?" >> $O/status.txt
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=15 > $O/pytest_parity.log 2>&1 ; echo "parity rc=$?" >> $O/status.txt
tail -15 $O/pytest_parity.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_spin.json 2> $O/bench.err ; echo "bench rc=$?" >> $O/status.txt
GLX_READBACK=sync timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_sync.json 2>> $O/bench.err ; echo "bench sync rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --profile 0 > $O/bench_noprof.json 2>> $O/bench.err ; echo "bench noprof rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_prof.json 2> $O/prof.err ; echo "prof rc=$?" >> $O/status.txt
cat $O/bench_spin.json $O/bench_sync.json $O/bench_noprof.json | python -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['ms_per_step'], json.loads(l)['roofline']['achieved'], json.loads(l)['roofline']['atr_GBs']) for l in sys.stdin if l.strip()]"
cat $O/status.txt
