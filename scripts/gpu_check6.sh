set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_comm.py -m gpu -q --maxfail=5 > $O/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> $O/status.txt
tail -2 $O/pytest_kernels.log
for X in 1 0; do
GLX_AX_XCD=$X timeout -k 10 300 python scripts/kbench.py --ax 2820,1820,2420 --atr 102 --splits 0,4,8,16 --axb 1420,2420,1220 --axb3 1220 > $O/kbench_f64_x$X.jsonl 2>> $O/kbench.err ; echo "kbench x$X rc=$?" >> $O/status.txt
done
GLX_AX_XCD=1 timeout -k 10 300 python scripts/kbench.py --dtype f32 --ax 2820,1820 --atr 1102 --splits 0,4,8,16 --axb 1430,1420,2430 > $O/kbench_f32_x1.jsonl 2>> $O/kbench.err ; echo "kbench32 rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/b_pgd.json 2> $O/bench.err ; echo "b_pgd rc=$?" >> $O/status.txt
python -c "import json; d=json.load(open('$O/b_pgd.json')); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['atr_avg_launch_us'])"
cat $O/status.txt
