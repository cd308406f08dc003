set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q --maxfail=5 > $O/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> $O/status.txt
tail -3 $O/pytest_kernels.log
timeout -k 10 300 python scripts/kbench.py --ax 1420,2420,2421,1820,2820 --atr 102,1102 --splits 0,4,8 --axb 2420,1420,1430,2430,2220,2230,1220 --axb3 2220,1220,2230 > $O/kbench_f64.jsonl 2> $O/kbench.err ; echo "kbench rc=$?" >> $O/status.txt
timeout -k 10 300 python scripts/kbench.py --dtype f32 --ax 1420,2420,2421,1820,2820 --atr 102,1102,101 --splits 0,4,8 --axb 2420,1420,1430,2430,2220,2230,1220 > $O/kbench_f32.jsonl 2>> $O/kbench.err ; echo "kbench32 rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/b_pgd.json 2> $O/bench.err ; echo "b_pgd rc=$?" >> $O/status.txt
python -c "import json; d=json.load(open('$O/b_pgd.json')); print(d['value'], d['work'])"
cat $O/status.txt
