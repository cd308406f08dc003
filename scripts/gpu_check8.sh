set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r8; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q --maxfail=5 > $O/pytest_kernels.log 2>&1 ; echo "kernels rc=$?" >> $O/status.txt
tail -2 $O/pytest_kernels.log
GLX_AX_XCD=0 timeout -k 10 300 python scripts/kbench.py --ax 2420,2820,21420,22420,21410,41220,41210,41410,21820 --atr 102 --splits 0,4,8 --axb 1420,21420,21410,41210 > $O/kb64.jsonl 2>> $O/kbench.err ; echo "kbench rc=$?" >> $O/status.txt
GLX_AX_XCD=0 timeout -k 10 300 python scripts/kbench.py --dtype f32 --ax 1820,21420,22420,21410,41220,41210 --atr 1102 --splits 0,4,8 --axb 1430,21420,21410,41210 > $O/kb32.jsonl 2>> $O/kbench.err ; echo "kbench32 rc=$?" >> $O/status.txt
cat $O/status.txt
