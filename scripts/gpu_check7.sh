set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=gpurun_out/r7; mkdir -p $O
for N in 16384 16448 16320 17408; do
GLX_AX_XCD=0 timeout -k 10 200 python scripts/kbench.py --n $N --ax 2820,1820,2420 --atr 102 --splits 0,4 --axb 1420 > $O/kb_n$N.jsonl 2>> $O/kbench.err ; echo "kbench n$N rc=$?" >> $O/status.txt
done
cat $O/status.txt
