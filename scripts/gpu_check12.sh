#!/bin/bash
# LDS-staged A@X (kind 5): correctness, then batched/single sweeps against the current tiles.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r12; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > $O/pytest_kernels.log 2>&1; rc=$?; echo "kernels rc=$rc" >> $O/status.txt
tail -5 $O/pytest_kernels.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python scripts/kbench.py --ax 21820,52224,54214,52228 --splits 0 --atr 102 --axb 21420,52224,52324,52228,54224,52214,54214 --axb3 1220,52224,52214 --reps 20 > $O/kb_f64.jsonl 2> $O/kb_f64.err; echo "kb_f64 rc=$?" >> $O/status.txt
timeout -k 10 400 python scripts/kbench.py --dtype f32 --ax 21410,52224,54214,52228 --splits 0 --atr 1102 --axb 21410,52224,52324,52228,54224,52214,54214 --reps 20 > $O/kb_f32.jsonl 2> $O/kb_f32.err; echo "kb_f32 rc=$?" >> $O/status.txt
timeout -k 10 400 python scripts/kbench.py --ax 52224 --splits 4,8,16,32 --atr 102 --axb 52224,52228,52214 --reps 20 > $O/kb_f64_split.jsonl 2> $O/kb_f64s.err; echo "kb_f64s rc=$?" >> $O/status.txt
cat $O/status.txt
