#!/bin/bash
# Natural-layout LDS X staging: correctness, conflict counter, kernel sweep, end-to-end.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r16; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > $O/pytest_kernels.log 2>&1; rc=$?; echo "kernels rc=$rc" >> $O/status.txt
tail -2 $O/pytest_kernels.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python scripts/kbench.py --ax 21820,52224,52228,54214 --splits 0 --atr 102 --axb 21420,52224,52324,52228,54224,52214,54214 --axb3 1220,52224,52214 --reps 20 > $O/kb_f64.jsonl 2> $O/kb_f64.err; echo "kb_f64 rc=$?" >> $O/status.txt
timeout -k 10 400 python scripts/kbench.py --dtype f32 --ax 21410,52224,52228,52214 --splits 0 --atr 1102 --axb 21410,52224,52324,52228,54224,52214,54214 --reps 20 > $O/kb_f32.jsonl 2> $O/kb_f32.err; echo "kb_f32 rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python scripts/kbench.py --ax 21820 --splits 0 --atr 102 --axb 52224 --reps 10 > $O/k1.log 2> $O/pmc_sq.err; echo "pmc_sq rc=$?" >> $O/status.txt
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20"
for v in 21420 52224 54214; do GLX_AXB_VARIANT=$v $B > $O/b_pgd_$v.json 2>> $O/bench.err; echo "b_pgd_$v rc=$?" >> $O/status.txt; done
for v in 21410 52224 52214; do GLX_AXB_VARIANT=$v $B --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32_$v.json 2>> $O/bench.err; echo "b_fpgd32_$v rc=$?" >> $O/status.txt; done
for f in $O/b_*.json; do python -c "
import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['value'],1), 'ax %.1fus %.1fTF frac %.3f pair %.3f atr %.1fus' % (r['avg_launch_us'], r['mfma_tflops'], r['frac'], r['pair_frac'], r['atr_avg_launch_us']))"; done
cat $O/status.txt
