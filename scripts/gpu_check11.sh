#!/bin/bash
# MFMA ceiling microbench + new-roofline bench + stall/L2 counters on the dominant kernels.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r11; mkdir -p $O
timeout -k 10 120 scripts/mfma_peak > $O/mfma_peak.jsonl 2> $O/mfma_peak.err; echo "mfma_peak rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > $O/b_pgd.json 2> $O/bench.err; echo "b_pgd rc=$?" >> $O/status.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --warmup 20 --method gl_FProxGD_primal --dtype f32 > $O/b_fpgd32.json 2>> $O/bench.err; echo "b_fpgd32 rc=$?" >> $O/status.txt
P="python bench.py --steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- $P > /dev/null 2> $O/pmc_sq.err; echo "pmc_sq rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/pmc_tcc -o run -- $P > /dev/null 2> $O/pmc_tcc.err; echo "pmc_tcc rc=$?" >> $O/status.txt
cat $O/mfma_peak.jsonl
for f in $O/b_pgd.json $O/b_fpgd32.json; do python -c "
import json; d=json.load(open('$f')); print(d['value'], json.dumps(d['roofline']))"; done
cat $O/status.txt
