#!/bin/bash
# Stall breakdown of the batched A@X tiles (old 21420 vs LDS 52224) from kbench launches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r15; mkdir -p $O
K="python scripts/kbench.py --ax 21820 --splits 0 --atr 102 --axb 21420,52224 --reps 10"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- $K > $O/k1.log 2> $O/pmc_sq.err; echo "pmc_sq rc=$?" >> $O/status.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM_RD --kernel-trace --output-format csv -d $O/pmc_sq2 -o run -- $K > $O/k2.log 2> $O/pmc_sq2.err; echo "pmc_sq2 rc=$?" >> $O/status.txt
cat $O/status.txt
