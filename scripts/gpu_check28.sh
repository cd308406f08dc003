#!/bin/bash
# Ablation of the 8-wave LDS A@X tile inside the solver loop (timing only: ABL != 0 is wrong).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r28; mkdir -p $O
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 10"
for abl in 0 1 2 3 0; do
  GLX_AXL_ABL=$abl $B > $O/abl_$abl.json 2>> $O/err.log; rc=$?; echo "abl_$abl rc=$rc" >> $O/status.txt
  [ $rc -eq 0 ] || exit 1
  python -c "
import json; d=json.load(open('$O/abl_$abl.json')); r=d['roofline']; print('abl $abl', 'ax %.1f us %.1f TF' % (r['avg_launch_us'], r['mfma_tflops']), 'launches', r['launches'])"
done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $O/pmc.err; echo "pmc rc=$?" >> $O/status.txt
python - <<'PY'
import csv, collections
per=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open('gpurun_out/r28/pmc/run_counter_collection.csv')):
    per[r['Kernel_Name'][:50]][r['Counter_Name']].append(float(r['Counter_Value']))
for k in per:
    if 'k_ax_lds' not in k and 'atr_prox' not in k: continue
    c={n:sum(v)/len(v) for n,v in per[k].items()}; wc=c['SQ_WAVE_CYCLES']
    print(k, {n: '%.3g (%.3f)'%(v, v/wc) for n,v in sorted(c.items())})
PY
cat $O/status.txt | tr '\n' ' '
