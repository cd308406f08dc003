#!/bin/bash
# Round 4, VERDICT round 3 item 1: why k_atr_prox runs 183-200 us in round-3 windows against
# 169-173 us in round 2. Same box, interleaved, each arm under a rocprofv3 kernel trace:
#   head   — this tree
#   noDMA  — this tree with GLX_AX_DMA=0 (round 2's kind-5 tile for the dense pass)
#   keep0  — this tree with both Infinity-Cache hand-offs off
#   r2     — the round-2 tree (abtree/r2: its bench.py + libglx built from commit 7803943)
#   atr8   — this tree with the eight-wave A^T R panel (GLX_ATR_VARIANT=1028; 1024: PF 4)
# then the clock each kernel runs at (GRBM_GUI_ACTIVE / trace duration, PMC pass) and amd-smi
# power samples while whole NS solves run back to back.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r4_diag}; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k "atr_codes or eight_wave" > $O/pytest_atr8.log 2>&1 || { echo "atr8 tests failed"; tail -30 $O/pytest_atr8.log; exit 1; }
tail -2 $O/pytest_atr8.log > $O/summary.txt
B="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
run_arm() {   # name, dir, extra env...
  local name=$1 dir=$2; shift 2
  local extra=""
  [ "$dir" = "." ] && extra="--no-whole-solve"
  ( cd $dir && env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t_$name -o run -- python3 bench.py $B $extra > $GRAFT_REPO_ROOT/$O/$name.json 2> $GRAFT_REPO_ROOT/$O/$name.err ) || { echo "arm $name failed"; tail -5 $O/$name.err; return 1; }
  f=$(find $O/t_$name -name "*kernel_trace.csv" | head -1)
  echo "== $name" >> $O/summary.txt
  python3 scripts/trace_gaps.py $f --last 1000 | head -8 >> $O/summary.txt
  rm -rf $O/t_$name
}
for rep in 1 2; do
  run_arm head . GLX_X=1 || exit 1
  run_arm noDMA . GLX_AX_DMA=0 || exit 1
  run_arm keep0 . GLX_AX_KEEP_MIB=0 GLX_ATR_KEEP_MIB=0 || exit 1
  run_arm r2 abtree/r2 GLX_X=1 || exit 1
  run_arm atr8 . GLX_ATR_VARIANT=1028 || exit 1
  run_arm atr8p4 . GLX_ATR_VARIANT=1024 || exit 1
done
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/pmc -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/pmc.json 2> $O/pmc.err || exit 1
timeout -k 10 120 python3 scripts/power_sample.py --seconds 12 --out $O/power.jsonl > $O/power.log 2>&1 || echo "power sampling failed" >> $O/summary.txt
echo done >> $O/summary.txt
