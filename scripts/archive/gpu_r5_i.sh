#!/bin/bash
# Round 5 step I: the 32-column A^T R panel (WL 3) — kernel and fused-trial tests, C2's whole-solve
# golden, then C2 A/B against the 2-split 64-column form (GLX_ATR_NARROW=0).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_i; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fused.py tests/test_gpu_ns_golden.py -x -q --timeout 300 --timeout-method thread -k "atr_codes or narrow or baseline_configs or fused" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for nw in 0 1; do
    GLX_ATR_NARROW=$nw timeout -k 10 300 python3 bench.py --m 4096 --n 8192 --l 16 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2_$nw.$r.json 2> $O/c2_$nw.$r.err || { tail -20 $O/c2_$nw.$r.err; exit 1; }
    echo "narrow=$nw"; python3 scripts/r5_summ.py $O/c2_$nw.$r.json
  done
done
