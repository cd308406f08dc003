#!/bin/bash
# Round 4 experiments 5: k_resgrad2 with ordered prologue loads / granules issued ahead of the
# tile prefetch / relaxed LDS counters (tests + C2 trace, lags 24 and 12, XCD-local and
# agent-scope); FProxGD whole-solve nnz-budget sweep (C3 f32 split + f32 DMA tile, NS f64).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp5; rm -rf $O; mkdir -p $O
LAGS="24 12" OUT=r4_exp5/rg2 bash scripts/gpu_r4_rg2x.sh > $O/rg2.txt 2>&1 || { cat $O/rg2.txt; exit 1; }
tail -1 $O/rg2/pytest.log; grep -h "resgrad2\|k_ax_dma\|k_atr" $O/rg2/summary.txt
timeout -k 10 500 python3 -u scripts/nnz_budget_sweep.py 0.35 0.5 0.7 > $O/nnz.jsonl 2> $O/nnz.err || { tail -20 $O/nnz.err; exit 1; }
cat $O/nnz.jsonl
