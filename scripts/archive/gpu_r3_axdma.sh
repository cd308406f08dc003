#!/bin/bash
# Round 3: the LDS-DMA A@X tile (kind 8) — kernel numerics, then a kernel-trace sweep of the
# tile codes against the current kind-5 tiles at NS (one RHS), C2 (two RHS, l = 16) and the
# 1024 / 2048-row shards (two RHS).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_axdma; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_resgrad.py -x -q --timeout 120 --timeout-method thread -k "residual or resgrad" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
K="python3 scripts/kbench.py --splits 0 --reps 30 --no-ref --atr ''"
CODES=51328,52228,84208,84218,83208,83218,82408,82418,88108,88118,85208,85218,84204,84214
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ns -o run -- python3 scripts/kbench.py --splits 0 --reps 30 --no-ref --atr "" --ax $CODES > $O/ns.jsonl 2> $O/ns.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 scripts/kbench.py --m 4096 --n 8192 --l 16 --splits 0 --reps 30 --no-ref --atr "" --ax "" --axb 52228,84208,84218,83208,83218,82408,82418,88108,88118,85208,85218 > $O/c2.jsonl 2> $O/c2.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s1024 -o run -- python3 scripts/kbench.py --m 1024 --splits 0 --reps 30 --no-ref --atr "" --ax "" --axb 51328,52228,84208,84218,83208,83218,88108,88118,85208,85218 > $O/s1024.jsonl 2> $O/s1024.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s2048 -o run -- python3 scripts/kbench.py --m 2048 --splits 0 --reps 30 --no-ref --atr "" --ax "" --axb 51328,52228,84208,84218,83208,83218,88108,88118,85208,85218 > $O/s2048.jsonl 2> $O/s2048.err || exit 1
echo done
