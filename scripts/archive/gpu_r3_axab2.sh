#!/bin/bash
# Round 3: LDS-DMA A@X tile variants (hoisted LDS reads, 16-wave blocks) against kind 5.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_axab2; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "residual" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ab() {  # name args...
  name=$1; shift
  mkdir -p $O/$name
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- python3 scripts/ax_ab.py --order $O/$name/order.json "$@" > $O/$name.log 2>&1 || { echo "ab $name failed"; tail -20 $O/$name.log; exit 1; }
  python3 scripts/ax_ab.py --summarize $O/$name > $O/$name.summary.jsonl || exit 1
  echo "== $name"; cat $O/$name.summary.jsonl
}
ab ns1 --codes 51328,92278,92268,93178,94178,94168 --rounds 5
ab ns2 --nsrc 2 --codes 52228,92278,93178,94178 --rounds 4
ab c2 --m 4096 --n 8192 --l 16 --nsrc 2 --codes 52228,93168,92268,94168 --rounds 4
ab s1024 --m 1024 --nsrc 2 --codes 51328,52228,92268,94168,93168 --rounds 4
ab s2048 --m 2048 --nsrc 2 --codes 51328,52228,92268,94168,93168 --rounds 4
ab c5s --m 16384 --nsrc 1 --codes 51328,92278,94178 --rounds 3
echo done
