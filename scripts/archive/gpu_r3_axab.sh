#!/bin/bash
# Round 3: interleaved A/B of the A@X tiles (kind 5 vs the LDS-DMA kind 8) with and without the
# rotated K walk (GLX_AX_ROT), kernel-trace timed, at NS (1 and 2 RHS), C2 (2 RHS, l = 16) and
# the 1024-row shard (2 RHS).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_axab; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "residual" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ab() {  # name args...
  name=$1; shift
  mkdir -p $O/$name
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o run -- python3 scripts/ax_ab.py --order $O/$name/order.json "$@" > $O/$name.log 2>&1 || { echo "ab $name failed"; tail -20 $O/$name.log; exit 1; }
  python3 scripts/ax_ab.py --summarize $O/$name > $O/$name.summary.jsonl || exit 1
  echo "== $name"; cat $O/$name.summary.jsonl
}
ab ns1 --codes 51328,83208,83218,84208,84218 --env GLX_AX_ROT=0,1
ab ns2 --nsrc 2 --codes 52228,83208,83218 --env GLX_AX_ROT=0,1
ab c2 --m 4096 --n 8192 --l 16 --nsrc 2 --codes 52228,84208,83208,82408 --env GLX_AX_ROT=0,1
ab s1024 --m 1024 --nsrc 2 --codes 51328,52228,83208 --env GLX_AX_ROT=0,1
echo done
