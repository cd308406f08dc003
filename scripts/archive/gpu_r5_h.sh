#!/bin/bash
# Round 5 step H: the bitmap gather's 16-B row form (GLX_GATHER_BM=U,SEGW,1): kernel tests and
# trajectory bit-identity, then NS ProxGD A/B (200-step windows + whole solves).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_h; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "rows or flagged or bitmap or gather_waves" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 8,256,0 8,256,1 16,256,1 16,128,1; do
    GLX_GATHER_BM=$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_$v.$r.json 2> $O/ns_$v.$r.err || { tail -20 $O/ns_$v.$r.err; exit 1; }
    echo "bm=$v"; python3 scripts/r5_summ.py $O/ns_$v.$r.json
  done
done
