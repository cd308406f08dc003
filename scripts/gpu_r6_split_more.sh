#!/bin/bash
# Round 6: the fused row-sharded derive at ragged / three-rank / eight-rank split-candidate shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r6_split_more}; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dist.py \
  -k "row_sharded_split_candidate" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -6 $O/pytest.log
