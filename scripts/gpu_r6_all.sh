#!/bin/bash
# Round 6: the whole -m gpu suite (one pytest process), as the driver runs it at round end.
set -o pipefail
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread --maxfail=5 -m gpu tests \
  > $OUT/pytest_all.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $OUT/pytest_all.log
