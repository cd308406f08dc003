#!/bin/bash
# Round 5 step A: the MFMA row form of the split-candidate A e (k_at_rows) — kernel tests, the
# split-candidate / whole-solve / device-control parity suites, then an A/B against the VALU
# column-list gather (GLX_GATHER=valu) on NS ProxGD and FProxGD (200-step windows + whole solves),
# and the K-split count (GLX_ATROWS_S 2 / 4 / 8) on NS FProxGD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_a; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rows.log 2>&1 || { tail -30 $O/pytest_rows.log; exit 1; }
tail -1 $O/pytest_rows.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ns_golden.py tests/test_gpu_dc.py -x -q --timeout 300 --timeout-method thread -k "split or full_size or north_star or dc" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
summ() { python3 scripts/r5_summ.py "$@"; }
for r in 1 2; do
  for g in valu rows; do
    GLX_GATHER=$g timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_$g.$r.json 2> $O/ns_$g.$r.err || { tail -20 $O/ns_$g.$r.err; exit 1; }
    summ $O/ns_$g.$r.json
    GLX_GATHER=$g timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fi_$g.$r.json 2> $O/fi_$g.$r.err || { tail -20 $O/fi_$g.$r.err; exit 1; }
    summ $O/fi_$g.$r.json
  done
done
for s in 2 8; do
  GLX_ATROWS_S=$s timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fi_s$s.json 2> $O/fi_s$s.err || { tail -20 $O/fi_s$s.err; exit 1; }
  echo "S=$s"; summ $O/fi_s$s.json
  GLX_ATROWS_S=$s timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_s$s.json 2> $O/ns_s$s.err || { tail -20 $O/ns_s$s.err; exit 1; }
  echo "S=$s"; summ $O/ns_s$s.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --method gl_FProxGD_primal --steps 20 --warmup 5 --no-cpu-baseline > $O/tr.json 2> $O/tr.err || { tail -20 $O/tr.err; exit 1; }
python3 - $O/tr/run_kernel_stats.csv <<'PY'
import csv, sys
for row in sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: -float(x["TotalDurationNs"]))[:10]:
    print("%-70s calls %5s avg %7.1f us" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3))
PY
