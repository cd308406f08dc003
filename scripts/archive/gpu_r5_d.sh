#!/bin/bash
# Round 5 step D: the folded finalize with batched slab loads (GLX_AX_FIN A/B), FProxGD's
# row-form budget (GLX_SPLIT_NNZ 0.4 / 0.5 / 0.6), and the C3 summation-order band.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_d; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "folded or long_trajectory" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for fin in 0 1; do
    GLX_AX_FIN=$fin timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_fin$fin.$r.json 2> $O/ns_fin$fin.$r.err || { tail -20 $O/ns_fin$fin.$r.err; exit 1; }
    echo "fin=$fin"; python3 scripts/r5_summ.py $O/ns_fin$fin.$r.json
  done
done
for b in 0.4 0.5 0.6; do
  GLX_SPLIT_NNZ=$b timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 50 --warmup 10 --no-cpu-baseline > $O/fi_b$b.json 2> $O/fi_b$b.err || { tail -20 $O/fi_b$b.err; exit 1; }
  echo "budget=$b"; python3 scripts/r5_summ.py $O/fi_b$b.json
done
timeout -k 10 600 python3 scripts/c3_band.py > $O/c3_band.jsonl 2> $O/c3_band.err || { tail -20 $O/c3_band.err; exit 1; }
cat $O/c3_band.jsonl
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --m 4096 --n 8192 --l 16 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.$r.json 2> $O/c2.$r.err || { tail -20 $O/c2.$r.err; exit 1; }
  echo C2; python3 scripts/r5_summ.py $O/c2.$r.json
done
