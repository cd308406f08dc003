#!/bin/bash
# Round 5 step C: the bitmap gather (k_at_gather_bm, the trial kernels' column bitmaps) — kernel
# tests, split / whole-solve / device-control / sharded parity; the e / e_c distribution over whole
# NS solves; A/B of the three A e forms (GLX_GATHER=bm / lists / rows) on NS ProxGD and FProxGD;
# the driver's bench command with the reference-instance fields.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5_c; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rows.log 2>&1 || { tail -30 $O/pytest_rows.log; exit 1; }
tail -1 $O/pytest_rows.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ns_golden.py tests/test_gpu_dc.py tests/test_gpu_fused.py tests/test_gpu_dist.py tests/test_gpu_dc_dist.py -x -q --timeout 300 --timeout-method thread -k "split or full_size or north_star or dc or fused or world or folded" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 scripts/ec_distribution.py > $O/ec.jsonl 2> $O/ec.err || { tail -20 $O/ec.err; exit 1; }
cat $O/ec.jsonl
for r in 1 2; do
  for fin in 0 1; do
    GLX_AX_FIN=$fin timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_fin$fin.$r.json 2> $O/ns_fin$fin.$r.err || { tail -20 $O/ns_fin$fin.$r.err; exit 1; }
    echo "fin=$fin"; python3 scripts/r5_summ.py $O/ns_fin$fin.$r.json
  done
done
for r in 1 2; do
  for g in lists bm rows; do
    GLX_GATHER=$g timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/ns_$g.$r.json 2> $O/ns_$g.$r.err || { tail -20 $O/ns_$g.$r.err; exit 1; }
    python3 scripts/r5_summ.py $O/ns_$g.$r.json
    GLX_GATHER=$g timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --steps 200 --warmup 20 --no-cpu-baseline > $O/fi_$g.$r.json 2> $O/fi_$g.$r.err || { tail -20 $O/fi_$g.$r.err; exit 1; }
    python3 scripts/r5_summ.py $O/fi_$g.$r.json
  done
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err || { tail -20 $O/drv.err; exit 1; }
python3 scripts/r5_summ.py $O/drv.json
python3 -c "import json; d=json.loads([x for x in open('$O/drv.json') if x.startswith('{')][-1]); print(json.dumps(d['cpu_baseline'])); print(d['data']); print(json.dumps(d['whole_solve']['vs_reference'])); print(d['roofline']['session_plan'])"
