#!/bin/bash
# Round 4 experiment 10: f32 two-source LDS-DMA tile (82478, one 16-row tile per wave) for C3's
# dense [xc | y_next] batch: kernel numerics, then interleaved 200-step C3 windows against the
# kind-5 tile 52324.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp10; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "82478" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 52324 82478; do
    GLX_AXB_VARIANT=$v timeout -k 10 300 python3 bench.py --method gl_FProxGD_primal --dtype f32 --steps 200 --warmup 20 --no-cpu-baseline > $O/c3_$v.$r.json 2> $O/c3_$v.$r.err || { tail -20 $O/c3_$v.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); r=d['roofline']; w=d.get('whole_solve') or {}; print(sys.argv[1], '%.1f it/s' % d['value'], 'ax %.1f atr %.1f' % (r['avg_launch_us'], r.get('atr_avg_launch_us') or 0), 'whole', w.get('iters_per_s'), w.get('fval'))" $O/c3_$v.$r.json
  done
done
