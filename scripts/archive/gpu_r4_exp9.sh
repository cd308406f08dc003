#!/bin/bash
# Round 4 experiment 9: row-kernel grid cap (GLX_ROW_BLOCKS), second sweep with repetitions:
# the 1024-row comm-path model (ProxGD, FProxGD) and NS ProxGD / FProxGD 200-step windows.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4_exp9; rm -rf $O; mkdir -p $O
one() {   # tag, env value, bench args
  local tag=$1 rb=$2; shift 2
  GLX_ROW_BLOCKS=$rb timeout -k 10 200 python3 bench.py "$@" --no-cpu-baseline --no-whole-solve > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], '%.1f it/s' % d['value'])" $O/$tag.json $tag
}
for r in 1 2; do
  for rb in 0 768 512 384; do
    one pro_${rb}_$r $rb --m 1024 --force-comm --steps 400 --warmup 40 || exit 1
    one fpr_${rb}_$r $rb --method gl_FProxGD_primal --m 1024 --force-comm --steps 400 --warmup 40 || exit 1
  done
  for rb in 0 512; do
    one ns_${rb}_$r $rb --steps 200 --warmup 20 || exit 1
    one nsf_${rb}_$r $rb --method gl_FProxGD_primal --steps 200 --warmup 20 || exit 1
  done
done
