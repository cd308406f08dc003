#!/bin/bash
# Same-box interleaved A/B of bench arms, each under a rocprofv3 kernel trace (per-kernel window
# averages via scripts/trace_gaps.py) plus the bench line's it/s.
#   [WHOLE=1: keep the bench's whole-solve figure] OUT=name REPS=2 BENCH="--steps 200 --warmup 20" bash scripts/gpu_ab.sh 'arm1|dir|ENV=a ENV2=b' 'arm2|.|GLX_X=1' ...
# dir "." is this tree; another dir (e.g. abtree/r2) runs that tree's bench.py and libglx.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-ab}; rm -rf $O; mkdir -p $O
REPS=${REPS:-2}
B="--gpus 1 --no-cpu-baseline ${BENCH:---steps 200 --warmup 20}"
LAST=${LAST:-1000}
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    IFS='|' read -r name dir envs <<< "$spec"
    extra=""
    [ "$dir" = "." ] && [ -z "$WHOLE" ] && extra="--no-whole-solve"
    ( cd $dir && env GLX_AB=1 $envs timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t_$name -o run -- python3 bench.py $B $extra > $GRAFT_REPO_ROOT/$O/$name.$rep.json 2> $GRAFT_REPO_ROOT/$O/$name.$rep.err ) || { echo "arm $name failed"; tail -5 $O/$name.$rep.err; exit 1; }
    f=$(find $O/t_$name -name "*kernel_trace.csv" | head -1)
    v=$(python3 -c "import json,sys; d=json.loads(open('$O/$name.$rep.json').read().strip().splitlines()[-1]); w=d.get('whole_solve'); print('%.1f it/s' % d['value'] + (' whole %.1f it/s (k %d)' % (w['iters_per_s'], w['k']) if w else ''))")
    echo "== $name rep $rep: $v" >> $O/summary.txt
    python3 scripts/trace_gaps.py $f --last $LAST | head -7 >> $O/summary.txt
    rm -rf $O/t_$name
  done
done
echo done >> $O/summary.txt
