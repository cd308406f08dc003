#!/bin/bash
# Round 5: kernel traces of C2 and NS (200-step windows) with the deferred reductions off / on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_c2trace}; rm -rf $O; mkdir -p $O
for d in 0 1; do
  export GLX_DEFER_RED=$d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_d$d -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve --m 4096 --n 8192 --l 16 > $O/c2_d$d.json 2> $O/c2_d$d.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ns_d$d -o run -- python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --no-whole-solve > $O/ns_d$d.json 2> $O/ns_d$d.err || exit 1
done
for f in $(find $O -name "*.db" | sort); do python3 scripts/trace_db_summary.py $f; done > $O/summary.txt
python3 scripts/r5_summ.py $O/c2_d0.json $O/c2_d1.json $O/ns_d0.json $O/ns_d1.json >> $O/summary.txt
echo done >> $O/summary.txt
