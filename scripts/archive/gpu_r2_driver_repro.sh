#!/bin/bash
# Round 2: reproduce the driver's exact bench command and trace it.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_repro; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 200 $D > $O/driver_a.json 2> $O/driver_a.err || exit 1
timeout -k 10 200 $D --no-cpu-baseline > $O/driver_b.json 2> $O/driver_b.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_driver -o run -- $D --no-cpu-baseline > $O/driver_prof.json 2> $O/driver_prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_long -o run -- python3 bench.py --steps 400 --warmup 5 --no-cpu-baseline > $O/long_prof.json 2> $O/long_prof.err || exit 1
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/long.json 2> $O/long.err || exit 1
echo done
