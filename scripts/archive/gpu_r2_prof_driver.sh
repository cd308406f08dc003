#!/bin/bash
# Round 2: kernel trace + stats of the driver's exact bench command (with the default pre-warm).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2_prof_driver; rm -rf $O; mkdir -p $O
D="python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $D --no-cpu-baseline > $O/driver_prof.json 2> $O/driver_prof.err || exit 1
timeout -k 10 200 $D > $O/driver.json 2> $O/driver.err || exit 1
echo done
