#!/bin/bash
# Round 5: publish-kernel cost with the deferred reductions on a rejection-heavy instance.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${OUT:-r5_probe}; rm -rf $O; mkdir -p $O
for meth in gl_ProxGD_primal gl_FProxGD_primal; do
  for d in 0 1; do
    GLX_DEFER_RED=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${meth}_d$d -o run -- python3 scripts/defer_probe.py $meth 2.5 >> $O/probe.jsonl 2> $O/${meth}_d$d.err || exit 1
  done
done
cat $O/probe.jsonl
for f in $(find $O -name "*.db" | sort); do python3 scripts/trace_db_summary.py $f; done > $O/summary.txt
grep -h "==\|publish\|finalize\|k_prox_pgd\|k_fista_trial\|atr_" $O/summary.txt | cut -c1-150
