#!/bin/bash
# Round 3: the gfx clock each NS kernel runs at in the driver-form bench (GRBM_GUI_ACTIVE cycles
# per dispatch / its trace duration), one PMC pass with the kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3_clock; rm -rf $O; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/pmc -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-whole-solve > $O/bench.json 2> $O/bench.err || exit 1
python3 - $O <<'PY' | tee $O/status.txt
import csv, glob, sys, collections
O = sys.argv[1]
cc = glob.glob(O + "/pmc/**/*counter_collection.csv", recursive=True)
rows = []
for f in cc: rows += list(csv.DictReader(open(f)))
print("columns:", list(rows[0].keys()) if rows else None)
per = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    per[r["Kernel_Name"].split("(")[0][-40:]][r["Counter_Name"]].append((int(r.get("Dispatch_Id", 0) or 0), float(r["Counter_Value"])))
tr = glob.glob(O + "/pmc/**/*kernel_trace.csv", recursive=True)
dur = {}
for f in tr:
    for r in csv.DictReader(open(f)):
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, cs in per.items():
    g = cs.get("GRBM_GUI_ACTIVE", [])
    if len(g) < 5: continue
    ghz = [v / dur[d] for d, v in g if d in dur and dur[d] > 0]
    ghz.sort()
    print("%-42s n %4d  clock median %.2f GHz  p10 %.2f  p90 %.2f  avg dur %.1f us" % (k, len(ghz), ghz[len(ghz)//2], ghz[len(ghz)//10], ghz[9*len(ghz)//10], sum(dur[d] for d, v in g if d in dur)/max(1,len(g))/1e3))
PY
