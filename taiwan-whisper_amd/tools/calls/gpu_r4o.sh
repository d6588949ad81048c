#!/bin/bash
# Round 4, call O: where the c3 step's ~450 copyBuffer launches per step come from -- HIP API + memory-copy + kernel
# trace of a short bench run (no counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r4o
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --output-format csv -d $R/gpurun_out/r4o/tr -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $R/gpurun_out/r4o/tr.log 2>&1 || exit 1
cd $R
ls gpurun_out/r4o/tr
python3 - <<'PY'
import csv, collections, glob
d = "gpurun_out/r4o/tr"
for f in sorted(glob.glob(d + "/*.csv")):
    print(f)
api = glob.glob(d + "/*hip_api_trace.csv")
if api:
    c = collections.Counter(r["Function"] for r in csv.DictReader(open(api[0])))
    print("HIP API calls:", c.most_common(25))
mc = glob.glob(d + "/*memory_copy_trace.csv")
if mc:
    rows = list(csv.DictReader(open(mc[0])))
    print("memory copies:", len(rows), list(rows[0].keys()) if rows else None)
    c = collections.Counter((r.get("Direction"), r.get("Bytes", r.get("Size"))) for r in rows)
    print(c.most_common(25))
PY
