#!/bin/bash
# Round-end evidence on a 1-GPU box (run from the repo root through gpurun):
#   1. FETCH_SIZE and WRITE_SIZE passes over a short bench run (separate --pmc runs, kernel trace off)
#      -> profiles/pmc_latest.json via pmc_summary.py (gfx950 corrections there)
#   2. kernel-trace + stats of the same bench command -> gpurun_out/prof/run_kernel_stats.csv
#   3. the default bench line (with the CPU baseline) -> gpurun_out/bench.log
# Every GPU step has its own time limit; the first failure ends the script.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-latest}
export TMPDIR=/tmp
OUT=$R/gpurun_out
mkdir -p $OUT
BENCH="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $BENCH > $OUT/pmc_fetch.log 2>&1
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $BENCH > $OUT/pmc_write.log 2>&1
echo "write pass done"
python3 $R/taiwan-whisper_amd/tools/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_$TAG.json $TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "trace pass done"
cd $R
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1
echo "bench done"
tail -1 $OUT/bench.log
