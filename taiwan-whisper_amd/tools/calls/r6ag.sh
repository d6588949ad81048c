#!/bin/bash
# Config 2: kernel trace of the step by (kernel, grid) on the final tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $R/gpurun_out/r6ag_prof_c2.log 2>&1 || exit 1
cd $R
python3 taiwan-whisper_amd/tools/trace_by_grid.py gpurun_out/prof_c2 > gpurun_out/r6ag_c2_by_grid.txt
cp gpurun_out/prof_c2/run_kernel_stats.csv gpurun_out/r6ag_c2_kernel_stats.csv
rm -rf gpurun_out/prof_c2
