#!/bin/bash
# c5 (long-form) line on the default workload, then a kernel trace of a 120 s recording (greedy windows: the
# per-decode-step launch structure) summarised per (kernel, grid).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python3 -u bench.py --config c5 > gpurun_out/r5_c5.log 2>&1 || exit 1
tail -1 gpurun_out/r5_c5.log | cut -c1-600
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5 -o run -- python3 $R/bench.py --config c5 --seconds 120 --longform-kwargs none > $R/gpurun_out/prof_c5.log 2>&1 || exit 1
cd $R
python3 taiwan-whisper_amd/tools/trace_by_grid.py gpurun_out/prof_c5 > gpurun_out/prof_c5_by_grid.txt
cp gpurun_out/prof_c5/run_kernel_stats.csv gpurun_out/prof_c5_kernel_stats.csv
rm -rf gpurun_out/prof_c5          # the raw trace is hundreds of MB (gpurun copies back <= 64 MiB)
head -40 gpurun_out/prof_c5_by_grid.txt
