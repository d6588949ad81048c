#!/bin/bash
# Decode-step GEMV cost by batch rows: per-launch chains at 1 / 4 / 8 rows, and a kernel trace of the batch-8 step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for r in 1 4 8; do
  timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_step.py 20 1 --rows=$r > gpurun_out/r6f_rows$r.log 2>&1 || exit 1
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b8 -o run -- python3 $R/taiwan-whisper_amd/tools/bench_step.py 10 8 --step-only > $R/gpurun_out/r6f_prof_b8.log 2>&1 || exit 1
cd $R
python3 taiwan-whisper_amd/tools/trace_by_grid.py gpurun_out/prof_b8 > gpurun_out/r6f_step_b8_by_grid.txt
rm -rf gpurun_out/prof_b8
