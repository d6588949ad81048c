#!/bin/bash
# c4 and c5 lines (fp16, the reference's dtype) on the end-of-round tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/bench_c4.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c4.log | cut -c1-200
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c5.log | cut -c1-200
