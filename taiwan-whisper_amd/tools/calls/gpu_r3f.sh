#!/bin/bash
# fp16 persistent-GEMM fix: GPU suite, then c4 / c5 (fp16) and c3 lines, and a c4 kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/bench_c4.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c4.log | cut -c1-250
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c5.log | cut -c1-250
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c3.log | cut -c1-250
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_fp16 -o run -- python3 $R/bench.py --config c4 --new-tokens 32 > $R/gpurun_out/prof_c4_fp16.log 2>&1 || exit $?
echo "trace done"
exit $rc
