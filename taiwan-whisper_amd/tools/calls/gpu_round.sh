#!/bin/bash
# Runs the GPU test suite (no -x: report every failure) then the default bench; each GPU step
# time-limited.  Usage: gpu_round.sh [pytest selection...]
mkdir -p gpurun_out
sel=${@:-tests}
timeout -k 10 1000 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/pytest_gpu.log | tail -120
tail -3 gpurun_out/pytest_gpu.log
# a timeout / abort / segfault: nothing more on the GPU in this call
case $rc in 124|134|137|139) exit $rc;; esac
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
rc2=$?; tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
exit $rc2
