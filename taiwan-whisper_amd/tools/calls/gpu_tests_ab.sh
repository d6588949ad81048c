#!/bin/bash
# GPU test suite (no -x), then the default bench and an env A/B of it; each GPU step time-limited, the
# first timeout / abort / segfault ends the script.  usage: gpu_tests_ab.sh "ENV_B" [bench args]
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -30
tail -22 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
envb=${1:-TW_NOTHING=1}; shift
timeout -k 10 280 python -u bench.py "$@" > gpurun_out/bench_a.log 2>&1 || exit $?
tail -1 gpurun_out/bench_a.log
env $envb timeout -k 10 280 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/bench_b.log 2>&1 || exit $?
tail -1 gpurun_out/bench_b.log
exit $rc
