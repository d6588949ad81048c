#!/bin/bash
# Final round-3 check of the committed tree: new fp16 GEMM tests, the whole GPU suite, smoke(), the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp16_gpu.py -m gpu -q -k "gemm" --timeout 200 --timeout-method thread > gpurun_out/f16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/f16_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.log 2>&1 || exit $?; tail -1 gpurun_out/bench_final.log | cut -c1-400
exit $rc
