#!/bin/bash
# Persistent decoder-step kernel: bit-identity tests first (stop on failure), the GPU suite, then c5 and c3 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BASE=$R/taiwan-whisper_amd/ab/libtw_hip_base.so
timeout -k 10 300 python -u -m pytest tests/test_decode_step_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ds_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/ds_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
echo "== c5 mega"; timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/c5_mega.log 2>&1 || exit $?; tail -1 gpurun_out/c5_mega.log
echo "== c5 per-launch"; TW_DECODE_MEGA=0 timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/c5_base.log 2>&1 || exit $?; tail -1 gpurun_out/c5_base.log
echo "== c3 base"; TW_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
echo "== c3 new"; timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
exit $rc
