#!/bin/bash
# Round 4, call A: GPU suite on the working tree, then a same-box A/B of the working-tree library against
# ab/libtw_hip_base.so (own GEMM shapes, then the c3 bench, alternating).  Every GPU step has its own time limit;
# the steps are chained so a failure ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4a_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r4a_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/r4a_gpu_tests.txt
for i in 1 2; do
  echo "== gemm base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
  echo "== gemm cand $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
done
for i in 1 2; do
  echo "== bench base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-420 || exit 1
  echo "== bench cand $i"; timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-420 || exit 1
done
