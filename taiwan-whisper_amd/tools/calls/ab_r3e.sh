#!/bin/bash
# A/B of the working-tree library against ab/libtw_hip_base.so on the own GEMM shapes (no hipBLASLt) and the c3 step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
BASE=$R/taiwan-whisper_amd/ab/libtw_hip_base.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -20 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
for i in 1 2; do
  echo "== base $i"; TW_HIP_LIB=$BASE timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70
  echo "== new $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70
done
echo "== bench base"; TW_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1 | cut -c1-420
echo "== bench new"; timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1 | cut -c1-420
