#!/bin/bash
# Split-K dW products on the 256x256 tile where the cost model prefers it: GEMM / training tests, then same-box
# A/B of c2 and c3 with the 256 option off (TW_SK256_R=0) and on (default R = 1.4).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distill_gpu.py tests/test_fp16_train_gpu.py tests/test_fp32_gpu.py -q -x --timeout 600 --timeout-method thread > gpurun_out/r6al_tests.log 2>&1 || { tail -30 gpurun_out/r6al_tests.log; exit 1; }
tail -2 gpurun_out/r6al_tests.log
for cfg in c2 c3; do
  for i in 1 2; do
    for r in 0 1.4; do
      echo "== $cfg R=$r run $i"
      TW_SK256_R=$r timeout -k 10 400 python -u bench.py --config $cfg --no-cpu-baseline --no-teacher-fwd > gpurun_out/r6al_b.log 2>&1 || { tail -20 gpurun_out/r6al_b.log; exit 1; }
      tail -1 gpurun_out/r6al_b.log | cut -c1-140
    done
  done
done 2>&1 | tee gpurun_out/r6al_ab.log
