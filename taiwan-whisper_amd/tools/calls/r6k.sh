#!/bin/bash
# dW split-K for few-tile weight gradients + the dX-head tile threshold: GEMM / training tests, then c2 and c3 A/B.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_fp32_gpu.py tests/test_distill_gpu.py tests/test_fullsize_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/r6k_tests.log 2>&1 || { tail -30 gpurun_out/r6k_tests.log; exit 1; }
tail -2 gpurun_out/r6k_tests.log
REPS=2 T=400 bash taiwan-whisper_amd/tools/calls/ab.sh \
  "python -u bench.py --config c2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160" \
  "python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160" > gpurun_out/r6k_ab.log 2>&1
