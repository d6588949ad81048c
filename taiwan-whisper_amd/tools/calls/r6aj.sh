#!/bin/bash
# dQ backward kernel on a 3-deep K/V ring: attention / training tests, then same-box A/B of c2
# (base = the library before the change).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distill_gpu.py tests/test_fp16_train_gpu.py tests/test_fullsize_gpu.py tests/test_fp32_gpu.py -q -x --timeout 600 --timeout-method thread > gpurun_out/r6aj_tests.log 2>&1 || { tail -30 gpurun_out/r6aj_tests.log; exit 1; }
tail -2 gpurun_out/r6aj_tests.log
REPS=2 T=400 bash taiwan-whisper_amd/tools/calls/ab.sh \
  "python -u bench.py --config c2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160" > gpurun_out/r6aj_ab.log 2>&1
