#!/bin/bash
# Decode attention: V loaded beside K on small grids (threshold 0 = off, 160, 512 workgroups): decode tests on the
# 512 library, then the decode step A/B at batch 1 / 6 / 8.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_decode_gpu.py tests/test_fallback_gpu.py tests/test_lv2_decode_gpu.py tests/test_batched_longform_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread > gpurun_out/r6i_tests.log 2>&1 || { tail -30 gpurun_out/r6i_tests.log; exit 1; }
tail -2 gpurun_out/r6i_tests.log
LIBS="off=ab/libtw_hip_fuse0.so f160=ab/libtw_hip_fuse160.so f512=ab/libtw_hip_fuse512.so" REPS=2 T=300 bash taiwan-whisper_amd/tools/calls/ab.sh \
  "python -u taiwan-whisper_amd/tools/bench_step.py 20 1,6,8 --step-only" > gpurun_out/r6i_ab.log 2>&1
