#!/bin/bash
# GEMV reduce-scatter sums + load-first row staging: bit-identity tests, then same-box A/B against the round's base.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_gpu.py tests/test_fallback_gpu.py tests/test_batched_longform_gpu.py tests/test_fp16_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -k "gemv or decode or generate or fallback or batched or greedy or timestamps or longform" > gpurun_out/r6g_tests.log 2>&1 || { tail -30 gpurun_out/r6g_tests.log; exit 1; }
tail -3 gpurun_out/r6g_tests.log
REPS=2 T=300 bash taiwan-whisper_amd/tools/calls/ab.sh "python -u taiwan-whisper_amd/tools/bench_step.py 20 1,6,8 --rows=8" > gpurun_out/r6g_ab.log 2>&1
