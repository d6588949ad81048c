#!/bin/bash
# Round 6: re-pinned large-v2 decode tests + batched long-form tests, GEMM tests (dX head tile), and the decode-step
# weight warm-up sweep.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6c_step|timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_step.py 20 1,6 --step-only --prefetch=0,64,128,256" \
  "r6c_tests|timeout -k 10 900 python -u -m pytest tests/test_lv2_decode_gpu.py tests/test_batched_longform_gpu.py tests/test_kernels_gpu.py -m gpu -v -s --timeout 600 --timeout-method thread"
