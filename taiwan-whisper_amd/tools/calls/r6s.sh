#!/bin/bash
# In-place loss gradient over the student logits (tw_kl_ce dS == S): kernel bit-identity, step parity tests, bench.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6s_tests|timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_distill_gpu.py tests/test_configs_gpu.py tests/test_fp16_train_gpu.py tests/test_fullsize_gpu.py tests/test_dp_gpu.py -q -x --timeout 600 --timeout-method thread" \
  "r6s_bench|timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
