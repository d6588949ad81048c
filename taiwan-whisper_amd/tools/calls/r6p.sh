#!/bin/bash
# fp16 distillation (--dtype float16): the new fp16 training kernels and the step vs HF fp16 autocast, then the full
# GPU suite (regressions of the shared kernels) and the default bench line.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6p_f16|timeout -k 10 600 python -u -m pytest tests/test_fp16_train_gpu.py -v --timeout 300 --timeout-method thread" \
  "r6p_tests|timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread --deselect tests/test_fp16_train_gpu.py" \
  "r6p_bench|timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline"
