#!/bin/bash
# fp16 distillation measured: c3 / c2 steps with --dtype fp16 (fp16 teacher, fp16 autocast, loss scaler) beside the
# bf16 lines on the same box, and the fp16 step-parity tests with their printed distances.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6r_f16_steps|timeout -k 10 600 python -u -m pytest tests/test_fp16_train_gpu.py -k 'step or scaler' -v -s --timeout 300 --timeout-method thread" \
  "r6r_c3_fp16|timeout -k 10 300 python -u bench.py --dtype fp16 --no-cpu-baseline" \
  "r6r_c3_bf16|timeout -k 10 300 python -u bench.py --no-cpu-baseline" \
  "r6r_c2_fp16|timeout -k 10 300 python -u bench.py --config c2 --dtype fp16 --no-cpu-baseline" \
  "r6r_c2_bf16|timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline"
