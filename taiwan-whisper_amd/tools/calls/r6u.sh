#!/bin/bash
# fp16 GEMM: ragged grids as whole tiles + edge strips, hybrid fp16 GELU (fast above -3, torch's formula below):
# fp16 kernel / decode / training tests, then c3 fp16 training and c4 fp16 decode lines.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6u_tests|timeout -k 10 900 python -u -m pytest tests/test_fp16_train_gpu.py tests/test_fp16_gpu.py tests/test_decode_configs_gpu.py tests/test_lv2_decode_gpu.py tests/test_batched_longform_gpu.py -v --timeout 600 --timeout-method thread" \
  "r6u_c3_fp16|timeout -k 10 300 python -u bench.py --dtype fp16 --no-cpu-baseline" \
  "r6u_c4|timeout -k 10 400 python -u bench.py --config c4 --no-cpu-baseline"
