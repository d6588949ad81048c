#!/bin/bash
# fp16 ragged grids as whole tiles + edge strips: fp16 tests, then same-box A/B of the c3 fp16 step (base = the
# committed library).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_fp16_train_gpu.py tests/test_fp16_gpu.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r6v_tests.log 2>&1 || { tail -30 gpurun_out/r6v_tests.log; exit 1; }
tail -2 gpurun_out/r6v_tests.log
REPS=2 T=400 bash taiwan-whisper_amd/tools/calls/ab.sh \
  "python -u bench.py --dtype fp16 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160" > gpurun_out/r6v_ab.log 2>&1
