#!/bin/bash
# LayerNorm statistics on DPP (GEMV prologue + ln_fwd_bf16_kernel): bit-identity tests, then A/B against the
# reduce-scatter library (decode step, c3 step).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_decode_gpu.py tests/test_fallback_gpu.py tests/test_distill_gpu.py tests/test_lv2_decode_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -k "gemv or decode or generate or fallback or layernorm or ln or distill or train or 16bit" > gpurun_out/r6h_tests.log 2>&1 || { tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -3 gpurun_out/r6h_tests.log
LIBS="rs=ab/libtw_hip_rs.so cand=taiwan-whisper_amd/tw/_lib/libtw_hip.so" REPS=2 T=300 bash taiwan-whisper_amd/tools/calls/ab.sh \
  "python -u taiwan-whisper_amd/tools/bench_step.py 20 1,8 --rows=8" \
  "python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-200" > gpurun_out/r6h_ab.log 2>&1
