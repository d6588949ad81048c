#!/bin/bash
# Round 4, call L: residual (bf16 stream) epilogue loading 4 row blocks per memory round trip instead of 2
# (ab/libtw_hip_rb4.so) against the in-tree library: GEMM tests on the candidate, the epilogue micro-bench (PP_ONLY),
# and the c3 line (teacher forward: the teacher encoder's bf16 residual stream) same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TW_HIP_LIB=$R/ab/libtw_hip_rb4.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r4l_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4l_tests.txt | tail -6; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  echo "== epi tree $i"; PP_ONLY=1 timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_epilogue.py 2>&1 | grep -E "res bf16|bias\+round" || exit 1
  echo "== epi rb4 $i"; TW_HIP_LIB=$R/ab/libtw_hip_rb4.so PP_ONLY=1 timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_epilogue.py 2>&1 | grep -E "res bf16|bias\+round" || exit 1
done
for i in 1 2; do
  for lib in tree rb4; do
    echo "== c3 $lib $i"
    if [ $lib = rb4 ]; then export TW_HIP_LIB=$R/ab/libtw_hip_rb4.so; else unset TW_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4l_c3_$lib$i.log 2>&1 || exit 1
    tail -1 gpurun_out/r4l_c3_$lib$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d['roofline']['achieved'])"
  done
done
