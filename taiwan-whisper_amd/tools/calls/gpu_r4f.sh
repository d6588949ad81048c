#!/bin/bash
# Round 4, call F: the epilogue's cost split (p4e no epilogue / p4s computed, not stored / p4z stored into tile 0 / p4),
# the GEMM parity tests, and same-box A/B of the 256-tile fill rule (TW_PP_MINFILL, the working tree) against
# ab/libtw_hip_base.so on c3 and c2.  Every GPU step has its own time limit; a timeout or crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4f_tests.txt 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4f_tests.txt | tail -8
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  echo "== epi cand $i"; timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e,p4s,p4z 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2; do
  echo "== bench base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4f_c3_base$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r4f_c3_base$i.log | cut -c1-200
  echo "== bench cand $i"; timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4f_c3_cand$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r4f_c3_cand$i.log | cut -c1-200
done
for i in 1 2; do
  echo "== c2 base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-200 || exit 1
  echo "== c2 cand $i"; timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-200 || exit 1
done
