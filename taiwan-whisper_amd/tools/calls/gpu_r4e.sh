#!/bin/bash
# Round 4, call E: write-through (sc1) epilogue stores of the persistent GEMM -- parity tests of the GEMM kernels on the
# candidate, then same-box A/B against ab/libtw_hip_base.so: epilogue-cost variants and own GEMM shapes, the c3 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4e_tests.txt 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4e_tests.txt | tail -8
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
  echo "== epi base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4z 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== epi cand $i"; timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4z 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2; do
  echo "== bench base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-330 || exit 1
  echo "== bench cand $i"; timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-330 || exit 1
done
for i in 1 2; do
  echo "== c2 base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-200 || exit 1
  echo "== c2 cand $i"; timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-200 || exit 1
done
