#!/bin/bash
# Round 4, call A: GPU suite on the working tree (failures reported, not fatal), then same-box A/Bs: the working-tree
# library against ab/libtw_hip_base.so on the own GEMM shapes and the c3 bench, and the attention forward ring depth
# (TW_ATTN_FWD=0: 2-stage, 2: 3-stage).  Every GPU step has its own time limit; a timeout or crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4a_gpu_tests.txt 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4a_gpu_tests.txt | tail -12
[ $rc -le 1 ] || exit $rc                                   # 1 = test failures; anything else (timeout, crash) stops
for i in 1 2; do
  echo "== gemm base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
  echo "== gemm cand $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
done
for i in 1 2; do
  for v in 0 2; do
    echo "== attn variant $v run $i"
    TW_ATTN_FWD=$v timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep "^fwd" || exit 1
  done
done
for i in 1 2; do
  echo "== bench base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-420 || exit 1
  echo "== bench cand $i"; timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline | tail -1 | cut -c1-420 || exit 1
done
