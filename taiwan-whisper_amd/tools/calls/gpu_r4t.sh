#!/bin/bash
# Round 4, call T: attention forward on v_mfma_f32_16x16x32, software-pipelined (scores of tile kt+1 beside the softmax of tile kt) (candidate = the tree's lib) against the 16x16x32
# kernel (ab/libtw_hip_base.so, same tree otherwise): GPU parity of everything that runs attention, the
# attention micro-bench A/B, and c3 lines A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k "attn or attention" > gpurun_out/r4t_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4t_tests.txt | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base cand; do
    echo "== attn $v run $i"
    if [ $v = base ]; then L=ab/libtw_hip_base.so; else L=taiwan-whisper_amd/tw/_lib/libtw_hip.so; fi
    TW_HIP_LIB=$R/$L timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep "^fwd" || exit 1
  done
done
