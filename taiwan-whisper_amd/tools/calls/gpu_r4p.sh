#!/bin/bash
# Round 4, call P: attention forward on v_mfma_f32_32x32x16 (candidate = the tree's lib) against the 16x16x32
# kernel (ab/libtw_hip_base.so, same tree otherwise): GPU parity of everything that runs attention, the
# attention micro-bench A/B, and c3 lines A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_distill_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_fp32_gpu.py tests/test_torch_ops_gpu.py \
  tests/test_decode_gpu.py tests/test_beam_gpu.py > gpurun_out/r4p_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4p_tests.txt | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base cand; do
    echo "== attn $v run $i"
    if [ $v = base ]; then L=ab/libtw_hip_base.so; else L=taiwan-whisper_amd/tw/_lib/libtw_hip.so; fi
    TW_HIP_LIB=$R/$L timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep "^fwd" || exit 1
  done
done
for i in 1 2; do
  for v in base cand; do
    echo "== c3 $v run $i"
    if [ $v = base ]; then L=ab/libtw_hip_base.so; else L=taiwan-whisper_amd/tw/_lib/libtw_hip.so; fi
    TW_HIP_LIB=$R/$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4p_c3.log 2>&1 || exit 1
    tail -1 gpurun_out/r4p_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d.get('teacher_fwd_mfma_frac'), d['roofline']['achieved'])"
  done
done
