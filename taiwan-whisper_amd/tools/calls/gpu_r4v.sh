#!/bin/bash
# Round 4, call V (after U: 8 loads in flight lost 15-25 %, nontemporal won 3 %): U = 4 + nontemporal (candC),
# U = 2 + nontemporal (candD) against the kept kernel.  Call U: cross-attention decode (tw_decode_attn, one workgroup per (clip, head)) with 8 K/V loads in
# flight per lane instead of 4 (candA = ab/libtw_hip_candA.so) and the same with nontemporal K/V loads (candB =
# the tree's lib) against the kept kernel (ab/libtw_hip_base.so): decode parity, the c4-shape micro-bench
# (fp16, B = 512) and the bf16 shapes, then c4 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
TW_HIP_LIB=$R/ab/libtw_hip_candC.so timeout -k 10 900 $T tests/test_decode_gpu.py tests/test_fp16_gpu.py tests/test_fp32_gpu.py tests/test_beam_gpu.py \
  tests/test_kernels_gpu.py -k "decode or greedy or fp16 or fp32 or beam or generate" > gpurun_out/r4v_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4v_tests.txt | tail -6; [ $rc -eq 0 ] || exit $rc
lib() { case $1 in base) echo $R/ab/libtw_hip_base.so;; *) echo $R/ab/libtw_hip_$1.so;; esac; }
for i in 1 2; do
  for v in base candC candD; do
    echo "== decode attn $v run $i"
    TW_HIP_LIB=$(lib $v) timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_decode_attn.py fp16 512 256 || exit 1
    TW_HIP_LIB=$(lib $v) timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_decode_attn.py 1 16 64 128 || exit 1
  done
done
for v in base candC candD base candC; do
  echo "== c4 $v"
  TW_HIP_LIB=$(lib $v) timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r4v_c4.log 2>&1 || exit 1
  tail -1 gpurun_out/r4v_c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('ms_per_decode_step'), d['roofline']['achieved'])"
done
