#!/bin/bash
# Round 4, call W: add+LayerNorm of the bf16 stream with nontemporal x / r loads and x_out stores (the tree's lib)
# against plain ones (ab/libtw_hip_base.so = the final round-4 tree): LN parity, tools/bench_ln.py, c3 lines
# (teacher forward ms/clip).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_distill_gpu.py -k "layernorm or ln or distill or train or fp16" > gpurun_out/r4w_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4w_tests.txt | tail -6; [ $rc -eq 0 ] || exit $rc
lib() { case $1 in base) echo $R/ab/libtw_hip_base.so;; *) echo $R/taiwan-whisper_amd/tw/_lib/libtw_hip.so;; esac; }
for i in 1 2; do
  for v in base cand; do
    echo "== ln $v run $i"
    TW_HIP_LIB=$(lib $v) timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_ln.py 2>&1 | grep "bfloat16" || exit 1
  done
done
for i in 1 2; do
  for v in base cand; do
    echo "== c3 $v run $i"
    TW_HIP_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4w_c3.log 2>&1 || exit 1
    tail -1 gpurun_out/r4w_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d.get('teacher_fwd_mfma_frac'), d['roofline']['achieved'])"
  done
done
