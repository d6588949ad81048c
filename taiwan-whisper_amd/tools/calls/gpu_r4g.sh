#!/bin/bash
# Round 4, call G: attention forward with the row sums on the matrix pipe (TW_ATTN_FWD=5) and the maximum3 row-max
# chain (default kernel): parity (kernel tests on the default, attention + distillation tests on variant 5), the
# attention micro-bench 0 vs 5, and same-binary A/Bs on c3 / c2 (TW_ATTN_FWD=5, TW_PP_MINFILL=101 = fill rule off).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_fp16_gpu.py > gpurun_out/r4g_tests_default.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4g_tests_default.txt | tail -6; [ $rc -le 1 ] || exit $rc
TW_ATTN_FWD=5 timeout -k 10 600 $T tests/test_kernels_gpu.py -k "attn or attention" tests/test_distill_gpu.py tests/test_torch_ops_gpu.py > gpurun_out/r4g_tests_v5.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4g_tests_v5.txt | tail -6; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for v in 0 5; do
    echo "== attn variant $v run $i"
    TW_ATTN_FWD=$v timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep "^fwd" || exit 1
  done
done
for i in 1 2; do
  for e in "X=0" "TW_ATTN_FWD=5" "TW_PP_MINFILL=101"; do
    echo "== c3 $e run $i"
    env $e timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4g_c3.log 2>&1 || exit 1
    tail -1 gpurun_out/r4g_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d['roofline']['achieved'])"
  done
done
for i in 1 2; do
  for e in "X=0" "TW_PP_MINFILL=101"; do
    echo "== c2 $e run $i"
    env $e timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-120 || exit 1
  done
done
