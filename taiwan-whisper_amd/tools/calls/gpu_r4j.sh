#!/bin/bash
# Round 4, call J: persistent-GEMM staging without per-lane bound arithmetic (ab/libtw_hip_cand.so: the lane part of
# the DMA source offset hoisted, rows bounded by the buffer descriptor) -- GEMM parity tests on it, the L2 diagnostic
# (ab/libtw_hip_diag.so: p4l = every tile stages L2-resident panels), then same-box A/B against the in-tree library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TW_HIP_LIB=$R/ab/libtw_hip_cand.so timeout -k 10 600 python -u -m pytest tests/test_beam_gpu.py tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_configs_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4j_tests.txt | tail -8; [ $rc -le 1 ] || exit $rc
echo "== diag"; TW_HIP_LIB=$R/ab/libtw_hip_diag.so timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e,p4l,p4le,p6e 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
  echo "== gemm tree $i"; timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== gemm cand $i"; TW_HIP_LIB=$R/ab/libtw_hip_cand.so timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2; do
  for lib in tree cand; do
    echo "== c3 $lib $i"
    if [ $lib = cand ]; then export TW_HIP_LIB=$R/ab/libtw_hip_cand.so; else unset TW_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4j_c3_$lib$i.log 2>&1 || exit 1
    tail -1 gpurun_out/r4j_c3_$lib$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d['roofline']['achieved'])"
  done
done
