#!/bin/bash
# Round 4, call H: full GPU suite on the working tree (maximum3 attention row max, inline-zero score accumulators,
# pack-once GELU epilogue, attention backward: interior tiles unmasked + v_exp, dK/dV at 2 workgroups per CU), then
# same-box A/Bs against ab/libtw_hip_base.so (HEAD~1): persistent-GEMM shapes, attention, the c3 line; and the
# main-loop diagnostics of ab/libtw_hip_diag.so (p4e no epilogue, p5e A-half 1 not read, p6e no restaging, p7e no
# waits).  Every GPU step has its own limit; a timeout or crash ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4h_gpu_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4h_gpu_tests.txt | tail -10; [ $rc -le 1 ] || exit $rc
echo "== diag"; TW_HIP_LIB=$R/ab/libtw_hip_diag.so timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e,p5e,p6e,p7e 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
  echo "== epi base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== epi cand $i"; timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_pp_prio.py p4 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2; do
  echo "== attn base $i"; TW_HIP_LIB=$R/ab/libtw_hip_base.so timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep -E "^fwd|^bwd" || exit 1
  echo "== attn cand occ1 $i"; TW_ATTN_BWD_OCC=1 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep -E "^bwd" || exit 1
  echo "== attn cand $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep -E "^fwd|^bwd" || exit 1
done
for i in 1 2; do
  for lib in base cand; do
    echo "== c3 $lib $i"
    if [ $lib = base ]; then export TW_HIP_LIB=$R/ab/libtw_hip_base.so; else unset TW_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4h_c3_$lib$i.log 2>&1 || exit 1
    tail -1 gpurun_out/r4h_c3_$lib$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('teacher_fwd_ms_per_clip'), d['roofline']['achieved'])"
    echo "== c2 $lib $i"
    timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd > gpurun_out/r4h_c2_$lib$i.log 2>&1 || exit 1
    tail -1 gpurun_out/r4h_c2_$lib$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('step_mfma_frac'))"
  done
done
