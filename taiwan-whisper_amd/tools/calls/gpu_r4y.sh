#!/bin/bash
# Round 4, call Y: LayerNorm backward instantiated per exact 256-column chunk count, 768 blocks at D = 1280 (the tree's lib)
# against call X's kernel (ab/libtw_hip_base.so = tree e57f39c): LN parity + the distillation
# tests, tools/bench_ln.py bwd, c2 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py tests/test_distill_gpu.py tests/test_torch_ops_gpu.py tests/test_fp32_gpu.py -k "layernorm or ln or distill or train or linear or fp32" > gpurun_out/r4y_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4y_tests.txt | tail -6; [ $rc -eq 0 ] || exit $rc
lib() { case $1 in base) echo $R/ab/libtw_hip_base.so;; *) echo $R/taiwan-whisper_amd/tw/_lib/libtw_hip.so;; esac; }
for i in 1 2; do
  for v in base cand; do
    echo "== ln bwd $v run $i"
    TW_HIP_LIB=$(lib $v) timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_ln.py bwd || exit 1
  done
done
for i in 1 2; do
  for v in base cand; do
    echo "== c2 $v run $i"
    TW_HIP_LIB=$(lib $v) timeout -k 10 300 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r4y_c2.log 2>&1 || exit 1
    tail -1 gpurun_out/r4y_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('step_mfma_frac'))"
  done
done
