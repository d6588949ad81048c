#!/bin/bash
# LayerNorm backward writes the 16-bit stream gradient (no separate cast pass): training / config / fp16 tests, then a
# same-box A/B of c2 and c3 against TW_LN_G16=0 (the separate cast), alternating runs.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distill_gpu.py tests/test_fp16_train_gpu.py tests/test_fullsize_gpu.py tests/test_torch_ops_gpu.py -q -x --timeout 600 --timeout-method thread > gpurun_out/r6aa_tests.log 2>&1 || { tail -30 gpurun_out/r6aa_tests.log; exit 1; }
tail -2 gpurun_out/r6aa_tests.log
for i in 1 2; do
  for v in 0 1; do
    echo "== TW_LN_G16=$v c2 run $i"
    TW_LN_G16=$v timeout -k 10 400 python -u bench.py --config c2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160 || exit 1
  done
done > gpurun_out/r6aa_ab.log 2>&1
