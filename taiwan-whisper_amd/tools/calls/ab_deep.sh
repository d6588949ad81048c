#!/bin/bash
# TW_GEMM_DEEP (4-stage 128x128 ring for grids of <= one tile per CU): parity under the toggle, then c4 A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TW_GEMM_DEEP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py -m gpu -q -k "gemm" --timeout 200 --timeout-method thread > gpurun_out/deep_pytest.log 2>&1 || { tail -20 gpurun_out/deep_pytest.log; exit 1; }
tail -1 gpurun_out/deep_pytest.log
for i in 1 2; do
  for env in "TW_NOTHING=1" "TW_GEMM_DEEP=1"; do
    echo "== c4 $env $i"; env $env timeout -k 10 300 python -u bench.py --config c4 --new-tokens 64 | tail -1 | cut -c1-260 || exit 1
  done
done
for env in "TW_NOTHING=1" "TW_GEMM_DEEP=1"; do
  echo "== c5 $env"; env $env timeout -k 10 300 python -u bench.py --config c5 --seconds 600 | tail -1 | cut -c1-260 || exit 1
done
