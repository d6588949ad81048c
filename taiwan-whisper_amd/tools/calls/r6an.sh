#!/bin/bash
# GEMM microbench of the weight-gradient shapes with the split-K 256 tile off (R = 0) and on (default).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
for r in 0 1.4; do
  echo "== R=$r c2"
  TW_SK256_R=$r timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_gemm.py c2 2>&1 | grep "dW" || exit 1
  echo "== R=$r c3"
  TW_SK256_R=$r timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_gemm.py dW 2>&1 | grep "dW" || exit 1
done 2>&1 | tee gpurun_out/r6an_dw.log
