#!/bin/bash
# Own-kernel GEMM timings per step shape (TW_GEMM_VENDOR=0: nothing routed to hipBLASLt), next to hipBLASLt;
# then the tile-order sweep (TW_GEMM_GROUP_M) and the decoder-shape tile variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TW_GEMM_VENDOR=0 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" || exit 1
for gm in 1 2 4 16; do
  echo "== group_m $gm"
  TW_GEMM_GROUP_M=$gm TW_GEMM_VENDOR=0 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | grep -v "K= 5120" || exit 1
done
TW_GEMM_VENDOR=0 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_gemm_dec.py 2>&1 | grep -v amdgpu.ids || exit 1
