#!/bin/bash
# Own-kernel GEMM timings per step shape (TW_GEMM_VENDOR=0: nothing routed to hipBLASLt), next to hipBLASLt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TW_GEMM_VENDOR=0 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" || exit 1
TW_GEMM_VENDOR=0 timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_gemm_dec.py 2>&1 | grep -v amdgpu.ids || exit 1
