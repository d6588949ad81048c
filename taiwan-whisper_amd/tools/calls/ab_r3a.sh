#!/bin/bash
# Session A/B: base library (committed sources) vs the working tree, GEMM per shape + attention variants + bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BASE=$R/taiwan-whisper_amd/ab/libtw_hip_base.so
TW_ATTN_FWD=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k "attention or gemm" --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
echo "== base vendor/shape"; TW_HIP_LIB=$BASE timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep -v amdgpu.ids
echo "== new vendor/shape"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep -v amdgpu.ids
for gm in 1 4 16; do echo "== new group_m $gm"; TW_GEMM_GROUP_M=$gm timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm"; done
for v in 0 1 0 1; do echo "== new attn variant $v"; TW_ATTN_FWD=$v timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_attn.py 2>&1 | grep fwd; done
echo "== bench base"; TW_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
echo "== bench new"; timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
echo "== bench new attn1"; TW_ATTN_FWD=1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
echo "== bench new attn1 vendor0"; TW_GEMM_VENDOR=0 TW_ATTN_FWD=1 timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1
