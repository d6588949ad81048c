#!/bin/bash
# Round 4, call I: the working tree's GPU suite, own GEMM vs hipBLASLt (torch.matmul) on the step's shapes, then the
# round's evidence: PMC traffic passes + kernel trace + bench line (profile_round.sh).  Every GPU step has its own limit; the first failure ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4i_gpu_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4i_gpu_tests.txt | tail -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u taiwan-whisper_amd/tools/bench_vendor.py > gpurun_out/r4i_vendor.txt 2>&1 || exit 1
grep "^gemm" gpurun_out/r4i_vendor.txt
bash taiwan-whisper_amd/tools/profile_round.sh r04 || exit 1
