#!/bin/bash
# Round 4, call D: GPU suite (failures reported, not fatal), then call C's traces (c3, c2) and the c2 line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4d_gpu_tests.txt 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r4d_gpu_tests.txt | tail -12
[ $rc -le 1 ] || exit $rc
bash taiwan-whisper_amd/tools/gpu_r4c.sh
