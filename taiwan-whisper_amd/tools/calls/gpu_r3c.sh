#!/bin/bash
# GPU suite, then the vendor on/off kernel traces and the per-shape PMC passes (enc qkv vs enc fc1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
bash taiwan-whisper_amd/tools/prof_vendor_ab.sh || exit $?
bash taiwan-whisper_amd/tools/pmc_shapes.sh "96000 3840 1280" "96000 5120 1280" "28608 3840 1280" || exit $?
exit $rc
