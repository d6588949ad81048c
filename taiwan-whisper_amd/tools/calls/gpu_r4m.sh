#!/bin/bash
# Round 4, call M: the student's input-gradient GEMMs as stored-W transposed-operand products vs a transposed W copy on
# the forward route (tools/bench_dx.py), same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python3 -u taiwan-whisper_amd/tools/bench_dx.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4m_dx.txt || exit 1
