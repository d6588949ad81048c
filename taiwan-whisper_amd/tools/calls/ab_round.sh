#!/bin/bash
# Same-box A/B of a candidate tree against a baseline library (TW_HIP_LIB=ab/libtw_hip_base.so, built from the
# committed sources): optional pytest selection first, then the given tool alternately on both libraries, then
# bench.py on both.  Every GPU step has its own time limit; the first failure ends the script.
# usage: ab_round.sh "<pytest -k expr or empty>" "<tool.py args>" [bench steps]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BASE=$R/taiwan-whisper_amd/ab/libtw_hip_base.so
K=$1
TOOL=$2
STEPS=${3:-5}
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread \
    > gpurun_out/ab_pytest.log 2>&1
  tail -2 gpurun_out/ab_pytest.log
fi
if [ -n "$TOOL" ]; then
  for i in 1 2; do
    echo "== base $i"; TW_HIP_LIB=$BASE timeout -k 10 200 python -u taiwan-whisper_amd/tools/$TOOL
    echo "== new $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/$TOOL
  done
fi
if [ "$STEPS" != "0" ]; then
  echo "== bench base"; TW_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline | tail -1
  echo "== bench new"; timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 2 --no-cpu-baseline | tail -1
fi
