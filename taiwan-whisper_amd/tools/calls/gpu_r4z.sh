#!/bin/bash
# Round 4, last call: the whole GPU suite and the default bench line on the final tree (after the LayerNorm backward
# changes of calls X / Y), plus the c2 line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/z_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/z_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/z_bench.log 2>&1 || exit 1
tail -1 gpurun_out/z_bench.log | cut -c1-200
timeout -k 10 400 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/z_c2.log 2>&1 || exit 1
tail -1 gpurun_out/z_c2.log | cut -c1-200
