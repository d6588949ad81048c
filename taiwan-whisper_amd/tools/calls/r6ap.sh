#!/bin/bash
# c2 bench line on the final tree (split-K 256 tile), two runs.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --config c2 > gpurun_out/r6ap_bench_c2.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config c2 --no-cpu-baseline --no-teacher-fwd > gpurun_out/r6ap_bench_c2_b.log 2>&1
