#!/bin/bash
# Last check of the final tree (split-K 256 tile): GPU suite, smoke, default bench line.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6ao_tests|timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread" \
  "r6ao_smoke|timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6ao_bench|timeout -k 10 400 python -u bench.py"
