#!/bin/bash
# Round-6 final evidence, part 1: GPU suite, smoke, profiles (PMC traffic, kernel trace, MFMA-busy), default bench.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6ah_tests|timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread" \
  "r6ah_smoke|timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6ah_profile|bash taiwan-whisper_amd/tools/profile_round.sh r06_v5" \
  "r6ah_mfma|bash taiwan-whisper_amd/tools/pmc_mfma.sh"
