#!/bin/bash
# Round 6 evidence: the whole GPU suite, smoke, the round's profiles (PMC traffic passes, kernel trace, MFMA-busy
# passes, the default bench line) and the c2 / c4 lines.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6e_tests|timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread" \
  "r6e_smoke|timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "r6e_profile|bash taiwan-whisper_amd/tools/profile_round.sh r06" \
  "r6e_mfma|bash taiwan-whisper_amd/tools/pmc_mfma.sh" \
  "r6e_c2|timeout -k 10 400 python -u bench.py --config c2 --no-cpu-baseline" \
  "r6e_c4|timeout -k 10 600 python -u bench.py --config c4"
