#!/bin/bash
# Round 4, final evidence on the final tree: the whole GPU suite, then profile_round.sh (FETCH/WRITE PMC passes,
# kernel trace + stats, the default bench line), pmc_mfma.sh (MFMA-busy of the teacher forward and the c3 step),
# and the c2 / c4 lines.  Each GPU step time-limited; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/final_tests.txt; [ $rc -eq 0 ] || exit $rc
bash taiwan-whisper_amd/tools/profile_round.sh r04_v3 || exit 1
bash taiwan-whisper_amd/tools/pmc_mfma.sh || exit 1
cd $R
timeout -k 10 400 python -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/final_c2.log 2>&1 || exit 1
tail -1 gpurun_out/final_c2.log | cut -c1-200
timeout -k 10 400 python -u bench.py --config c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/final_c4.log 2>&1 || exit 1
tail -1 gpurun_out/final_c4.log | cut -c1-200
