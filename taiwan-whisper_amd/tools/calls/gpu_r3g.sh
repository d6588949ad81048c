#!/bin/bash
# c3 A/B of two host-side toggles (same box), then the round's PMC evidence (traffic + MFMA-busy) on the default tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for env in "TW_NOTHING=1" "TW_DEFER_RES=2" "TW_GEMM_GROUP_DEC=2" "TW_NOTHING=1"; do
  echo "== $env"; env $env timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1 | cut -c1-330 || exit 1
done
for env in "TW_NOTHING=1" "TW_GEMM_SK_SUB_MINK=1024" "TW_NOTHING=1" "TW_GEMM_SK_SUB_MINK=1024"; do
  echo "== c4 $env"; env $env timeout -k 10 300 python -u bench.py --config c4 --new-tokens 64 | tail -1 | cut -c1-200 || exit 1
done
bash taiwan-whisper_amd/tools/profile_round.sh r03 > gpurun_out/profile_round.log 2>&1 || { tail -5 gpurun_out/profile_round.log; exit 1; }
tail -3 gpurun_out/profile_round.log
bash taiwan-whisper_amd/tools/pmc_mfma.sh > gpurun_out/pmc_mfma.log 2>&1 || { tail -5 gpurun_out/pmc_mfma.log; exit 1; }
tail -4 gpurun_out/pmc_mfma.log
