#!/bin/bash
# PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit-miss, each its own run) + kernel trace of single GEMM shapes
# (tools/one_gemm.py), to compare the L2 / HBM traffic of two shapes.  usage: pmc_shapes.sh "M N K" ["M N K" ...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for s in "$@"; do
  tag=$(echo $s | tr ' ' '_')
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
    gt=$(echo $grp | cut -c1-9)
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcs/${tag}_$gt -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py $s > /dev/null 2>&1
  done
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmcs/${tag}_trace -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py $s > /dev/null 2>&1
  echo "$s done"
done
