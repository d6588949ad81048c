#!/bin/bash
# Same-box A/B of the in-tree library against a candidate (TW_HIP_LIB=$1): own-kernel GEMM shapes, then the c3
# bench alternately.  usage: ab_lib.sh <candidate .so path relative to the repo root>
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
CAND=$R/$1
for i in 1 2; do
  echo "== base $i"; timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
  echo "== cand $i"; TW_HIP_LIB=$CAND timeout -k 10 200 python -u taiwan-whisper_amd/tools/bench_vendor.py 2>&1 | grep "^gemm" | cut -c1-70 || exit 1
done
for i in 1 2; do
  echo "== bench base $i"; timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1 | cut -c1-330 || exit 1
  echo "== bench cand $i"; TW_HIP_LIB=$CAND timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline | tail -1 | cut -c1-330 || exit 1
done
