#!/bin/bash
# Kernel trace + stats of the c3 bench with and without hipBLASLt (TW_GEMM_VENDOR=0), for the per-kernel
# breakdown of what the own kernels lose on the vendor-routed shapes.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
for v in 1 0; do
  TW_GEMM_VENDOR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_v$v.log 2>&1
  echo "vendor=$v trace done"
done
