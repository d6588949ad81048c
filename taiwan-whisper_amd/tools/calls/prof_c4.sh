#!/bin/bash
# Kernel traces of a short c4 run (512 clips, 32 new tokens) in fp16 and bf16, for the per-kernel decode-step breakdown.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
cd /tmp
for dt in fp16 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4_$dt -o run -- python3 $R/bench.py --config c4 --new-tokens 32 --dtype $dt > $R/gpurun_out/prof_c4_$dt.log 2>&1
  echo "$dt trace done"; tail -1 $R/gpurun_out/prof_c4_$dt.log | cut -c1-200
done
