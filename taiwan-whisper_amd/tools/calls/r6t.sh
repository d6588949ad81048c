#!/bin/bash
# c3 step kernel traces by (kernel, grid): --dtype fp16 vs bf16 (where the fp16 distillation step loses time).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for dt in fp16 bf16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$dt -o run -- python3 $R/bench.py --dtype $dt --steps 2 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $R/gpurun_out/r6t_prof_$dt.log 2>&1 || exit 1
  python3 $R/taiwan-whisper_amd/tools/trace_by_grid.py $R/gpurun_out/prof_$dt > $R/gpurun_out/r6t_c3_${dt}_by_grid.txt
  rm -rf $R/gpurun_out/prof_$dt
done
