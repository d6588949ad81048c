#!/bin/bash
# Round 4, call C: kernel traces of the c3 and c2 steps (per-kernel, per-grid time breakdown) and the c2 line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4c
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $OUT/prof_c3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $OUT/prof_c2.log 2>&1 || exit 1
cd $R
python3 taiwan-whisper_amd/tools/trace_by_grid.py $OUT/prof_c3 --reps 4 --top 50 > $OUT/trace_c3.txt 2>&1
python3 taiwan-whisper_amd/tools/trace_by_grid.py $OUT/prof_c2 --reps 4 --top 50 > $OUT/trace_c2.txt 2>&1
head -30 $OUT/trace_c3.txt
head -40 $OUT/trace_c2.txt
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline | tail -1 | cut -c1-600
