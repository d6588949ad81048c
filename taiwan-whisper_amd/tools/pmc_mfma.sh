#!/bin/bash
# MFMA-busy evidence (north_star: "validated by rocprof HBM GB/s and MFMA-busy counters"): one --pmc
# pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE; kernel trace off) over
#   (1) the large-v2 teacher forward (B = 64, 1 warm-up + 2 reps), (2) a short c3 bench run;
# summaries -> gpurun_out/mfma/*.txt|json (copy to profiles/).  Each GPU step time-limited.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mfma
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
CTR="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $CTR --output-format csv -d $OUT/teacher -o run -- python3 $R/taiwan-whisper_amd/tools/prof_teacher.py --reps 2 > $OUT/teacher.log 2>&1
echo "teacher pass done"
timeout -s KILL 300 rocprofv3 --pmc $CTR --output-format csv -d $OUT/step -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $OUT/step.log 2>&1
echo "step pass done"
cd $R
python3 taiwan-whisper_amd/tools/mfma_summary.py $OUT/teacher "teacher forward (large-v2, B=64, 3 reps)" --json $OUT/teacher.json | tee $OUT/teacher.txt
python3 taiwan-whisper_amd/tools/mfma_summary.py $OUT/step "c3 distillation step (B=64, 3 steps)" --json $OUT/step.json | tee $OUT/step.txt
