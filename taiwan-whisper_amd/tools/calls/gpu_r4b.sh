#!/bin/bash
# Round 4, call B: L2-traffic study of the persistent forward GEMM.  For each step shape and tile order (group_m =
# runs of m-tiles walked n-tile by n-tile: 1 = row-major), one FETCH_SIZE pass and one TCC_HIT/TCC_MISS pass
# (separate --pmc runs) and one timing run; plus the gfx950 counter list.  Every GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for shape in "96000 3840 1280" "28608 51904 1280" "28608 5120 1280"; do
  tag=$(echo $shape | tr ' ' '_')
  for g in 1 4 8; do
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f_${tag}_g$g -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py $shape $((g << 24)) > /dev/null 2>&1 || exit 1
    timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/h_${tag}_g$g -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py $shape $((g << 24)) > /dev/null 2>&1 || exit 1
  done
  echo "pmc $tag done"
done
cd $R
timeout -k 10 300 python3 -u taiwan-whisper_amd/tools/bench_group.py 1,2,4,8 > $OUT/group_times.txt 2>&1 || exit 1
timeout -k 10 300 python3 -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e,p4z > $OUT/epi_cost.txt 2>&1 || exit 1
cat $OUT/epi_cost.txt
cat $OUT/group_times.txt
python3 taiwan-whisper_amd/tools/l2_summary.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
