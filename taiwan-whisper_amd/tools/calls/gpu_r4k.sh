#!/bin/bash
# Round 4, call K: MFMA-busy passes (pmc_mfma.sh), a kernel trace of the c2 step (by grid) and the c2 line, the
# persistent GEMM's fp16 instantiation against bf16 on the same shapes, and the c4 / c5 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r4k
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash taiwan-whisper_amd/tools/pmc_mfma.sh || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r4k/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 3 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $R/gpurun_out/r4k/prof_c2.log 2>&1 || exit 1
cd $R
python3 taiwan-whisper_amd/tools/trace_by_grid.py gpurun_out/r4k/prof_c2 --reps 4 --top 40 > gpurun_out/r4k/trace_c2.txt 2>&1
head -25 gpurun_out/r4k/trace_c2.txt
timeout -k 10 300 python3 -u bench.py --config c2 --no-cpu-baseline > gpurun_out/r4k/bench_c2.log 2>&1 || exit 1
tail -1 gpurun_out/r4k/bench_c2.log | cut -c1-400
echo "== bf16"; timeout -k 10 300 python3 -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e 2>&1 | grep -v amdgpu.ids || exit 1
echo "== fp16"; timeout -k 10 300 python3 -u taiwan-whisper_amd/tools/bench_pp_prio.py p4,p4e fp16 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python3 -u bench.py --config c4 > gpurun_out/r4k/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/r4k/bench_c4.log | cut -c1-300
