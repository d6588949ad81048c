#!/bin/bash
# Round-3 evidence on the default tree: GPU suite, the c3 bench line (CPU baseline included), c2 / c4 / c5 lines,
# the kernel trace of the c3 bench, then the own-GEMM per-shape sweep.  Each GPU step time-limited; a timeout /
# abort / segfault ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c3.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c3.log
timeout -k 10 200 python -u bench.py --config c2 > gpurun_out/bench_c2.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/bench_c4.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c4.log | cut -c1-300
timeout -k 10 300 python -u bench.py --config c5 > gpurun_out/bench_c5.log 2>&1 || exit $?; tail -1 gpurun_out/bench_c5.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_c3.log 2>&1 || exit $?
echo "trace done"
cd $R
bash taiwan-whisper_amd/tools/gemm_own_shapes.sh > gpurun_out/gemm_own_shapes.log 2>&1 || exit $?
echo "sweep done"
exit $rc
