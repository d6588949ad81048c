#!/bin/bash
# Bias-gradient column sums in 64-row chunks (more blocks in flight) + a 16-column final reduce: kernel / training
# tests, then c2 and c3 lines, and a c2 kernel trace by grid.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6x_tests|timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_distill_gpu.py tests/test_fp16_train_gpu.py tests/test_torch_ops_gpu.py -q -x --timeout 600 --timeout-method thread" \
  "r6x_c2|timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --no-teacher-fwd" \
  "r6x_c3|timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-teacher-fwd" || exit 1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c2 -o run -- python3 $R/bench.py --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-teacher-fwd > $R/gpurun_out/r6x_prof_c2.log 2>&1 || exit 1
python3 $R/taiwan-whisper_amd/tools/trace_by_grid.py $R/gpurun_out/prof_c2 > $R/gpurun_out/r6x_c2_by_grid.txt
rm -rf $R/gpurun_out/prof_c2
