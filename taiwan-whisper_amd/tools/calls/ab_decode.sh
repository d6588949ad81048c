#!/bin/bash
# Decode-path A/B (c4 / c5 workloads) of the tree against ab/libtw_hip_base.so: decode + fp32 tests, the
# decode-attention tool on both libraries, a kernel trace of one c4 step (new), then c4 on both.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
BASE=$R/taiwan-whisper_amd/ab/libtw_hip_base.so
timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_fp32_gpu.py tests/test_fallback_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/abd_pytest.log 2>&1
tail -2 gpurun_out/abd_pytest.log
for i in 1 2; do
  echo "== base $i"; TW_HIP_LIB=$BASE timeout -k 10 120 python -u taiwan-whisper_amd/tools/bench_decode_attn.py
  echo "== new $i"; timeout -k 10 120 python -u taiwan-whisper_amd/tools/bench_decode_attn.py
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- \
  python3 bench.py --config c4 --steps 1 --warmup 1 > gpurun_out/prof_c4.log 2>&1
echo "trace done"
echo "== c4 base"; TW_HIP_LIB=$BASE timeout -k 10 300 python -u bench.py --config c4 | tail -1
echo "== c4 new"; timeout -k 10 300 python -u bench.py --config c4 | tail -1
