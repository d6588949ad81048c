#!/bin/bash
# Round 4, call N: the student's dX products on the forward route (transposed W copy) -- training-path GPU tests, then
# same-box c2 / c3 lines against a copy of the tree with the previous tw/modeling.py (ab/modeling_base.py).  Rerun
# for the selective route (plain-epilogue products only).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_distill_gpu.py tests/test_configs_gpu.py tests/test_fullsize_gpu.py tests/test_torch_ops_gpu.py tests/test_dp_gpu.py tests/test_fp32_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.txt 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/r4n_tests.txt | tail -8; [ $rc -le 1 ] || exit $rc
B=/tmp/tw_base_$$
mkdir -p $B && cp -r bench.py oracle taiwan-whisper_amd $B/ && cp ab/modeling_base.py $B/taiwan-whisper_amd/tw/modeling.py
for i in 1 2; do
  echo "== c2 base $i"; timeout -k 10 300 python3 -u $B/bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-120 || exit 1
  echo "== c2 cand $i"; timeout -k 10 300 python3 -u bench.py --config c2 --steps 6 --warmup 2 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-120 || exit 1
done
for i in 1 2; do
  echo "== c3 base $i"; timeout -k 10 300 python3 -u $B/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-120 || exit 1
  echo "== c3 cand $i"; timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-120 || exit 1
done
rm -rf $B
