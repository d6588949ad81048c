#!/bin/bash
# Head-major cross K/V: decode / fp32 / fallback / pseudo-labelling / token-agreement tests, the layout tool,
# then c4 and c5 with TW_XKV_HEAD_MAJOR=0 and 1.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
TW_XKV_HEAD_MAJOR=1 timeout -k 10 500 python -u -m pytest tests/test_decode_gpu.py tests/test_fp32_gpu.py tests/test_fallback_gpu.py \
  tests/test_pseudo_labelling_gpu.py tests/test_token_agreement_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/xkv_pytest.log 2>&1
tail -2 gpurun_out/xkv_pytest.log
(cd taiwan-whisper_amd/tools && timeout -k 10 200 python -u bench_decode_layout.py)
for c in c4 c5; do
  echo "== $c row-interleaved"; TW_XKV_HEAD_MAJOR=0 timeout -k 10 300 python -u bench.py --config $c | tail -1
  echo "== $c head-major"; TW_XKV_HEAD_MAJOR=1 timeout -k 10 300 python -u bench.py --config $c | tail -1
done
