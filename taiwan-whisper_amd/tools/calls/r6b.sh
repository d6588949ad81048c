#!/bin/bash
# Round 6: GPU suite (without the lv2 file, whose fixture is being regenerated), c5 batched long-form lines, and the
# one-rank RCCL bench rehearsal.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6b_tests|timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --ignore=tests/test_lv2_decode_gpu.py" \
  "r6b_c5_b1_none|timeout -k 10 300 python -u bench.py --config c5 --seconds 600 --longform-kwargs none" \
  "r6b_c5_b8_none|timeout -k 10 400 python -u bench.py --config c5 --seconds 600 --batch 8 --longform-kwargs none" \
  "r6b_c5_b1_ref|timeout -k 10 300 python -u bench.py --config c5 --seconds 600" \
  "r6b_c5_b8_ref|timeout -k 10 500 python -u bench.py --config c5 --seconds 600 --batch 8" \
  "r6b_rccl1|TW_BENCH_FORCE_EXCHANGE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline"
