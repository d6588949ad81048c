#!/bin/bash
# Round-6 final evidence, part 2: the c2 / c4 / c5 lines (c5 single recording with the reference kwargs, and 8
# recordings in one call) and the driver's 2-rank command shape rehearsed over gloo on one GPU.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
bash taiwan-whisper_amd/tools/calls/gpu_steps.sh \
  "r6ai_c2|timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline" \
  "r6ai_c3_fp16|timeout -k 10 300 python -u bench.py --dtype fp16 --no-cpu-baseline" \
  "r6ai_c4|timeout -k 10 400 python -u bench.py --config c4" \
  "r6ai_c5|timeout -k 10 400 python -u bench.py --config c5" \
  "r6ai_c5_b8_none|timeout -k 10 300 python -u bench.py --config c5 --seconds 600 --batch 8 --longform-kwargs none" \
  "r6ai_c5_b8_ref|timeout -k 10 400 python -u bench.py --config c5 --seconds 600 --batch 8" \
  "r6ai_rehearse2|TW_BENCH_REHEARSE=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-teacher-fwd"
