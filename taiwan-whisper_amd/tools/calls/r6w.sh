#!/bin/bash
# fp16 autocast defers the residual update to the next LayerNorm (tw_add_layernorm_fwd_f16): same-box A/B of the c3
# fp16 step against TW_DEFER_RES=0 (every residual in the GEMM epilogue), alternating runs.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for d in 0 1; do
    echo "== TW_DEFER_RES=$d run $i"
    TW_DEFER_RES=$d timeout -k 10 400 python -u bench.py --dtype fp16 --no-cpu-baseline --no-teacher-fwd | tail -1 | cut -c1-160 || exit 1
  done
done > gpurun_out/r6w_ab.log 2>&1
