#!/bin/bash
# Split-K tile rate R sweep, same box: c2 at R = 1.1 / 1.4 / 2.0, c3 at 1.4 / 2.0.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export PYTHONUNBUFFERED=1
run() {
  echo "== $1 R=$2"
  TW_SK256_R=$2 timeout -k 10 400 python -u bench.py --config $1 --no-cpu-baseline --no-teacher-fwd > gpurun_out/r6am_b.log 2>&1 || { tail -20 gpurun_out/r6am_b.log; exit 1; }
  tail -1 gpurun_out/r6am_b.log | cut -c1-140
}
{ for i in 1 2; do for r in 1.1 1.4 2.0; do run c2 $r || exit 1; done; done
  for i in 1 2; do for r in 1.4 2.0; do run c3 $r || exit 1; done; done; } 2>&1 | tee gpurun_out/r6am_ab.log
