#!/bin/bash
# Same-box A/B: each command runs REPS times alternately on every library of LIBS ("name=path ..." relative to the
# repo root; the default is ab/libtw_hip_base.so against the tree's library).  Each run has its own time limit
# (T seconds, default 300); the first failure, timeout or abort ends the call.
# usage: [LIBS="base=ab/libtw_hip_base.so cand=taiwan-whisper_amd/tw/_lib/libtw_hip.so"] [REPS=2] [T=300] ab.sh "<cmd>" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
LIBS=${LIBS:-"base=ab/libtw_hip_base.so cand=taiwan-whisper_amd/tw/_lib/libtw_hip.so"}
for cmd in "$@"; do
  for i in $(seq 1 ${REPS:-2}); do
    for lv in $LIBS; do
      name=${lv%%=*}; path=${lv#*=}
      echo "== [$name run $i] $cmd"
      TW_HIP_LIB=$R/$path timeout -k 10 ${T:-300} bash -c "$cmd"
      rc=$?
      [ $rc -ne 0 ] && { echo "== exit $rc"; exit $rc; }
    done
  done
done
exit 0
