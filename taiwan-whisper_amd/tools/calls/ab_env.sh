#!/bin/bash
# Same-tree A/B of an environment switch read once per process: optional pytest selection, then the tool and
# a bench command alternately with ENV_A and ENV_B.  usage: ab_env.sh "<pytest -k expr>" "ENV_A" "ENV_B" "<tool args>" "<bench args>"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$1" --timeout 120 --timeout-method thread \
    > gpurun_out/abe_pytest.log 2>&1
  tail -2 gpurun_out/abe_pytest.log
fi
for i in 1 2; do
  if [ -n "$4" ]; then
    echo "== A($2) $i"; env $2 timeout -k 10 200 python -u taiwan-whisper_amd/tools/$4
    echo "== B($3) $i"; env $3 timeout -k 10 200 python -u taiwan-whisper_amd/tools/$4
  fi
done
if [ -n "$5" ]; then
  echo "== bench A($2)"; env $2 timeout -k 10 300 python -u bench.py $5 | tail -1
  echo "== bench B($3)"; env $3 timeout -k 10 300 python -u bench.py $5 | tail -1
fi
