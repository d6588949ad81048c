#!/bin/bash
# Runs "name|command" steps in order on the GPU box, each under its own time limit (given in the step),
# logging to gpurun_out/<name>.log.  A step that times out, aborts or segfaults (124/134/137/139) ends the
# call: nothing more runs on the GPU after it.  Ordinary failures (pytest exit 1) do not stop later steps.
mkdir -p gpurun_out
rc_all=0
for step in "$@"; do
  name=${step%%|*}; cmd=${step#*|}
  echo "== $name: $cmd"
  bash -c "$cmd" > gpurun_out/$name.log 2>&1
  rc=$?
  echo "== $name exit $rc"; tail -4 gpurun_out/$name.log
  [ $rc -ne 0 ] && rc_all=$rc
  case $rc in 124|134|137|139) echo "== stopping after $name"; exit $rc;; esac
done
exit $rc_all
