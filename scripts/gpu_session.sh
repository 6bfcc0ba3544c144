#!/bin/bash
# One GPU session: each GPU step under its own time limit; stop at the first crash/timeout.
# usage: scripts/gpu_session.sh "<step1>" "<step2>" ...   (each step: a shell command string)
# A step's rc: 0 ok, 1 (test failures) continue, anything else (abort/segv/timeout) stop.
mkdir -p gpurun_out
n=0
for step in "$@"; do
  n=$((n+1))
  echo "=== step $n: $step"
  bash -c "$step"
  rc=$?
  echo "=== step $n rc=$rc"
  if [ $rc -gt 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
