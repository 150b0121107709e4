#!/bin/bash
# Run GPU steps in order: each argument is "SECONDS LOG CMD..." (one string).
# A step's ordinary failure (exit 1-2) is logged and the next step runs; a
# time limit, abort, crash or signal (exit 124, >= 128) ends the script there.
for step in "$@"; do
  read -r secs log cmd <<< "$step"
  echo "== $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "rc=$rc $log" >> gpurun_out/steps.log
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then
    echo "stopping after rc=$rc ($log)" >> gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
