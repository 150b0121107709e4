#!/bin/bash
# The one GPU runner: every gpurun call of the project goes through it.
#
#   gpurun --timeout S -- 'bash tools/gpu_steps.sh [-x] "SECS LOG CMD..." ...'
#
# Each argument is one step: a time limit in seconds, a log file name under
# gpurun_out/, then the command (run by bash, so pipes and env assignments
# work).  Steps run in order, each under `timeout -k 10 SECS`.  A step's
# ordinary failure (exit 1-2) is logged and the next step runs, unless -x is
# given (then the script stops at the first failing step).  A time limit,
# abort, crash or signal (exit 124, >= 128) always ends the script there: no
# further GPU step runs after a hang or a fault.  gpurun_out/steps.log records
# every step's command and exit status.
set -u
stop_on_fail=0
if [ "${1:-}" = "-x" ]; then
  stop_on_fail=1
  shift
fi
mkdir -p gpurun_out
export TMPDIR=/tmp
rc_all=0
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
  if [ $rc -ne 0 ]; then
    rc_all=$rc
    if [ $stop_on_fail -eq 1 ]; then
      echo "stopping after rc=$rc ($log), -x" >> gpurun_out/steps.log
      exit $rc
    fi
  fi
done
exit $rc_all
