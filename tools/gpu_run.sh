#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/timeout (exit >= 124 or signal),
# carry on past ordinary failures (exit 1/2) so later measurements still run.
# Usage: tools/gpu_run.sh "<label>|<timeout_s>|<command>" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
overall=0
for spec in "$@"; do
  label=${spec%%|*}; rest=${spec#*|}; tmo=${rest%%|*}; cmd=${rest#*|}
  echo "=== [$label] ($(date +%T)) $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== [$label] rc=$rc"
  tail -n 25 "gpurun_out/$label.log"
  if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then
    echo "!!! stopping after [$label] rc=$rc (fault/timeout)"; exit $rc
  fi
  [ $rc -ne 0 ] && overall=$rc
done
exit $overall
