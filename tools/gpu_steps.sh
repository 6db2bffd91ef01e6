#!/bin/bash
# Run GPU steps in order ("name|seconds|command" per argument), each under its own time limit,
# output to gpurun_out/<name>.log.  A step that FAILS (exit 1: failing tests) lets the next one run;
# a crash, abort, fault or time limit (any other non-zero status) ends the call there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
worst=0
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc: $(tail -1 gpurun_out/$name.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  [ $rc -gt $worst ] && worst=$rc
done
exit $worst
