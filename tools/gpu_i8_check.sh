#!/bin/bash
# int8 all-pairs (BASELINE config 5): GPU parity tests, then tools/bench_i8.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_allpairs.py -m gpu -x -q -k "i8" --timeout 120 --timeout-method thread > gpurun_out/pytest_i8.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_i8.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_i8.py ${I8_ARGS:-} > gpurun_out/bench_i8.log 2>&1; rc=$?
tail -1 gpurun_out/bench_i8.log | cut -c1-400
exit $rc
