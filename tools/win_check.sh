#!/bin/bash
# GPU-box: frontend parity tests, then the windowed front-end bench (both semantics, both grids).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_frontend.py tests/test_gpu_track.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_fe.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_fe.log
[ $rc -eq 0 ] || exit $rc
for args in "" "--as-built" ${WIN_EXTRA:-}; do
  timeout -k 10 300 python tools/bench_window.py --cpu-seconds 0 $args > gpurun_out/win.log 2>&1
  rc=$?; echo "bench_window [$args] rc=$rc"; tail -1 gpurun_out/win.log
  [ $rc -eq 0 ] || exit $rc
done
