#!/bin/bash
# pose parity/tolerance tests (GPU) + pose timing + the headline bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_pose.py tests/test_gpu_track.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pose.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_pose.log; [ $rc -eq 0 ] || exit $rc
POSE_BATCHES=1024 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pose_timing.log 2>&1 || exit $?
grep "hyp=256" gpurun_out/pose_timing.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --check 2 --score-steps 0 --extra-steps 0 --window-steps 0 ${BENCH_ARGS:-} > gpurun_out/bench_pose.log 2>&1; rc=$?
tail -1 gpurun_out/bench_pose.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stages_ms_per_step"])'
exit $rc
