#!/bin/bash
# round 4, call b: new GPU tests (image -> pose, long frame 1), the f16 probe, phase traces,
# the near-threshold PMC profile, the image -> pose bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_image_to_pose.py tests/test_gpu_allpairs.py -k "image or raw or long_frame" \
    -m gpu -q -rf --timeout 150 --timeout-method thread > gpurun_out/pytest_r04b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_r04b.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_image_pose.py > gpurun_out/bench_image_pose.log 2>&1
rc=$?; echo "image_pose rc=$rc"; tail -3 gpurun_out/bench_image_pose.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r04a.sh
