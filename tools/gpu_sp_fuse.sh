#!/bin/bash
# SuperPoint / image -> pose tests and the image -> pose bench (heads' fp32 epilogue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py > gpurun_out/${TAG}_sp_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_sp_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_image_pose.py > gpurun_out/${TAG}_image_pose.json 2>gpurun_out/${TAG}_image_pose.err
rc=$?; cat gpurun_out/${TAG}_image_pose.json; [ $rc -eq 0 ] || exit $rc
