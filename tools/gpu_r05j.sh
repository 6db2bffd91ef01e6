#!/bin/bash
# the 4-wave re-screen: allpairs parity, SuperPoint-descriptor timing, image -> pose at 1-3 pipelines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05j}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_allpairs.py tests/test_gpu_image_to_pose.py tests/test_gpu_sequence.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_real.py > gpurun_out/${TAG}_real.json 2>gpurun_out/${TAG}_err.log || exit $?
cat gpurun_out/${TAG}_real.json
for pl in 1 2 3; do
  timeout -k 10 200 python tools/bench_image_pose.py --pipelines $pl > gpurun_out/${TAG}_image_pose_p$pl.json 2>>gpurun_out/${TAG}_err.log || exit $?
  cut -c 150-700 gpurun_out/${TAG}_image_pose_p$pl.json
done
