#!/bin/bash
# round 4, call c: the shipping build's new tests, A/B of builds, traced timing experiments
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_image_to_pose.py tests/test_gpu_superpoint.py -m gpu -q -rf \
    --timeout 150 --timeout-method thread > gpurun_out/pytest_r04c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04c.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/bench_image_pose.py > gpurun_out/bench_image_pose.log 2>&1
rc=$?; echo "image_pose rc=$rc"; tail -1 gpurun_out/bench_image_pose.log | cut -c1-600
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TRACES="${TRACES:-trace:0.01875 nodma_trace:0.01875 noquant_trace:0.01875 nofold_trace:0.01875 trace:0.05 nocoop_trace:0.05 base_trace:0.05}" \
    bash tools/gpu_trace_exp.sh || exit $?
VARIANTS="${VARIANTS:-ship base nocoop cc}" TESTS_FOR="${TESTS_FOR:-ship cc}" AB_SCORE=5 bash tools/gpu_ab.sh
