#!/bin/bash
# k_pose_ransac under bench.py's noisy_pose keypoints (0.5 px, 20 % outliers): time by
# (hypotheses, refine_iters) at 8192 pairs, then block 0's phase clocks (PE_TRACE build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
POSE_BATCHES=8192 POSE_NOISE=1 POSE_HYPS=128,256 POSE_ITERS=0,3,10 timeout -k 10 200 python tools/pose_timing.py \
  > gpurun_out/${TAG}_pose_scan.log 2>&1 || exit $?
cat gpurun_out/${TAG}_pose_scan.log
POSE_BATCHES=256 POSE_NOISE=1 POSE_HYPS=256 POSE_ITERS=10 MV_LIB=build_variants/libmaveric_posetrace.so \
  timeout -k 10 200 python tools/pose_timing.py > gpurun_out/${TAG}_pose_trace.log 2>&1 || exit $?
grep -m 3 "pose phases" gpurun_out/${TAG}_pose_trace.log
