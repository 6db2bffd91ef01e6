#!/bin/bash
# round 4: k_pose_ransac at 4 waves per SIMD (shipping, 128 VGPRs + spills) against 3 (pw3, no
# spills): the pose GPU tests on pw3, the headline A/B, and the pose alone on noisy keypoints
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MV_LIB=build_variants/libmaveric_pw3.so timeout -k 10 300 python -m pytest tests/test_gpu_pose.py tests/test_gpu_kitti_e2e.py \
    -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pw3_tests.log 2>&1
rc=$?; echo "tests pw3 rc=$rc"; tail -2 gpurun_out/pw3_tests.log; [ $rc -eq 0 ] || exit $rc
TESTS_FOR="" VARIANTS="ship pw3" AB_NOISE=0.01875 bash tools/gpu_ab.sh || exit $?
for rep in 1 2; do
  for v in ship pw3; do
    lib=maveric-slam_amd/libmaveric_hip.so; [ $v = ship ] || lib=build_variants/libmaveric_$v.so
    MV_LIB=$lib POSE_NOISE=1 POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=20 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pt_${v}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pose_timing $v rc=$rc"; tail -3 gpurun_out/pt_${v}_$rep.log; exit $rc; }
    echo "noisy pose $v rep $rep: $(grep '^B=' gpurun_out/pt_${v}_$rep.log | head -3 | tr '\n' ' ')"
  done
done
