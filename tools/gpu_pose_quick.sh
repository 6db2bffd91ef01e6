set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -m pytest tests/test_gpu_pose.py tests/test_gpu_kitti_e2e.py tests/test_gpu_track.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_pose.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pose.log; [ $rc -eq 0 ] || exit $rc
POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pt_clean.log 2>&1 || exit 3
POSE_NOISE=1 POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pt_noisy.log 2>&1 || exit 4
cat gpurun_out/pt_clean.log gpurun_out/pt_noisy.log | grep "B="
