#!/bin/bash
# Pose-kernel ablation on the GPU box: rebuild with each PE_* switch set in VARIANTS
# (';'-separated) and time k_pose_ransac alone (tools/pose_timing.py, untraced: the
# PE_TRACE build's printf makes the kernel 2.5x slower and skews its phase split).
# Leaves the default build behind.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
IFS=';' read -ra VS <<< "${VARIANTS:-}"
i=0
for V in "${VS[@]}"; do
  touch maveric-slam_amd/csrc/hip/k_pose_intended.hip
  make -s -C maveric-slam_amd/csrc -j16 EXTRA="$V" > gpurun_out/pa_$i.build 2>&1 || { echo "build failed: $V"; exit 2; }
  POSE_BATCHES=1024 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pa_$i.log 2>&1
  rc=$?
  echo "[$V] rc=$rc: $(grep 'hyp=256 iters=10' gpurun_out/pa_$i.log)"
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
touch maveric-slam_amd/csrc/hip/k_pose_intended.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
