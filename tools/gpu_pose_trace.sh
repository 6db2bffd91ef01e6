#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
touch maveric-slam_amd/csrc/hip/k_pose_intended.hip
make -s -C maveric-slam_amd/csrc -j16 EXTRA="-DPE_TRACE=1" > gpurun_out/pe_build.log 2>&1 || exit 2
POSE_BATCHES=1024 timeout -k 10 200 python tools/pose_timing.py > gpurun_out/pe_trace.log 2>&1; rc=$?
grep "pose phases" gpurun_out/pe_trace.log | sort | uniq -c | sort -rn | head -12
grep "hyp=256" gpurun_out/pe_trace.log
exit $rc
