#!/bin/bash
# k_q8d_match phase trace: the library rebuilt with -DMV_TRACE (+ $EXTRA), traced, then the
# default build restored.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
touch maveric-slam_amd/csrc/hip/k_allpairs_direct.hip
make -s -C maveric-slam_amd/csrc -j16 EXTRA="-DMV_TRACE ${EXTRA:-}" > gpurun_out/trace_build.log 2>&1 || exit 2
timeout -k 10 120 python tools/trace_direct.py > gpurun_out/trace_direct.log 2>&1; rc=$?
cat gpurun_out/trace_direct.log | tail -25
touch maveric-slam_amd/csrc/hip/k_allpairs_direct.hip
make -s -C maveric-slam_amd/csrc -j16 > /dev/null 2>&1
exit $rc
