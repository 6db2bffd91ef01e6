#!/bin/bash
# k_q8_match phase trace (library rebuilt with -DQ8_EXP_TRACE plus $EXTRA), then the default build back
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
touch maveric-slam_amd/csrc/hip/k_allpairs_q8.hip
make -s -C maveric-slam_amd/csrc -j16 EXTRA="-DQ8_EXP_TRACE ${EXTRA:-}" > gpurun_out/trace_build.log 2>&1 || exit 2
timeout -k 10 120 python tools/trace_q8.py > gpurun_out/trace_q8.log 2>&1; rc=$?
head -12 gpurun_out/trace_q8.log
exit $rc
